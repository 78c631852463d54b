"""Waits in front of every s_barrier of the kernels of an asm file (hipcc -S): which barriers
wait for vector memory (vmcnt) as well as LDS (lgkmcnt).

python scripts/asm_barriers.py file.s name-filter..."""
import re
import sys

s = open(sys.argv[1]).read()
filt = sys.argv[2:]
for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\n\.Lfunc_end", s, re.S):
    name, body = m.group(1), m.group(2)
    if filt and not any(f in name for f in filt):
        continue
    lines = body.split("\n")
    print(name)
    for i, l in enumerate(lines):
        if "s_barrier" in l:
            w = [x.strip() for x in lines[max(0, i - 6):i] if "s_waitcnt" in x]
            print(f"  line {i:5d}: {w}")
