"""Per-kernel register / spill / LDS table of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

python scripts/resource_usage.py [source.hip] [name-filter] [-DNAME=VAL ...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = [a for a in sys.argv[1:] if not a.startswith("-D")]
defs = [a for a in sys.argv[1:] if a.startswith("-D")]
src = args[0] if args and args[0] else f"{ROOT}/transcriptioncycleinference_amd/csrc/tci_dram.hip"
filt = args[1] if len(args) > 1 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-mllvm",
       "-amdgpu-mfma-vgpr-form", "-fPIC", f"-I{ROOT}/include", f"-I{ROOT}/transcriptioncycleinference_amd/csrc",
       "--cuda-device-only", "-c", src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage", *defs]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        demangled = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        short = re.sub(r"\(.*", "", demangled.replace("tci::(anonymous namespace)::", "")).replace("void ", "")
        cur = {"name": short}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
print(f"{'kernel':44s} {'VGPR':>5s} {'SGPR':>5s} {'Vspill':>6s} {'Sspill':>6s} {'LDS':>6s} {'occ':>4s}")
for r in rows:
    if filt in r["name"]:
        print(f"{r['name'][:44]:44s} {r.get('VGPRs','?'):>5s} {r.get('TotalSGPRs','?'):>5s} {r.get('VGPRs Spill','?'):>6s} "
              f"{r.get('SGPRs Spill','?'):>6s} {r.get('LDS Size [bytes/block]','?'):>6s} {r.get('Occupancy [waves/SIMD]','?'):>4s}")
