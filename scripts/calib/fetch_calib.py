#!/usr/bin/env python3
"""FETCH_SIZE calibration for gfx950: read known byte counts with 8-B and
16-B per-lane loads (fetch_calib.hip) so the counter's factor for the likelihood kernel's own load
shapes is measured, not assumed. Build here:  python scripts/calib/fetch_calib.py --build
Run under rocprofv3 on the GPU box (one --pmc pass):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o pmc -- python3 scripts/calib/fetch_calib.py
and summarise:  python scripts/calib/fetch_calib.py --summary OUT"""
import ctypes
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(os.path.dirname(os.path.dirname(HERE)), "build", "calib", "libfetch_calib.so")
SIZES_MB = (64, 256)  # bytes read per dispatch (well past every L2 and the 256 MB MALL at the top)


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           os.path.join(HERE, "fetch_calib.hip"), "-o", SO])


def run():
    import torch

    lib = ctypes.CDLL(SO)
    lib.calib_launch.restype = ctypes.c_int
    lib.calib_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    blocks = 256 * 8
    dst = torch.empty(blocks * 256, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    plan = []
    for mb in SIZES_MB:
        n = mb * 1024 * 1024 // 8
        src = torch.rand(n, dtype=torch.float64, device=dev)
        for width in (1, 2):
            for rep in range(3):
                assert lib.calib_launch(src.data_ptr(), dst.data_ptr(), n, width, blocks, ctypes.c_void_p(st.cuda_stream)) == 0
                plan.append({"bytes": n * 8, "width_bytes": 8 * width, "rep": rep})
        torch.cuda.synchronize()
        del src
    print(json.dumps(plan))


def summary(out_dir):
    import csv

    files = glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True)
    rows = [r for f in files for r in csv.DictReader(open(f)) if "calib_read" in r.get("Kernel_Name", "")]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    by_dispatch = {}
    for r in rows:
        by_dispatch.setdefault(int(r["Dispatch_Id"]), []).append(r)
    res = []
    for i, (d, rs) in enumerate(sorted(by_dispatch.items())):
        val = sum(float(r["Counter_Value"]) for r in rs)
        name = rs[0]["Kernel_Name"]
        res.append({"dispatch": d, "kernel": name.split("(")[0], "FETCH_SIZE_kb": val})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    elif "--summary" in sys.argv:
        summary(sys.argv[sys.argv.index("--summary") + 1])
    else:
        run()
