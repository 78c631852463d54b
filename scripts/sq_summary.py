#!/usr/bin/env python3
"""Per-wave means of the SQ counters collected by rocprofv3 --pmc SQ_ passes, per library variant
(dispatches alternate between variants in ab_variants.py order)."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
out = {}
for d in sorted(glob.glob(f"{root}/sq_*")):
    for f in glob.glob(f"{d}/**/pmc_counter_collection.csv", recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "tci_cohort_kernel" not in r["Kernel_Name"]:
                continue
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for disp, cnt in sorted(per.items()):
            for k, v in cnt.items():
                out.setdefault(k, []).append(v)
print(json.dumps({k: {"mean": sum(v) / len(v), "n": len(v)} for k, v in sorted(out.items())}, indent=1))
