#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (scripts/gpu_pmc.sh) for the likelihood kernel.

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes, following
MI355X_MICROARCH.md's HBM/rocprofv3 section: FETCH_SIZE (KB) reads 1/2 of the bytes of a wide
coalesced read on gfx950; WRITE_SIZE is exact for streaming stores. The x2 read correction is
measured for this kernel's own load shapes: scripts/calib/fetch_calib.py reads 64 and 256 MB once
with 8-B and with 16-B per-lane loads, and FETCH_SIZE is half the bytes read in every case
(profiles/r03_calib/fetch_size_calibration.json).
Usage: python scripts/pmc_summary.py gpurun_out/<tag> <workload> > profiles/pmc_traffic.json
"""
import collections
import csv
import glob
import json
import sys


def main(prefix, workload):
    agg = collections.defaultdict(list)
    for p in range(1, 8):
        files = glob.glob(f"{prefix}_p{p}/**/*counter_collection.csv", recursive=True)
        rows = [r for f in files for r in csv.DictReader(open(f))]
        for r in rows:
            if "tci_cohort_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in agg.items()}
    fetch, write = mean.get("FETCH_SIZE"), mean.get("WRITE_SIZE")
    out = {
        "workload": workload,
        "source": prefix,
        "hbm_bytes_per_launch": None if fetch is None or write is None else (2 * fetch + write) * 1024,
        "fetch_size_kb_raw": fetch,
        "write_size_kb": write,
        "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts exactly 1/2 of the bytes read "
                      "with 8-B and 16-B per-lane loads: profiles/r03_calib/fetch_size_calibration.json)",
        "counters_mean_per_launch": mean,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
