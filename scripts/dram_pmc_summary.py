#!/usr/bin/env python3
"""Per-dispatch means of the PMC passes of scripts/gpu_dram_pmc.sh for the DRAM kernels.
usage: python scripts/dram_pmc_summary.py gpurun_out/<tag>"""
import collections
import csv
import glob
import json
import sys

KERNELS = ("k_chain", "k_draws", "k_adapt_mfma", "k_walk", "k_adapt_gt")


def main(prefix):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{prefix}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values()), "mean_per_dispatch": m}
        if m.get("SQ_WAVE_CYCLES"):
            wc = m["SQ_WAVE_CYCLES"]
            d["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / wc
            d["wait_inst_any_frac"] = m.get("SQ_WAIT_INST_ANY", 0) / wc
            d["active_valu_frac"] = m.get("SQ_ACTIVE_INST_VALU", 0) / wc
            d["active_lds_frac"] = m.get("SQ_ACTIVE_INST_LDS", 0) / wc
        if m.get("SQ_WAVES"):
            d["valu_per_wave"] = m.get("SQ_INSTS_VALU", 0) / m["SQ_WAVES"]
            d["mfma_f64_per_wave"] = m.get("SQ_INSTS_VALU_MFMA_F64", 0) / m["SQ_WAVES"]
        out[k] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
