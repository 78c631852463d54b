#!/usr/bin/env python3
"""A/B timing of kernel build variants, interleaved in ONE process (cdna_hip_programming.md
§5.4 rule 24). Build here:  python scripts/ab_variants.py --build
Run on the GPU box:         python scripts/ab_variants.py --run [--rounds 9 --launches 20]
Every variant is also checked against the first one: bit for bit (`bitwise_equal_to_first`,
`rows_differing_in_bits`) and, separately, to 1e-12 relative (`rel_vs_first`)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "ab")

# Diagnostics builds (measurement only; the ablations give wrong results on purpose). Any other
# variant is given ad hoc as NAME=DEF1+DEF2 (e.g. "x=TCI_FOO=1+TCI_BAR=2") for a one-off A/B;
# rejected experiments are not kept as knobs in the sources (git history has them).
VARIANTS = {
    "ship": [],
    "old": None,   # a prebuilt library of the previous commit, copied to build/ab/libtci_old.so
    "prev": None,  # a prebuilt library of the previous working state
    "abl_rows": ["TCI_ABLATE=1"],
    "abl_interp": ["TCI_ABLATE=4"],
    "abl_scan": ["TCI_ABLATE=8"],
    "abl_all": ["TCI_ABLATE=15"],
    "abl_loads": ["TCI_ABLATE=16"],
    "abl_launch": ["TCI_ABLATE=32"],
    "chainprof": ["TCI_CHAIN_PROFILE=1"],
    "chainprof2": ["TCI_CHAIN_PROFILE=2"],
    "adaptprof": ["TCI_ADAPT_PROFILE=1"],
    "adapt_nochol": ["TCI_ADAPT_ABLATE=1"],
    "adapt_nocov": ["TCI_ADAPT_ABLATE=2"],
    "draws_nonorm": ["TCI_DRAWS_ABLATE=1"],
    "draws_nomfma": ["TCI_DRAWS_ABLATE=2"],
    "draws_noscal": ["TCI_DRAWS_ABLATE=4"],
    "draws_noR": ["TCI_DRAWS_ABLATE=8"],
}


def parse_variant(spec):
    """'name' (a table entry) or 'name=DEF1+DEF2' (ad hoc) -> name; registers ad hoc defines."""
    if "=" in spec:
        name, defs = spec.split("=", 1)
        VARIANTS[name] = defs.split("+")
        return name
    return spec


def build(names, jobs=4):
    from concurrent.futures import ThreadPoolExecutor

    from transcriptioncycleinference_amd.build import build_library

    os.makedirs(OUT, exist_ok=True)
    todo = [n for n in names if VARIANTS.get(n) is not None]
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda n: build_library(out=os.path.join(OUT, f"libtci_{n}.so"), defines=VARIANTS[n]), todo))


def run(names, rounds, launches, proposals, distinct=1):
    import torch

    import bench
    from transcriptioncycleinference_amd import Likelihood, testdata

    cells = testdata()
    theta, cid, active = bench.proposal_batch(cells, proposals, seed=20201028)
    dev = torch.device("cuda", 0)
    th_d = torch.from_numpy(theta).to(dev)
    # bench-like: launches cycle through `distinct` resident batches (batch 0 is the checked one)
    th_all = [th_d] + [torch.from_numpy(bench.proposal_batch(cells, proposals, seed=20201028 + i)[0]).to(dev)
                       for i in range(1, distinct)]
    cid_d = torch.from_numpy(cid).to(dev)
    act_d = torch.from_numpy(active).to(dev)
    # "main": the in-tree libtci.so (the shipped build)
    lks = {n: Likelihood(cells, bench.CONSTRUCT, 0, lib_path=None if n == "main" else os.path.join(OUT, f"libtci_{n}.so"))
           for n in names}
    outs = {n: torch.empty(len(cid), dtype=torch.float64, device=dev) for n in names}
    st = torch.cuda.current_stream(dev)
    for n in names:  # warm + correctness
        lks[n].ss_batch_device(th_d, cid_d, outs[n], act_d, stream=st)
    torch.cuda.synchronize()
    times = {n: [] for n in names}
    for _ in range(rounds):
        for n in names:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(launches):
                lks[n].ss_batch_device(th_all[i % distinct], cid_d, outs[n], act_d, stream=st)
            e1.record(st)
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / launches * 1e3)
    ref = outs[names[0]].cpu().numpy()  # every variant's last launch read the same batch
    act = active.astype(bool)
    res = {}
    for n in names:
        got = outs[n].cpu().numpy()
        rr = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
        rr[~act] = 0
        rel = float(np.nanmax(rr))
        # bit-for-bit agreement (NaN == NaN) reported apart from the 1e-12 relative check
        same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
        bits_equal = bool(np.all(same))
        n_diff_bits = int((~same).sum())
        bad = np.nonzero(~(rr <= 1e-12))[0]
        if len(bad):
            print(n, "mismatching rows", len(bad), "first", [(int(i), int(cid[i]), float(ref[i]), float(got[i])) for i in bad[:8]], file=sys.stderr)
        t = np.array(times[n])
        res[n] = {"median_us": float(np.median(t)), "min_us": float(t.min()), "rel_vs_first": rel,
                  "bitwise_equal_to_first": bits_equal, "rows_differing_in_bits": n_diff_bits,
                  "evals_per_s": float(act.sum() / (np.median(t) * 1e-6)), "defines": VARIANTS.get(n)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--variants", default="ship,abl_rows,abl_interp,abl_scan,abl_all")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--proposals", type=int, default=256)
    ap.add_argument("--distinct", type=int, default=1, help="resident batches cycled (bench.py: 8)")
    a = ap.parse_args()
    names = [parse_variant(v) for v in a.variants.split(",")]
    if a.build:
        build(names)
    if a.run:
        run(names, a.rounds, a.launches, a.proposals, a.distinct)
