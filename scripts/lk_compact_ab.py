#!/usr/bin/env python3
"""A/B in one process: the bench launch (299 TestData cells x 256 proposals, 8 resident proposal
batches cycled) evaluated with the row list (k_compact_rows + the likelihood kernel over the listed
in-bounds rows, TCI_LK_COMPACT=1) and without it (one-wave blocks over every row, the flag read by
each wave, TCI_LK_COMPACT=0). Both contexts hold the same cells; the SS of every batch must be equal
bit for bit. Prints per-launch µs (HIP events around 40 back-to-back launches, both kernels of the
listed form included) over interleaved rounds, and the evals/s each gives.
usage: python scripts/lk_compact_ab.py [rounds]
Needs the row-list build (TCI_LK_COMPACT): the commit before "Remove the row-list likelihood form";
the shipped library ignores the switch (measured, not kept)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from transcriptioncycleinference_amd import Likelihood, testdata  # noqa: E402

rounds_n = int(sys.argv[1]) if len(sys.argv) > 1 else 15
cells = testdata()
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
lks = {}
for name, flag in (("rowlist", "1"), ("flags", "0")):
    os.environ["TCI_LK_COMPACT"] = flag
    lks[name] = Likelihood(cells, bench.CONSTRUCT, 0)
rounds = bench.ProposalRounds(cells, 256, 8, 20201028, dev)
outs = {}
for name, lk in lks.items():
    res = []
    for r in range(len(rounds.theta)):
        lk.ss_batch_device(rounds.theta[r], rounds.cid, rounds.out, rounds.active[r], stream=st)
        torch.cuda.synchronize()
        res.append(rounds.out.cpu().numpy().copy())
    outs[name] = np.stack(res)
equal = bool(np.array_equal(outs["rowlist"].view(np.uint64), outs["flags"].view(np.uint64)))
times = {k: [] for k in lks}
for name, lk in lks.items():
    bench.kernel_mode(lk, rounds, 64, st)  # warm-up
for _ in range(rounds_n):
    for name, lk in lks.items():
        _, ms, _ = bench.kernel_mode(lk, rounds, 40, st)
        times[name].append(ms * 1e3)
n_act = float(np.mean(rounds.n_active))
out = {"workload": f"TestData 299 cells x 256 proposals ({rounds.B} rows, {n_act:.0f} in bounds per launch)",
       "bitwise_equal": equal, "rounds": rounds_n, "launches_per_round": 40}
for name, ts in times.items():
    med = float(np.median(ts))
    out[name] = {"median_us": med, "min_us": float(np.min(ts)), "max_us": float(np.max(ts)),
                 "evals_per_s": n_act / (med * 1e-6)}
print(json.dumps(out, indent=1))
