#!/usr/bin/env python3
"""Where the wall time of bench.py's end-to-end fit goes beyond the device time of the step loop:
plan_fit (host), dram_run (its wall vs the step loop's HIP-event time: setup, copies, results),
the forward model at the means, and the result assembly. TestData, 299 chains.
usage: python scripts/fit_overhead.py [n_steps] [repeats]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from transcriptioncycleinference_amd import Likelihood, testdata  # noqa: E402
from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run, fit, plan_fit  # noqa: E402

n_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
lk = Likelihood(testdata())
cl = lk.cells
ids = list(range(cl.n_cells))
fit(lk, n_steps=2000, n_burn=100, seed=1)  # warm-up
out = []
for _ in range(reps):
    t0 = time.perf_counter()
    plan = plan_fit(cl, ids, 1)
    t1 = time.perf_counter()
    keep = np.array(plan.cells, np.int32)
    nb = max(1, n_steps // 20)
    o = DramOptions(n_steps=n_steps, burnintime=nb, stats_from=nb, seed=1 * 1000003 + 20201028)
    r = dram_run(lk, keep, plan.x0, plan.lower, plan.upper, plan.prior_mu, plan.prior_sig, plan.qcov_diag, 1.0, o,
                 chain_keys=keep.astype(np.int64))
    t2 = time.perf_counter()
    lk.forward(r.mean, keep, grid="raw")
    t3 = time.perf_counter()
    tf0 = time.perf_counter()
    fr = fit(lk, n_steps=n_steps, n_burn=nb, seed=1)
    tf1 = time.perf_counter()
    out.append({"plan_ms": (t1 - t0) * 1e3, "dram_run_wall_ms": (t2 - t1) * 1e3, "step_loop_device_ms": r.elapsed_ms,
                "dram_run_outside_loop_ms": (t2 - t1) * 1e3 - r.elapsed_ms, "forward_ms": (t3 - t2) * 1e3,
                "fit_wall_ms": (tf1 - tf0) * 1e3, "fit_device_ms": fr.elapsed_ms,
                "fit_outside_loop_ms": (tf1 - tf0) * 1e3 - fr.elapsed_ms})
print(json.dumps({"n_steps": n_steps, "runs": out}, indent=1))
