#!/usr/bin/env python3
"""A/B in one process: the fused engine's draws split in two (k_draws_rng on a second stream one
chunk ahead + k_draws multiplying by R: TCI_DRAWS_SPLIT=1, the default) against one draws launch
per chunk (TCI_DRAWS_SPLIT=0), on the 299-cell TestData fit of bench.py's end-to-end leg (n_burn =
n_steps / 20, adaptint 100). Interleaved rounds; per variant the device time of the step loop, the
wall time, the per-class kernel time (HIP events, a separate run with kernel_times: the events
themselves serialise nothing but add their own gaps), and whether every output equals the other
variant's bit for bit. TCI_RNG_WGS values may be swept: variants "split:<wgs>".
usage: python scripts/dram_split_ab.py [n_steps] [rounds] [variants, e.g. one,split,split:64]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from transcriptioncycleinference_amd import Likelihood, testdata  # noqa: E402
from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run, plan_fit  # noqa: E402

n_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
variants = (sys.argv[3] if len(sys.argv) > 3 else "one,split").split(",")
lk = Likelihood(testdata(), lib_path=os.environ.get("TCI_LIB"))  # TCI_LIB: an A/B build variant
cl = lk.cells
plan = plan_fit(cl, list(range(cl.n_cells)), 1)
cells = np.array(plan.cells, np.int32)
n_burn = max(1, n_steps // 20)


def setenv(v):
    os.environ["TCI_DRAWS_SPLIT"] = "0" if v == "one" else "1"
    if v.startswith("split:"):
        os.environ["TCI_RNG_WGS"] = v.split(":")[1]
    else:
        os.environ.pop("TCI_RNG_WGS", None)


def run(v, kt=False, steps=n_steps):
    setenv(v)
    o = DramOptions(n_steps=steps, burnintime=n_burn, adaptint=100, stats_from=n_burn, seed=7, kernel_times=kt)
    t0 = time.perf_counter()
    r = dram_run(lk, cells, plan.x0, plan.lower, plan.upper, plan.prior_mu, plan.prior_sig, plan.qcov_diag, 1.0, o,
                 chain_keys=cells.astype(np.int64))
    return r, time.perf_counter() - t0


def bits(r):
    return [np.ascontiguousarray(a).view(np.uint8) for a in (r.mean, r.std, r.final_theta, r.sigma_mean,
                                                               r.sigma_std, r.accept_rate, r.n_evals)]


run(variants[0], steps=2000)  # warm-up (code objects, allocations)
res = {v: {"device_ms": [], "wall_s": []} for v in variants}
first = {}
for _ in range(rounds):
    for v in variants:
        r, wall = run(v)
        res[v]["device_ms"].append(float(r.elapsed_ms))
        res[v]["wall_s"].append(wall)
        first.setdefault(v, bits(r))
ref = first[variants[0]]
out = {"workload": f"TestData {len(cells)} chains, {n_steps} steps, n_burn {n_burn}, adaptint 100", "rounds": rounds}
for v in variants:
    r, _ = run(v, kt=True, steps=min(n_steps, 2000))
    d = res[v]
    med = float(np.median(d["device_ms"]))
    out[v] = {"device_ms_median": med, "device_ms": d["device_ms"], "wall_s_median": float(np.median(d["wall_s"])),
              "us_per_step_device": med * 1e3 / (n_steps - 1),
              "us_per_step_wall": float(np.median(d["wall_s"])) * 1e6 / (n_steps - 1),
              "bitwise_equal_to_first": all(np.array_equal(a, b) for a, b in zip(first[v], ref)),
              "kernel_us_per_launch_2000_steps": {k: (float(r.kernel_ms[i]) * 1e3 / max(int(r.kernel_launches[i]), 1))
                                                  for i, k in enumerate(("draws", "walk", "adapt", "draws_rng"))},
              "kernel_launches": [int(x) for x in r.kernel_launches]}
print(json.dumps(out, indent=1))
