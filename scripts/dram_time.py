#!/usr/bin/env python3
"""Time the GPU-resident DRAM on the 299-cell TestData (end-to-end chains, SURVEY §8(d) mode ii)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from transcriptioncycleinference_amd import Likelihood, testdata  # noqa: E402
from transcriptioncycleinference_amd.mcmc import DramOptions, fit  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
engine = sys.argv[2] if len(sys.argv) > 2 else "auto"
burn_div = int(sys.argv[3]) if len(sys.argv) > 3 else 2  # n_burn = steps / burn_div (bench.py: 20)
n_cells = int(sys.argv[4]) if len(sys.argv) > 4 else 0    # fit only the first n_cells cells (0 = all)
# TCI_MAX_CHUNK (environment): rows per draws pass + chain walk (0 = automatic: adaptint)
lk = Likelihood(testdata(), lib_path=os.environ.get("TCI_LIB"))  # TCI_LIB: an A/B build variant
t0 = time.perf_counter()
fr = fit(lk, n_steps=steps, n_burn=steps // burn_div, seed=1, opts=DramOptions(engine=engine, max_chunk=int(os.environ.get("TCI_MAX_CHUNK", "0"))),
         cells=list(range(n_cells)) if n_cells else None)
wall = time.perf_counter() - t0
print(json.dumps({"engine": engine, "n_steps": steps, "chains": len(fr.MCMCresults), "device_ms": fr.elapsed_ms, "wall_s": wall,
                  "us_per_step": fr.elapsed_ms * 1e3 / (steps - 1), "ssfun_evals": fr.n_evals,
                  "evals_per_s": fr.n_evals / (fr.elapsed_ms * 1e-3),
                  "accept_rate_median": float(np.median(fr.accept_rate))}))
