#!/usr/bin/env python3
"""Bitwise comparison of two library builds on the same DRAM fit (A/B of a change that must not
move any bit): python scripts/dram_lib_equal.py LIB_A LIB_B [STEPS] [CELLS] [CFG]
("main" = the in-tree build; "LIB@NAME=VALUE" also sets the environment variable NAME for that
run, e.g. main@TCI_DRAM_OVERLAP=0 against main). CFG 0: TestData cells; 4/5: BASELINE config-4/5 synthetic cells
(TCI_SYNTH_POINTS points per cell, default 200)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from transcriptioncycleinference_amd import Likelihood, testdata  # noqa: E402
from transcriptioncycleinference_amd.mcmc import DramOptions, fit  # noqa: E402


def run(lib, steps, n, cfg):
    lib, _, env = lib.partition("@")
    if env:
        k, _, v = env.partition("=")
        os.environ[k] = v
    path = None if lib == "main" else lib
    if cfg == 0:
        cells, con = testdata(), "P2P-MS2v5-LacZ-PP7v4"
    else:
        import bench
        cells, _, con = bench.synthetic_config_cells(cfg, 0, 1, 0, int(os.environ.get("TCI_SYNTH_POINTS", "200")))[:3]
    engine = os.environ.get("TCI_ENGINE", "auto")
    with Likelihood(cells, con, lib_path=path) as lk:
        fr = fit(lk, n_steps=steps, n_burn=steps // 4, seed=3, cells=list(range(n)), opts=DramOptions(engine=engine))
    if env:
        os.environ.pop(k)
    # every output: the scalar summaries, mean/sigma of dR, the final states, acceptance, evaluations
    rows = []
    for k, r in enumerate(fr.MCMCresults):
        sc = [r[f] for f in sorted(r) if np.isscalar(r[f]) and isinstance(r[f], float)]
        rows.append(np.concatenate([sc, r["mean_dR"], r["sigma_dR"], fr.final_theta[k], [fr.accept_rate[k]]]))
    return np.concatenate(rows + [np.atleast_1d(np.asarray(fr.n_evals, np.float64)).ravel()])  # ragged rows: flat


a, b = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
n = int(sys.argv[4]) if len(sys.argv) > 4 else 40
cfg = int(sys.argv[5]) if len(sys.argv) > 5 else 0
ra, rb = run(a, steps, n, cfg), run(b, steps, n, cfg)
same = ra.shape == rb.shape and bool(np.array_equal(ra, rb, equal_nan=True))
print(json.dumps({"a": a, "b": b, "steps": steps, "cells": n, "cfg": cfg, "bitwise_equal": same,
                  "max_abs_diff": float(np.nanmax(np.abs(ra - rb))) if ra.shape == rb.shape else None}))
sys.exit(0 if same else 1)
