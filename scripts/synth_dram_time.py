#!/usr/bin/env python3
"""Time the GPU-resident DRAM fit of BASELINE configs 4/5 (10,000 synthetic cells x 200 points) on
one GPU:  python scripts/synth_dram_time.py CFG STEPS [CFG STEPS ...]   (TCI_ENGINE=auto|fused|batched|walk, TCI_LIB=variant .so,
TCI_SYNTH_POINTS=points per cell, default 200)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if os.environ.get("TCI_LIB"):  # an A/B build variant (scripts/ab_variants.py) for every Likelihood
    from transcriptioncycleinference_amd import _lib, likelihood

    _load = _lib.load
    likelihood._lib.load = lambda path=None: _load(path or os.environ["TCI_LIB"])

args = sys.argv[1:]
for i in range(0, len(args), 2):
    cfg, steps = int(args[i]), int(args[i + 1])
    out, _ = bench.synthetic_end_to_end(cfg, 0, 1, 0, steps, reduce=lambda x, op: x,
                                        engine=os.environ.get("TCI_ENGINE", "auto"),
                                        n_points=int(os.environ.get("TCI_SYNTH_POINTS", "200")))
    print(json.dumps(out), flush=True)
