#!/usr/bin/env python3
"""Host-pointer tci_ss_batch latency against the batch size, with the zero-copy path (theta, ids,
flags and SS in one pinned device-mapped buffer, the default up to TCI_ZERO_COPY_MAX = 1 MB) and
without it (TCI_ZERO_COPY_MAX=0: hipMemcpy in and out), and with zero copy at every size. The threshold is read once per process, so
each setting runs in a child process:  python scripts/zero_copy_sweep.py  (prints one JSON line)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS = (1, 299, 1196, 2990, 8970, 29900)


def child():
    import numpy as np

    sys.path.insert(0, ROOT)
    import bench
    from transcriptioncycleinference_amd import Likelihood, testdata

    cells = testdata()
    theta, cid, active = bench.proposal_batch(cells, 100, seed=7)  # 299 x 100 rows, cell-major
    out = {}
    with Likelihood(cells, bench.CONSTRUCT, 0) as lk:
        for B in ROWS:
            th, c = theta[:B], cid[:B]
            lk.ss_batch(th, c)  # warm
            reps = max(20, min(2000, 200000 // max(B, 1)))
            t0 = time.perf_counter()
            for _ in range(reps):
                lk.ss_batch(th, c)
            dt = (time.perf_counter() - t0) / reps
            out[B] = {"us_per_call": dt * 1e6, "bytes_in": int(th.nbytes + c.nbytes), "evals_per_s": B / dt}
    print(json.dumps(out))


def main():
    res = {}
    for name, env in (("zero_copy_default", {}), ("copies", {"TCI_ZERO_COPY_MAX": "0"}),
                      ("zero_copy_always", {"TCI_ZERO_COPY_MAX": str(1 << 31)})):
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=e, capture_output=True, text=True,
                           timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:], file=sys.stderr)
            sys.exit(r.returncode)
        res[name] = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps({"rows": list(ROWS), "threshold_bytes": 1 << 20, **res}))


if __name__ == "__main__":
    child() if "--child" in sys.argv else main()
