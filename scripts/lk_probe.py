#!/usr/bin/env python3
"""Price the bench launch's parts (likelihood kernel, 299 cells x 256 proposals): the shipped batch,
the same batch with every row inactive (wave launch + flag read only), with every row active (the
bounds-rejected proposals evaluated too), the in-bounds rows alone, compacted (B = 55k rows), and the
same rows with the rejected ones all after (or all before) the in-bounds ones."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from transcriptioncycleinference_amd import Likelihood, testdata  # noqa: E402

cells = testdata()
theta, cid, active = bench.proposal_batch(cells, 256, seed=20201028)
dev = torch.device("cuda", 0)
lk = Likelihood(cells, bench.CONSTRUCT, 0)
st = torch.cuda.current_stream(dev)
act = active.astype(bool)
cases = {"bench": (theta, cid, active), "all_inactive": (theta, cid, np.zeros_like(active)),
         "all_active": (theta, cid, np.ones_like(active)),
         "compacted": (np.ascontiguousarray(theta[act]), np.ascontiguousarray(cid[act]), np.ones(act.sum(), np.uint8))}
# the same rows reordered: the in-bounds rows first (their order kept), the rejected rows after them
order = np.concatenate([np.flatnonzero(act), np.flatnonzero(~act)])
cases["active_first"] = (np.ascontiguousarray(theta[order]), np.ascontiguousarray(cid[order]),
                         np.ascontiguousarray(active[order]))
order2 = np.concatenate([np.flatnonzero(~act), np.flatnonzero(act)])
cases["inactive_first"] = (np.ascontiguousarray(theta[order2]), np.ascontiguousarray(cid[order2]),
                           np.ascontiguousarray(active[order2]))
res = {}
for name, (th, ci, ac) in cases.items():
    th_d, ci_d, ac_d = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (th, ci, ac))
    out = torch.empty(len(ci), dtype=torch.float64, device=dev)
    for _ in range(10):
        lk.ss_batch_device(th_d, ci_d, out, ac_d, stream=st)
    torch.cuda.synchronize()
    ts = []
    for _ in range(15):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(40):
            lk.ss_batch_device(th_d, ci_d, out, ac_d, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 40 * 1e3)
    res[name] = {"rows": len(ci), "active": int(ac.sum()), "median_us": float(np.median(ts))}
# the bench batch as two halves launched on two streams (two hardware queues: is the workgroup
# dispatch of the one-wave blocks a limit?)
th_d, ci_d, ac_d = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (theta, cid, active))
out = torch.empty(len(cid), dtype=torch.float64, device=dev)
h = len(cid) // 2
s2 = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]


def two():
    ev = torch.cuda.Event()
    ev.record(st)
    for k, (a, b) in enumerate(((0, h), (h, len(cid)))):
        s2[k].wait_event(ev)
        lk.ss_batch_device(th_d[a:b], ci_d[a:b], out[a:b], ac_d[a:b], stream=s2[k])
    for k in range(2):
        e = torch.cuda.Event()
        e.record(s2[k])
        st.wait_event(e)


for _ in range(10):
    two()
torch.cuda.synchronize()
ts = []
for _ in range(15):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(40):
        two()
    e1.record(st)
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 40 * 1e3)
res["bench_two_streams"] = {"rows": len(cid), "active": int(active.sum()), "median_us": float(np.median(ts))}
print(json.dumps(res, indent=1))
