"""Generate the committed golden fixtures from the reference's own data files.

Run in the build container (where ``/root/reference`` exists)::

    python tests/golden/make_golden.py

Inputs (read-only, MAT v5, loaded with ``scipy.io.loadmat`` -- a data loader
that executes nothing from the file):

* ``TestScripts/TestData.mat``                    -> ``testdata.npz``
  the 299-cell dataset (``data(i).time/MS2/PP7``, README.md:11-16), packed as
  ragged SoA: ``offsets[C+1]`` int64 and ``t``, ``ms2``, ``pp7`` float64.
* ``TestScripts/28-Oct-2020-TestData.mat``         -> ``forward_means.npz``
  the posterior means ``MCMCresults(c).mean_*`` assembled into theta
  ``[v,tau,ton,MS2_basal,PP7_basal,A,R,dR]`` (TranscriptionCycleMCMC.m:210)
  and the reference's OWN forward-model outputs at those means,
  ``MCMCplot(c).simMS2/simPP7`` (written at TranscriptionCycleMCMC.m:307-309).
  These are known-answer vectors produced by MATLAB itself.
* ``TestScripts/28-Oct-2020-TestData_RawChain.mat`` -> ``chain_theta.npz``
  all 2,990 raw chain rows as theta (field order re-mapped to theta order) and
  the ``s2chain`` sigma^2 draws, plus ``ss``: the SS of every row computed by
  the oracle restatement (``oracle/oracle.py``).  The reference stores no SS;
  ``ss`` is pinned by the forward-model goldens above (bit-exact) and
  statistically by ``s2chain`` (mcmcstat draws 1/s2 ~ Gamma(N/2, 2/SS),
  see tests/test_oracle_golden.py).
* both result files                                -> ``result_schema.json``
  the variable names of each file and the field names, in order, of ``MCMCresults``,
  ``MCMCplot`` and ``MCMCchain`` (TranscriptionCycleMCMC.m:149-157,373-378), so the writer
  is pinned to the reference's own files, not to a list of our own.

``python tests/golden/make_golden.py --schema`` regenerates only the schema.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import scipy.io as sio

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/TestScripts"
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402  (fixture generation is test infrastructure)


def _load(name):
    return sio.loadmat(os.path.join(REF, name), squeeze_me=True, struct_as_record=False)


def schema():
    import json

    out = {}
    for fname, tag in (("28-Oct-2020-TestData.mat", "results_file"), ("28-Oct-2020-TestData_RawChain.mat",
                                                                        "rawchain_file")):
        d = _load(fname)
        out[tag] = {"variables": sorted(k for k in d if not k.startswith("__"))}
        for k, v in d.items():
            if k.startswith("__") or not hasattr(np.atleast_1d(v)[0], "_fieldnames"):
                continue
            out[tag][k] = list(np.atleast_1d(v)[0]._fieldnames)
    res = _load("28-Oct-2020-TestData.mat")["MCMCresults"]
    out["results_file"]["ApprovedFits_values"] = sorted({int(r.ApprovedFits) for r in res})
    ci = [int(r.cell_index) for r in res]
    out["results_file"]["n_entries"] = len(ci)
    out["results_file"]["cell_index_is_1_to_n"] = ci == list(range(1, len(ci) + 1))
    with open(os.path.join(HERE, "result_schema.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


def main():
    data = _load("TestData.mat")["data"]
    C = len(data)
    lens = np.array([len(np.atleast_1d(c.time)) for c in data], dtype=np.int64)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    t = np.concatenate([np.asarray(c.time, np.float64) for c in data])
    ms2 = np.concatenate([np.asarray(c.MS2, np.float64) for c in data])
    pp7 = np.concatenate([np.asarray(c.PP7, np.float64) for c in data])
    np.savez_compressed(os.path.join(HERE, "testdata.npz"), offsets=offsets, t=t, ms2=ms2, pp7=pp7,
                        name=np.array(str(data[0].name)))

    res = _load("28-Oct-2020-TestData.mat")
    thetas, sim_ms2, sim_pp7, cell_index = [], [], [], []
    for c in range(C):
        m = res["MCMCresults"][c]
        p = res["MCMCplot"][c]
        th = np.concatenate([[m.mean_v, m.mean_tau, m.mean_ton, m.mean_MS2_basal, m.mean_PP7_basal,
                              m.mean_A, m.mean_R], np.asarray(m.mean_dR, np.float64)])
        assert len(th) == 7 + lens[c]
        assert np.array_equal(np.asarray(p.t_plot, np.float64), t[offsets[c]:offsets[c + 1]])
        thetas.append(th)
        sim_ms2.append(np.asarray(p.simMS2, np.float64))
        sim_pp7.append(np.asarray(p.simPP7, np.float64))
        cell_index.append(int(m.cell_index) - 1)
    th_off = np.concatenate([[0], np.cumsum([len(x) for x in thetas])]).astype(np.int64)
    np.savez_compressed(os.path.join(HERE, "forward_means.npz"), theta=np.concatenate(thetas),
                        theta_offsets=th_off, sim_ms2=np.concatenate(sim_ms2),
                        sim_pp7=np.concatenate(sim_pp7), cell_index=np.array(cell_index, np.int32))

    chain = _load("28-Oct-2020-TestData_RawChain.mat")["MCMCchain"]
    construct = O.builtin_construct("P2P-MS2v5-LacZ-PP7v4")
    rows, cell_id, step, s2, ss = [], [], [], [], []
    for c in range(C):
        q = chain[c]
        nrow = len(np.atleast_1d(q.v_chain))
        dat = {"xdata": t[offsets[c]:offsets[c + 1]],
               "ydata": np.concatenate([ms2[offsets[c]:offsets[c + 1]], pp7[offsets[c]:offsets[c + 1]]])}
        dRc = np.atleast_2d(np.asarray(q.dR_chain, np.float64))
        for k in range(nrow):
            th = np.concatenate([[q.v_chain[k], q.tau_chain[k], q.ton_chain[k], q.MS2_basal_chain[k],
                                  q.PP7_basal_chain[k], q.A_chain[k], q.R_chain[k]], dRc[k]])
            rows.append(th)
            cell_id.append(c)
            step.append(k)
            s2.append(float(q.s2chain[k]))
            ss.append(O.sum_of_squares(construct, dat, th))
    r_off = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.int64)
    np.savez_compressed(os.path.join(HERE, "chain_theta.npz"), theta=np.concatenate(rows),
                        theta_offsets=r_off, cell_id=np.array(cell_id, np.int32),
                        step=np.array(step, np.int32), s2=np.array(s2), ss=np.array(ss))
    for f in ("testdata.npz", "forward_means.npz", "chain_theta.npz"):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    if "--schema" not in sys.argv:
        main()
    schema()
