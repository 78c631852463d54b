#!/usr/bin/env python3
"""Per-call cost of the MATLAB drop-in's C side (GPU box): the MEX gateway matlab/tci_mex.cpp
executed through the stand-in MATLAB API (matlab/mexstub/), its 'ss' command on one TestData cell --
what `tci_ssfun.m`'s fast path calls once per mcmcstat ssfun call (TranscriptionCycleMCMC.m:186,258).

Timed with prebuilt argument arrays (as MATLAB passes its own), against the same loop calling
'device_count' (no GPU work: the harness's ctypes call, argument dispatch and output array) and the
Python binding's tci_ssfun. MATLAB is absent, so the .m wrapper's own interpreter cost (two
isequaln compares of the caller's arrays on the fast path) cannot be timed here."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from mexharness import Mex, MxPtr  # noqa: E402


def per_call(fn, n):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main(n=4000):
    import ctypes as C

    from transcriptioncycleinference_amd import Likelihood, testdata
    from transcriptioncycleinference_amd.build import MEX_STUB, build_library, build_mex_stub

    build_library()
    if not os.path.exists(MEX_STUB):
        build_mex_stub()
    mex = Mex(MEX_STUB)
    cells = testdata()
    t, m, p = cells.cell(0)
    data = MxPtr(mex, mex.struct([{"time": t, "MS2": m, "PP7": p, "name": "TestData"}], ["time", "MS2", "PP7", "name"]))
    h = mex.call("create", data, "P2P-MS2v5-LacZ-PP7v4", 0.0)[0]
    gw = MxPtr(mex, mex.handle(int(h[0, 0])))
    x = np.concatenate([[2.0, 1.0, 1.0, 10.0, 5.0, 0.5, 15.0], np.zeros(len(t))])
    args_ss = [mex.string("ss"), gw.p, mex.double(1.0), mex.double(x)]
    args_dc = [mex.string("device_count")]
    L = mex.L

    def call(args):
        prhs = (C.c_void_p * len(args))(*args)
        plhs = (C.c_void_p * 1)()
        rc = L.mexstub_call(1, plhs, len(args), prhs)
        if rc != 0:
            raise RuntimeError(L.mexstub_error_msg().decode())
        L.mxDestroyArray(plhs[0])

    ss_us = per_call(lambda: call(args_ss), n)
    dc_us = per_call(lambda: call(args_dc), n)
    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4", device=0) as lk:
        py_us = per_call(lambda: lk.ssfun(x, 0), n)
    for a in args_ss[:1] + args_ss[2:] + args_dc:
        L.mxDestroyArray(a)
    mex.call("destroy", gw)
    print(json.dumps({"calls": n, "gateway_ss_us_per_call": ss_us, "gateway_device_count_us_per_call": dc_us,
                      "gateway_ss_minus_harness_us": ss_us - dc_us, "python_binding_tci_ssfun_us_per_call": py_us,
                      "note": "one TestData cell (N = 120), host pointers, synchronous (H2D theta, launch, D2H SS); "
                              "gateway timed through the stand-in MATLAB API via ctypes; 'device_count' = the "
                              "harness's own per-call cost"}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4000)
