"""ctypes binding of the C oracle ``oracle/libtci_oracle.so`` (built by ``oracle/Makefile``).

TEST INFRASTRUCTURE ONLY -- importable from ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg; never from the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libtci_oracle.so")

_dp = C.POINTER(C.c_double)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)


class _Construct(C.Structure):
    _fields_ = [("L0", C.c_double), ("n_seg", C.c_int32),
                ("ms2_start", _dp), ("ms2_end", _dp), ("ms2_loopn", _dp),
                ("pp7_start", _dp), ("pp7_end", _dp), ("pp7_loopn", _dp)]


def build() -> str:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_ss_batch.argtypes = [_i64p, _dp, _dp, _dp, C.c_int64, C.POINTER(_Construct), _dp, C.c_int64,
                                      _i32p, _u8p, C.c_int64, _dp, _i32p, C.c_int]
        L.oracle_ss_batch.restype = C.c_int
        L.oracle_forward.argtypes = [_dp, C.c_int64, C.POINTER(_Construct), _dp, C.c_int, _dp, _dp]
        L.oracle_forward.restype = C.c_int
        L.oracle_interp_grid.argtypes = [_dp, C.c_int64, _dp, C.c_int64]
        L.oracle_interp_grid.restype = C.c_int64
        L.oracle_max_threads.restype = C.c_int
        _lib = L
    return _lib


def _ptr(a, typ):
    return a.ctypes.data_as(typ) if a is not None else None


class _ConstructHolder:
    def __init__(self, cs):
        self.arrs = [np.ascontiguousarray(np.asarray(x, np.float64)) for x in
                     (cs.ms2_start, cs.ms2_end, cs.ms2_loopn, cs.pp7_start, cs.pp7_end, cs.pp7_loopn)]
        self.s = _Construct(float(cs.L0), len(self.arrs[0]), *[_ptr(a, _dp) for a in self.arrs])


def ss_batch(offsets, t, ms2, pp7, construct, theta, cell_id, active=None, nthreads=0):
    """Batched SS (OpenMP over rows). theta: (B, ld) float64 row-major."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    t = np.ascontiguousarray(t, np.float64)
    ms2 = np.ascontiguousarray(ms2, np.float64)
    pp7 = np.ascontiguousarray(pp7, np.float64)
    theta = np.ascontiguousarray(theta, np.float64)
    cell_id = np.ascontiguousarray(cell_id, np.int32)
    B, ld = theta.shape
    act = None if active is None else np.ascontiguousarray(active, np.uint8)
    out = np.empty(B)
    st = np.empty(B, np.int32)
    h = _ConstructHolder(construct)
    lib().oracle_ss_batch(_ptr(offsets, _i64p), _ptr(t, _dp), _ptr(ms2, _dp), _ptr(pp7, _dp),
                          len(offsets) - 1, C.byref(h.s), _ptr(theta, _dp), ld, _ptr(cell_id, _i32p),
                          _ptr(act, _u8p), B, _ptr(out, _dp), _ptr(st, _i32p), int(nthreads))
    return out, st


def forward(t, construct, theta, mode=0):
    """mode 0: raw times (TranscriptionCycleMCMC.m:307-309); mode 1: grid + interp1."""
    t = np.ascontiguousarray(t, np.float64)
    theta = np.ascontiguousarray(theta, np.float64)
    N = len(t)
    a = np.empty(N)
    b = np.empty(N)
    h = _ConstructHolder(construct)
    rc = lib().oracle_forward(_ptr(t, _dp), N, C.byref(h.s), _ptr(theta, _dp), int(mode), _ptr(a, _dp), _ptr(b, _dp))
    if rc != 0:
        raise RuntimeError(f"oracle_forward failed: {rc}")
    return a, b


def interp_grid(t):
    t = np.ascontiguousarray(t, np.float64)
    out = np.empty(len(t) + 8)
    M = lib().oracle_interp_grid(_ptr(t, _dp), len(t), _ptr(out, _dp), len(out))
    if M < 0:
        raise RuntimeError("grid failed")
    return out[:M]


def max_threads() -> int:
    return int(lib().oracle_max_threads())


# ---- the DRAM sampler restatement (oracle/tci_dram_oracle.c) -------------------------------------


class _DramOpts(C.Structure):
    _fields_ = [("n_steps", C.c_int64), ("burnintime", C.c_int64), ("adaptint", C.c_int64), ("ntry", C.c_int32),
                ("updatesigma", C.c_int32), ("drscale", C.c_double), ("adascale", C.c_double),
                ("qcovadj", C.c_double), ("burnin_scale", C.c_double), ("stats_from", C.c_int64),
                ("seed", C.c_uint64)]


class _DramOut(C.Structure):
    _fields_ = [("mean", _dp), ("std", _dp), ("final_theta", _dp), ("sigma_mean", _dp), ("sigma_std", _dp),
                ("accept_rate", _dp), ("n_evals", _i64p), ("chain", _dp), ("s2chain", _dp), ("R", _dp)]


class _U32x4(C.Structure):
    _fields_ = [("x", C.c_uint32), ("y", C.c_uint32), ("z", C.c_uint32), ("w", C.c_uint32)]


def philox(ctr, key):
    """Philox4x32-10 of the DRAM restatement (the GPU sampler's generator): 4 counter words, 2 key
    words -> 4 output words (for the generator's published known-answer vectors)."""
    L = lib()
    L.oracle_philox.argtypes = [_U32x4, C.c_uint32, C.c_uint32]
    L.oracle_philox.restype = _U32x4
    r = L.oracle_philox(_U32x4(*[int(v) & 0xFFFFFFFF for v in ctr]), int(key[0]) & 0xFFFFFFFF,
                        int(key[1]) & 0xFFFFFFFF)
    return (r.x, r.y, r.z, r.w)


def box_muller_pair(u1, u2):
    """The restatement's (and the GPU's) Box-Muller transcendental pair, elementwise:
    (-2 log u1, sin(2 pi u2), cos(2 pi u2)) in plain correctly-rounded FP64 arithmetic."""
    L = lib()
    L.bm_neg2log.argtypes = [C.c_double]
    L.bm_neg2log.restype = C.c_double
    L.bm_sincospi.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.bm_sincospi.restype = None
    u1 = np.asarray(u1, np.float64).ravel()
    u2 = np.asarray(u2, np.float64).ravel()
    lg = np.array([L.bm_neg2log(float(v)) for v in u1])
    sn, cs = np.empty(len(u2)), np.empty(len(u2))
    a, b = C.c_double(), C.c_double()
    for i, v in enumerate(u2):
        L.bm_sincospi(2.0 * float(v), C.byref(a), C.byref(b))
        sn[i], cs[i] = a.value, b.value
    return lg, sn, cs


def dram_run(cells, construct, cell_id, theta0, lower, upper, prior_mu, prior_sig, qcov_diag, sigma2_0, opts,
             keys=None, want_chain=False, want_R=False, nthreads=0):
    """mcmcrun's DRAM restated on the CPU (oracle/tci_dram_oracle.c), one chain per row, with the C
    oracle as ssfun. ``opts``: a ``transcriptioncycleinference_amd.mcmc.DramOptions`` (the fields of
    tci_dram_options); arrays as ``mcmc.dram_run``. Returns a dict of the outputs."""
    f = lambda a: np.ascontiguousarray(a, np.float64)  # noqa: E731
    theta0, lower, upper, prior_mu, prior_sig, qcov_diag = map(f, (theta0, lower, upper, prior_mu, prior_sig,
                                                                    qcov_diag))
    n, ld = theta0.shape
    cid = np.ascontiguousarray(cell_id, np.int32)
    s20 = f(np.broadcast_to(np.asarray(sigma2_0, np.float64), (n,)))
    k = None if keys is None else np.ascontiguousarray(keys, np.int64)
    o = _DramOpts(int(opts.n_steps), int(opts.burnintime), int(opts.adaptint), int(opts.ntry), int(bool(opts.updatesigma)),
                  float(opts.drscale), float(opts.adascale), float(opts.qcovadj), float(opts.burnin_scale),
                  int(max(opts.stats_from, 1)), int(opts.seed) & 0xFFFFFFFFFFFFFFFF)
    res = {"mean": np.zeros((n, ld)), "std": np.zeros((n, ld)), "final_theta": np.zeros((n, ld)),
           "sigma_mean": np.zeros(n), "sigma_std": np.zeros(n), "accept_rate": np.zeros(n),
           "n_evals": np.zeros(n, np.int64),
           "chain": np.zeros((int(opts.n_steps), n, ld)) if want_chain else None,
           "s2chain": np.zeros((int(opts.n_steps), n)) if want_chain else None,
           "R": np.zeros((n, ld, ld)) if want_R else None}
    out = _DramOut(*[_ptr(res[x], _dp) for x in ("mean", "std", "final_theta", "sigma_mean", "sigma_std",
                                                 "accept_rate")], _ptr(res["n_evals"], _i64p),
                   _ptr(res["chain"], _dp), _ptr(res["s2chain"], _dp), _ptr(res["R"], _dp))
    offsets = np.ascontiguousarray(cells.offsets, np.int64)
    t, m, p = (np.ascontiguousarray(a, np.float64) for a in (cells.t, cells.ms2, cells.pp7))
    h = _ConstructHolder(construct)
    L = lib()
    L.oracle_dram_run.argtypes = [_i64p, _dp, _dp, _dp, C.c_int64, C.POINTER(_Construct), C.c_int64, _i32p, _i64p,
                                  _dp, _dp, _dp, _dp, _dp, _dp, _dp, C.c_int64, C.POINTER(_DramOpts),
                                  C.POINTER(_DramOut), C.c_int]
    L.oracle_dram_run.restype = C.c_int
    rc = L.oracle_dram_run(_ptr(offsets, _i64p), _ptr(t, _dp), _ptr(m, _dp), _ptr(p, _dp), len(offsets) - 1,
                           C.byref(h.s), n, _ptr(cid, _i32p), _ptr(k, _i64p), _ptr(theta0, _dp), _ptr(lower, _dp),
                           _ptr(upper, _dp), _ptr(prior_mu, _dp), _ptr(prior_sig, _dp), _ptr(qcov_diag, _dp),
                           _ptr(s20, _dp), ld, C.byref(o), C.byref(out), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle_dram_run failed: {rc}")
    return res
