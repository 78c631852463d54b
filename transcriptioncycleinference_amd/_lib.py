"""ctypes binding of the C ABI in ``include/tci.h`` (``libtci.so``, built in-tree for gfx950).

There is no fallback: if the library is missing the import of any compute entry point
raises :class:`TciLibraryMissing`. The product path never calls a CPU implementation.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libtci.so")

TCI_OK = 0
TCI_EINVAL = -1
TCI_EHIP = -2
TCI_ENOMEM = -3
TCI_EDIM = -4
TCI_ERANGE = -5
TCI_MAX_SEG = 4
TCI_MAX_POINTS = 2048
TCI_GRID_INTERP = 0
TCI_GRID_RAW = 1

_dp = C.POINTER(C.c_double)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)


class TciLibraryMissing(ImportError):
    pass


class TciError(RuntimeError):
    """An error status returned through the C ABI (message from ``tci_last_error``)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[tci {code}] {msg}")
        self.code = code


class tci_cells(C.Structure):
    _fields_ = [("n_cells", C.c_int64), ("offsets", _i64p), ("t", _dp), ("ms2", _dp), ("pp7", _dp)]


class tci_construct(C.Structure):
    _fields_ = [("L0", C.c_double), ("n_seg", C.c_int32),
                ("ms2_start", _dp), ("ms2_end", _dp), ("ms2_loopn", _dp),
                ("pp7_start", _dp), ("pp7_end", _dp), ("pp7_loopn", _dp)]


class tci_info(C.Structure):
    _fields_ = [("device", C.c_int32), ("rows_per_lane", C.c_int32), ("n_cells", C.c_int64),
                ("max_points", C.c_int64), ("device_bytes", C.c_int64)]


class tci_dram_options(C.Structure):
    _fields_ = [("n_steps", C.c_int64), ("burnintime", C.c_int64), ("adaptint", C.c_int64), ("ntry", C.c_int32),
                ("updatesigma", C.c_int32), ("drscale", C.c_double), ("adascale", C.c_double),
                ("qcovadj", C.c_double), ("burnin_scale", C.c_double), ("stats_from", C.c_int64),
                ("thin", C.c_int64), ("seed", C.c_uint64), ("engine", C.c_int32), ("max_chunk", C.c_int32),
                ("chain_keys", C.POINTER(C.c_int64)), ("adapt_pmax", C.c_int64), ("kernel_times", C.c_int64)]


class tci_dram_outputs(C.Structure):
    _fields_ = [("mean", _dp), ("std", _dp), ("final_theta", _dp), ("sigma_mean", _dp), ("sigma_std", _dp),
                ("accept_rate", _dp), ("n_evals", _i64p), ("chain", _dp), ("s2chain", _dp), ("qcov_R", _dp),
                ("elapsed_ms", C.c_double), ("kernel_ms", C.c_double * 4), ("kernel_launches", C.c_int64 * 4)]


# (name, restype, argtypes) for every symbol declared in include/tci.h
SIGNATURES = [
    ("tci_construct_by_name", C.c_int, [C.c_char_p, C.POINTER(tci_construct)]),
    ("tci_create", C.c_int, [C.POINTER(tci_cells), C.POINTER(tci_construct), C.c_int, C.POINTER(C.c_void_p)]),
    ("tci_destroy", C.c_int, [C.c_void_p]),
    ("tci_last_error", C.c_char_p, [C.c_void_p]),
    ("tci_get_info", C.c_int, [C.c_void_p, C.POINTER(tci_info)]),
    ("tci_set_force_exact_scan", C.c_int, [C.c_void_p, C.c_int]),
    ("tci_ss_batch", C.c_int, [C.c_void_p, _dp, C.c_int64, _i32p, _u8p, C.c_int64, _dp]),
    ("tci_ss_batch_async", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                     C.c_void_p, C.c_void_p]),
    ("tci_ssfun", C.c_int, [C.c_void_p, C.c_int32, _dp, C.c_int64, _dp]),
    ("tci_forward", C.c_int, [C.c_void_p, _dp, C.c_int64, _i32p, C.c_int64, C.c_int, _dp, _dp, C.c_int64]),
    ("tci_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("tci_cell_points", C.c_int, [C.c_void_p, C.c_int32, _i64p]),
    ("tci_cell_grid", C.c_int, [C.c_void_p, C.c_int32, _dp, C.c_int64, _i64p]),
    ("tci_dram_defaults", C.c_int, [C.POINTER(tci_dram_options)]),
    ("tci_dram_run", C.c_int, [C.c_void_p, C.POINTER(tci_dram_options), C.c_int64, _i32p, _dp, _dp, _dp, _dp, _dp,
                               _dp, _dp, C.c_int64, C.POINTER(tci_dram_outputs)]),
    ("tci_version", C.c_char_p, []),
]

_lib = None


def load(path: str | None = None):
    """Load ``libtci.so`` (raises :class:`TciLibraryMissing` when it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise TciLibraryMissing(
            f"{p} not found: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')")
    lib = C.CDLL(p)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def ptr(a, typ):
    return None if a is None else a.ctypes.data_as(typ)
