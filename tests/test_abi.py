"""The C-ABI library loads and exports every symbol include/tci.h declares (no GPU calls)."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "tci.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tci_[a-z_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from transcriptioncycleinference_amd import _lib
    from transcriptioncycleinference_amd.build import build_library

    build_library()
    return _lib.load()


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("tci_create", "tci_destroy", "tci_ss_batch", "tci_ss_batch_async", "tci_ssfun", "tci_forward",
              "tci_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    from transcriptioncycleinference_amd import _lib

    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(declared_symbols()) == bound


def test_library_is_built_for_gfx950():
    from transcriptioncycleinference_amd.build import LIB

    data = open(LIB, "rb").read()
    assert b"gfx950" in data


def test_host_only_entry_points(lib):
    from transcriptioncycleinference_amd import _lib

    assert lib.tci_version().startswith(b"tci-mi355x")
    cs = _lib.tci_construct()
    assert lib.tci_construct_by_name(b"P2P-MS2v5-LacZ-PP7v4", C.byref(cs)) == 0
    assert cs.L0 == 6.626 and cs.n_seg == 1
    assert (cs.ms2_start[0], cs.ms2_end[0], cs.pp7_start[0], cs.pp7_end[0]) == (0.024, 1.299, 4.292, 5.758)
    assert lib.tci_construct_by_name(b"P2P-other", C.byref(cs)) == _lib.TCI_EINVAL
    assert lib.tci_destroy(None) == _lib.TCI_EINVAL
    assert lib.tci_last_error(None) == b"null context"


def test_create_rejects_bad_input_before_touching_a_device(lib):
    """Validation runs on the host before any HIP call (no GPU needed)."""
    import numpy as np

    from transcriptioncycleinference_amd import _lib
    from transcriptioncycleinference_amd.construct import builtin_construct

    cs, keep = builtin_construct("P2P-MS2v5-LacZ-PP7v4").to_c()

    def create(t, off):
        t = np.ascontiguousarray(t, np.float64)
        off = np.ascontiguousarray(off, np.int64)
        y = np.zeros_like(t)
        cells = _lib.tci_cells(len(off) - 1, _lib.ptr(off, _lib._i64p), _lib.ptr(t, _lib._dp),
                               _lib.ptr(y, _lib._dp), _lib.ptr(y, _lib._dp))
        h = C.c_void_p()
        rc = lib.tci_create(C.byref(cells), C.byref(cs), 0, C.byref(h))
        msg = lib.tci_last_error(h).decode() if h.value else ""
        if h.value:
            lib.tci_destroy(h)
        return rc, msg

    rc, msg = create([0.0], [0, 1])
    assert rc == _lib.TCI_EINVAL and "fewer than 2" in msg
    rc, msg = create([0.0, 1.0, 0.5], [0, 3])
    assert rc == _lib.TCI_EINVAL and "increasing" in msg
    rc, msg = create([0.0, np.nan], [0, 2])
    assert rc == _lib.TCI_EINVAL
    n = _lib.TCI_MAX_POINTS + 1  # past the long-cell kernel's LDS tables
    rc, msg = create(np.arange(float(n)), [0, n])
    assert rc == _lib.TCI_EINVAL and "max" in msg


def test_dram_engine_codes_match_the_header():
    """DramOptions.ENGINES (Python) carries the same codes as include/tci.h's TCI_DRAM_*."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    src = open(os.path.join(ROOT, "include", "tci.h")).read()
    hdr = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"#define TCI_DRAM_([A-Z]+) (\d+)", src)}
    assert hdr == DramOptions.ENGINES
    with pytest.raises(ValueError):
        DramOptions(engine="lockstep").to_c()
