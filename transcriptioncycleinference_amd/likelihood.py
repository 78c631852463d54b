"""Batched likelihood on one MI355X: a resident cell table + the HIP kernels behind ``include/tci.h``.

``Likelihood`` is the batched form of mcmcstat's ``model.ssfun`` (set at
``TranscriptionCycleMCMC.m:186,258``; contract ``ss = ssfun(theta, data)``): the parfor over cells
(``:161``) becomes one launch over B = cells x proposals rows.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .construct import Construct, as_construct
from .data import Cells


class Likelihood:
    """SS evaluator bound to one device and one dataset (the C ``tci_ctx``)."""

    def __init__(self, cells: Cells, construct="P2P-MS2v5-LacZ-PP7v4", device: int = 0,
                 lib_path: Optional[str] = None):
        self._lib = _lib.load(lib_path)  # lib_path: an A/B build variant (default: libtci.so)
        self.cells = cells
        self.construct: Construct = as_construct(construct)
        self.device = int(device)
        cs, self._cs_arrays = self.construct.to_c()
        self._cells_c = _lib.tci_cells(cells.n_cells, _lib.ptr(cells.offsets, _lib._i64p), _lib.ptr(cells.t, _lib._dp),
                                       _lib.ptr(cells.ms2, _lib._dp), _lib.ptr(cells.pp7, _lib._dp))
        h = C.c_void_p()
        rc = self._lib.tci_create(C.byref(self._cells_c), C.byref(cs), self.device, C.byref(h))
        if rc != _lib.TCI_OK:
            msg = self._lib.tci_last_error(h).decode() if h.value else "tci_create failed"
            if h.value:
                self._lib.tci_destroy(h)
            raise _lib.TciError(rc, msg)
        self._h = h
        self.lengths = cells.lengths.astype(np.int64)

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.tci_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc != _lib.TCI_OK:
            raise _lib.TciError(rc, self._lib.tci_last_error(self._h).decode())

    @property
    def info(self) -> dict:
        i = _lib.tci_info()
        self._check(self._lib.tci_get_info(self._h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in i._fields_}

    def set_force_exact(self, scan: bool = False, positions: bool = False):
        """Test hook: force the exact serial counter scan and/or the exact position sweep."""
        self._check(self._lib.tci_set_force_exact_scan(self._h, int(bool(scan)) | (int(bool(positions)) << 1)))

    def grid(self, cell: int) -> np.ndarray:
        m = C.c_int64()
        out = np.empty(int(self.lengths[cell]))
        self._check(self._lib.tci_cell_grid(self._h, int(cell), _lib.ptr(out, _lib._dp), len(out), C.byref(m)))
        return out[: m.value]

    # -- evaluation (host arrays, synchronous) -----------------------------
    def ss_batch(self, theta: np.ndarray, cell_id: Sequence[int], active: Optional[np.ndarray] = None) -> np.ndarray:
        """``ss[b] = ssfun(theta[b], cell[cell_id[b]])``; inactive rows -> +Inf."""
        theta = np.ascontiguousarray(np.atleast_2d(theta), np.float64)
        cid = np.ascontiguousarray(cell_id, np.int32)
        B, ld = theta.shape
        if len(cid) != B:
            raise ValueError("cell_id must have one entry per theta row")
        act = None if active is None else np.ascontiguousarray(active, np.uint8)
        if act is not None and len(act) != B:
            raise ValueError("active must have one entry per theta row")
        out = np.empty(B)
        self._check(self._lib.tci_ss_batch(self._h, _lib.ptr(theta, _lib._dp), ld, _lib.ptr(cid, _lib._i32p),
                                           _lib.ptr(act, _lib._u8p), B, _lib.ptr(out, _lib._dp)))
        return out

    def ssfun(self, theta: np.ndarray, cell: int) -> float:
        """One ``ssfun(theta, data)`` call for one cell."""
        th = np.ascontiguousarray(theta, np.float64)
        out = np.empty(1)
        self._check(self._lib.tci_ssfun(self._h, int(cell), _lib.ptr(th, _lib._dp), len(th), _lib.ptr(out, _lib._dp)))
        return float(out[0])

    def forward(self, theta: np.ndarray, cell_id: Sequence[int], grid: str = "interp"):
        """Simulated (MS2, PP7) at each row's acquisition times, shape (B, max N); NaN-padded.
        ``grid='raw'``: forward model on the raw times (TranscriptionCycleMCMC.m:307-309);
        ``grid='interp'``: through the uniform grid + interp1, as inside the SS."""
        mode = {"interp": _lib.TCI_GRID_INTERP, "raw": _lib.TCI_GRID_RAW}[grid]
        theta = np.ascontiguousarray(np.atleast_2d(theta), np.float64)
        cid = np.ascontiguousarray(cell_id, np.int32)
        B, ld = theta.shape
        ld_out = int(self.lengths[cid].max()) if B else 1
        ms2 = np.full((B, ld_out), np.nan)
        pp7 = np.full((B, ld_out), np.nan)
        self._check(self._lib.tci_forward(self._h, _lib.ptr(theta, _lib._dp), ld, _lib.ptr(cid, _lib._i32p), B, mode,
                                          _lib.ptr(ms2, _lib._dp), _lib.ptr(pp7, _lib._dp), ld_out))
        return ms2, pp7

    # -- evaluation (device buffers, asynchronous) --------------------------
    def ss_batch_device(self, theta, cell_id, out, active=None, stream=None) -> None:
        """Launch on device tensors already resident in HBM (torch tensors or raw pointers):
        ``theta`` (B, ld) float64, ``cell_id`` (B,) int32, ``out`` (B,) float64, optional
        ``active`` (B,) uint8. ``stream``: a torch stream / raw hipStream_t (None or 0 = the
        HIP default stream). Nothing is synchronised."""
        def addr(x):
            if x is None:
                return None
            return x.data_ptr() if hasattr(x, "data_ptr") else int(x)

        if hasattr(theta, "shape"):
            B, ld = int(theta.shape[0]), int(theta.shape[1])
            self._check_device_args(theta, cell_id, out, active, B)
        else:
            raise ValueError("theta must be a 2-D device tensor")
        st = getattr(stream, "cuda_stream", stream)
        self._check(self._lib.tci_ss_batch_async(self._h, addr(theta), ld, addr(cell_id), addr(active), B, addr(out),
                                                 st))

    @staticmethod
    def _check_device_args(theta, cell_id, out, active, B):
        import torch

        if theta.dtype != torch.float64 or not theta.is_contiguous() or not theta.is_cuda:
            raise ValueError("theta must be a contiguous float64 device tensor")
        if cell_id.dtype != torch.int32 or cell_id.numel() != B or not cell_id.is_cuda:
            raise ValueError("cell_id must be an int32 device tensor with one entry per row")
        if out.dtype != torch.float64 or out.numel() < B or not out.is_cuda:
            raise ValueError("out must be a float64 device tensor with >= B entries")
        if active is not None and (active.dtype != torch.uint8 or active.numel() != B or not active.is_cuda):
            raise ValueError("active must be a uint8 device tensor with one entry per row")


def version() -> str:
    return _lib.load().tci_version().decode()
