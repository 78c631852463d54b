"""Reference-named entry points (the MATLAB interface this path replaces), on the HIP path.

* ``SumofSquaresFunction_TranscriptionCycleMCMC(construct, data, x)``
  -- ``src/SumofSquaresFunction_TranscriptionCycleMCMC.m:1``: same arguments and meaning
  (``data = {'xdata': t, 'ydata': [MS2, PP7]}``, ``x = [v,tau,ton,MS2_basal,PP7_basal,A,R,dR]``),
  returns the scalar SS. Errors where the reference errors (undefined construct, grid/data
  length mismatch) by raising.
* ``make_ssfun(construct)`` -- the closure ``ssfun = @(x,data) ...`` of
  ``src/TranscriptionCycleMCMC.m:186``, i.e. what ``model.ssfun`` holds (``:258``).
* ``simulate_fluorescence(construct, t, theta)`` -- the forward evaluation the driver
  does at the posterior means, ``GetFluorFromPolPos(construct, ConstantElongationSim(...))``
  then ``simMS2 = mean_A*simMS2`` (``:307-309``), on the raw times.

Each distinct (construct, data) pair gets a cached single-cell device context, so repeated
calls with the same ``data`` (what mcmcstat does) do not re-upload.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np

from .construct import as_construct
from .data import from_lists
from .likelihood import Likelihood

_CACHE: "OrderedDict[tuple, Likelihood]" = OrderedDict()
_CACHE_MAX = 64


def _ctx_for(construct, t: np.ndarray, ms2: np.ndarray, pp7: np.ndarray, device: int) -> Likelihood:
    cs = as_construct(construct)
    h = hashlib.sha1()
    for a in (t, ms2, pp7):
        h.update(np.ascontiguousarray(a, np.float64).tobytes())
    key = (repr(cs), h.hexdigest(), device)
    lk = _CACHE.get(key)
    if lk is None:
        lk = Likelihood(from_lists([(t, ms2, pp7)]), cs, device)
        _CACHE[key] = lk
        while len(_CACHE) > _CACHE_MAX:
            _CACHE.popitem(last=False)[1].close()
    else:
        _CACHE.move_to_end(key)
    return lk


def _split_data(data):
    t = np.asarray(data["xdata"], np.float64).ravel()
    y = np.asarray(data["ydata"], np.float64).ravel()
    n = len(t)
    if len(y) != 2 * n:
        raise ValueError("data.ydata must be [MS2, PP7] with 2*length(xdata) entries (TranscriptionCycleMCMC.m:181)")
    return t, y[:n], y[n:]


def SumofSquaresFunction_TranscriptionCycleMCMC(construct, data, x, device: int = 0) -> float:  # noqa: N802
    """``SS = SumofSquaresFunction_TranscriptionCycleMCMC(construct,data,x)`` on the GPU."""
    t, m, p = _split_data(data)
    x = np.asarray(x, np.float64).ravel()
    if len(x) < 7 + len(t):
        raise ValueError(f"x must hold [v,tau,ton,MS2_basal,PP7_basal,A,R,dR(1:{len(t)})]")
    return _ctx_for(construct, t, m, p, device).ssfun(x, 0)


def make_ssfun(construct, device: int = 0):
    """``ssfun = @(x,data) SumofSquaresFunction_TranscriptionCycleMCMC(construct,data,x)``."""
    as_construct(construct)  # fail early on an undefined construct, as the reference would

    def ssfun(x, data):
        return SumofSquaresFunction_TranscriptionCycleMCMC(construct, data, x, device)

    return ssfun


def simulate_fluorescence(construct, t, theta, device: int = 0):
    """(simMS2, simPP7) of the forward model on the raw times t (TranscriptionCycleMCMC.m:307-309)."""
    t = np.asarray(t, np.float64).ravel()
    nan = np.full(len(t), np.nan)
    lk = _ctx_for(construct, t, nan, nan, device)
    ms2, pp7 = lk.forward(np.asarray(theta, np.float64)[None, :], [0], grid="raw")
    return ms2[0, : len(t)], pp7[0, : len(t)]


def clear_cache():
    while _CACHE:
        _CACHE.popitem()[1].close()
