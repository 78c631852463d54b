"""CPU oracle (numpy restatement) of the reference likelihood hot path.

TEST INFRASTRUCTURE ONLY.  This module is the *checker*, never the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it.  The shipped path (``transcriptioncycleinference_amd``) never
imports anything under ``oracle/`` and fails loudly when its HIP library is
missing.

It restates, line by line and in the reference's *matrix form* (the full
time x polymerase position matrix is materialised, exactly as MATLAB does),

* ``SumofSquaresFunction_TranscriptionCycleMCMC``
  (``/root/reference/src/SumofSquaresFunction_TranscriptionCycleMCMC.m:1-64``),
* ``ConstantElongationSim``
  (``/root/reference/src/dependencies/ConstantElongationSim.m:1-67``),
* ``GetFluorFromPolPos``
  (``/root/reference/src/GetFluorFromPolPos.m:1-71``),

plus the MATLAB builtins the path uses (``colon``, ``mean``, ``interp1``
linear, ``nansum``).  Pinned by the reference's own golden vectors
(``TestScripts/28-Oct-2020-TestData.mat`` ``MCMCplot.simMS2/simPP7`` at the
posterior means, see ``tests/test_oracle_golden.py``) and statistically by the
``s2chain`` sigma^2 draws of ``28-Oct-2020-TestData_RawChain.mat``.

Arithmetic-order rules (the discontinuous decisions -- ``floor(counter)`` and
the strict ``<``/``>`` masks -- depend on them):

* no fused multiply-add anywhere (numpy never fuses);
* the loading counter is accumulated sequentially, multiply then add
  (``ConstantElongationSim.m:60``);
* positions are accumulated forward, ``x(i+1,k) = x(i,k) + v*dt(i)``
  (``ConstantElongationSim.m:64``);
* the interpolation grid uses MATLAB's documented colon algorithm.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

EPS = np.finfo(np.float64).eps

# ---------------------------------------------------------------------------
# Construct table (GetFluorFromPolPos.m:18-30)
# ---------------------------------------------------------------------------


@dataclass
class Construct:
    """Reporter construct: gene length before the ``tau*v`` dwell term and the
    per-segment stem-loop map (``GetFluorFromPolPos.m:18-44``)."""

    L0: float
    ms2_start: Sequence[float]
    ms2_end: Sequence[float]
    ms2_loopn: Sequence[float]
    pp7_start: Sequence[float]
    pp7_end: Sequence[float]
    pp7_loopn: Sequence[float]
    name: str = field(default="custom")


def builtin_construct(name: str) -> Construct:
    """``GetFluorFromPolPos.m:18``: only ``'P2P-MS2v5-LacZ-PP7v4'`` is defined;
    any other string leaves the table undefined (MATLAB errors)."""
    if name == "P2P-MS2v5-LacZ-PP7v4":
        return Construct(6.626, [0.024], [1.299], [24.0], [4.292], [5.758], [24.0], name)
    raise ValueError(f"construct {name!r} is not defined (GetFluorFromPolPos.m:18)")


# ---------------------------------------------------------------------------
# MATLAB builtins
# ---------------------------------------------------------------------------


def matlab_mean(x: np.ndarray) -> float:
    """``mean`` of a row vector: sequential sum / count."""
    s = 0.0
    for xi in np.asarray(x, dtype=np.float64).tolist():
        s = s + xi
    return s / len(x) if len(x) else float("nan")


def matlab_colon(a: float, d: float, b: float) -> np.ndarray:
    """``a:d:b`` by MATLAB's documented colon algorithm (``colonop``).

    Used at ``SumofSquaresFunction_TranscriptionCycleMCMC.m:30``.
    """
    a, d, b = float(a), float(d), float(b)
    if not (math.isfinite(a) and math.isfinite(d) and math.isfinite(b)):
        return np.array([np.nan])
    if d == 0 or (a < b and d < 0) or (b < a and d > 0):
        return np.zeros(0)
    tol = 2.0 * EPS * max(abs(a), abs(b))
    sig = 1.0 if d > 0 else -1.0
    if a == math.floor(a) and d == 1:
        n = math.floor(b) - a
    elif a == math.floor(a) and d == math.floor(d):
        q = math.floor(a / d)
        r = a - q * d
        n = math.floor((b - r) / d) - q
    else:
        n = round_half_away((b - a) / d)
        if sig * (a + n * d - b) > tol:
            n = n - 1
    n = int(n)
    c = a + n * d
    if sig * (c - b) > -tol:
        c = b
    v = np.zeros(n + 1)
    k = np.arange(0, n // 2 + 1, dtype=np.float64)
    v[k.astype(int)] = a + k * d
    v[(n - k).astype(int)] = c - k * d
    if n % 2 == 0:
        v[n // 2] = (a + c) / 2
    return v


def round_half_away(x: float) -> float:
    """MATLAB ``round``: halves away from zero."""
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def interp1_linear(x: np.ndarray, y: np.ndarray, xq: np.ndarray) -> np.ndarray:
    """``interp1(x, y, xq)`` (default 'linear'); NaN outside ``[x(1), x(end)]``.

    Interval ``k`` is the last with ``x(k) <= xq`` (the last interval for
    ``xq == x(end)``); value ``y(k) + s*(y(k+1)-y(k))``, ``s = (xq-x(k))/(x(k+1)-x(k))``.
    The exact MATLAB interpolation formula is not published; it differs from
    this one at most at the ulp level (the SS is continuous in it).
    """
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    xq = np.asarray(xq, dtype=np.float64)
    out = np.full(xq.shape, np.nan)
    m = len(x)
    for j, q in enumerate(xq.tolist()):
        if not (q >= x[0] and q <= x[-1]):
            continue
        k = int(np.searchsorted(x, q, side="right")) - 1
        k = min(max(k, 0), m - 2)
        s = (q - x[k]) / (x[k + 1] - x[k])
        out[j] = y[k] + s * (y[k + 1] - y[k])
    return out


def nansum(x: np.ndarray) -> float:
    s = 0.0
    for xi in np.asarray(x, dtype=np.float64).tolist():
        if xi == xi:
            s = s + xi
    return s


# ---------------------------------------------------------------------------
# ConstantElongationSim.m
# ---------------------------------------------------------------------------


class ReferenceError(RuntimeError):
    """A MATLAB run-time error the reference would raise on this input."""


def constant_elongation_sim(v: float, ton: float, R: np.ndarray, t: np.ndarray) -> np.ndarray:
    """``ConstantElongationSim(v,ton,R,t)`` -> ``x`` (m x n position matrix)."""
    R = np.array(R, dtype=np.float64)[:-1]  # :33
    R[R < 0] = 0  # :36
    t = np.asarray(t, dtype=np.float64)
    m = t.shape[0]  # :39
    dt = np.empty(m - 1)
    for i in range(m - 1):  # :42-45
        dt[i] = t[i + 1] - t[i]
    if R.shape[0] != dt.shape[0]:
        raise ReferenceError("Matrix dimensions must agree (ConstantElongationSim.m:47)")
    prod = R * dt
    s = 0.0
    for p in prod.tolist():  # sum(R.*dt,2), sequential
        s = s + p
    n = int(math.floor(s)) if math.isfinite(s) else 0  # :47
    x = np.zeros((m, max(n, 0)))  # :50
    counter = 0.0  # :53
    vd = [v * dti for dti in dt.tolist()]
    for i in range(m - 1):  # :56
        if t[i] < ton:  # :57
            continue
        counter = counter + R[i] * dt[i]  # :60 (multiply, then add)
        kmax = math.floor(counter) if math.isfinite(counter) else 0  # :61
        if kmax <= 0:
            continue
        if kmax > x.shape[1]:
            # x(i,k) on the right-hand side reads past the last column.
            raise ReferenceError("Index exceeds matrix dimensions (ConstantElongationSim.m:64)")
        x[i + 1, :kmax] = x[i, :kmax] + vd[i]  # :64
        mask = x[i + 1, :kmax] < 0  # :65 (row mask used as a linear index)
        if mask.any():
            lin = np.nonzero(mask)[0]  # column-major linear indexing into x
            xf = x.reshape(-1, order="F")
            xf[lin] = 0
            x = xf.reshape(x.shape, order="F")
    return x


# ---------------------------------------------------------------------------
# GetFluorFromPolPos.m
# ---------------------------------------------------------------------------


def _rowsum(mat: np.ndarray) -> np.ndarray:
    """``sum(M,2)'``, accumulated column by column (sequential per row)."""
    out = np.zeros(mat.shape[0])
    for k in range(mat.shape[1]):
        out = out + mat[:, k]
    return out


def get_fluor_from_polpos(construct: Construct, PolPos: np.ndarray, v: float, tau: float,
                          MS2_basal: float, PP7_basal: float):
    """``[MS2,PP7] = GetFluorFromPolPos(construct,PolPos,v,tau,MS2_basal,PP7_basal)``."""
    L_MS2 = construct.L0 + tau * v  # :19
    L_PP7 = construct.L0 + tau * v  # :20
    MS2: np.ndarray | float = 0.0  # :29
    PP7: np.ndarray | float = 0.0  # :30
    for i in range(len(construct.ms2_start)):  # :47
        a, e = construct.ms2_start[i], construct.ms2_end[i]
        fv = construct.ms2_loopn[i] / 24  # :48
        MS2map = np.zeros(PolPos.shape)  # :49
        MS2map[(PolPos > e) & (PolPos < L_MS2)] = fv  # :50
        frac = (PolPos > a) & (PolPos < e)  # :51
        MS2map[frac] = (PolPos[frac] - a) * fv / (e - a)  # :52
        MS2 = MS2 + _rowsum(MS2map)  # :54
        MS2 = np.where(MS2 < MS2_basal, MS2_basal, MS2)  # :57

        a, e = construct.pp7_start[i], construct.pp7_end[i]
        fv = construct.pp7_loopn[i] / 24  # :60
        PP7map = np.zeros(PolPos.shape)  # :61
        PP7map[(PolPos > e) & (PolPos < L_PP7)] = fv  # :62
        frac = (PolPos > a) & (PolPos < e)  # :63
        PP7map[frac] = (PolPos[frac] - a) * fv / (e - a)  # :64
        PP7 = PP7 + _rowsum(PP7map)  # :66
        PP7 = np.where(PP7 < PP7_basal, PP7_basal, PP7)  # :69
    return np.asarray(MS2, dtype=np.float64), np.asarray(PP7, dtype=np.float64)


# ---------------------------------------------------------------------------
# SumofSquaresFunction_TranscriptionCycleMCMC.m
# ---------------------------------------------------------------------------


def interp_grid(t: np.ndarray) -> np.ndarray:
    """``SumofSquares...m:29-30``: ``dt = mean(diff(t)); t_interp = t(1):dt:t(end)``."""
    t = np.asarray(t, dtype=np.float64)
    d = np.empty(len(t) - 1)
    for i in range(len(t) - 1):
        d[i] = t[i + 1] - t[i]
    dt = matlab_mean(d)
    return matlab_colon(t[0], dt, t[-1])


def sum_of_squares(construct: Construct, data: dict, x: np.ndarray) -> float:
    """``SS = SumofSquaresFunction_TranscriptionCycleMCMC(construct,data,x)``."""
    t = np.asarray(data["xdata"], dtype=np.float64)  # :28
    t_interp = interp_grid(t)  # :29-30
    fluorExp = np.asarray(data["ydata"], dtype=np.float64)  # :33
    x = np.asarray(x, dtype=np.float64)
    v, tau, ton, MS2_basal, PP7_basal, A, R = (float(q) for q in x[:7])  # :35-41
    dR = x[7:]  # :42
    R_full = R + dR  # :45
    PolPos = constant_elongation_sim(v, ton, R_full, t_interp)  # :49
    MS2, PP7 = get_fluor_from_polpos(construct, PolPos, v, tau, MS2_basal, PP7_basal)  # :50
    MS2 = A * MS2  # :51
    MS2 = interp1_linear(t_interp, MS2, t)  # :55
    PP7 = interp1_linear(t_interp, PP7, t)  # :56
    fluorSim = np.concatenate([MS2, PP7])  # :57
    residuals = fluorExp - fluorSim  # :61
    return nansum(residuals ** 2)  # :64


def forward_raw(construct: Construct, t: np.ndarray, theta: np.ndarray):
    """Forward model on the raw acquisition times, as the plot/summary call at
    ``TranscriptionCycleMCMC.m:307-309`` does (no grid, no interp1)."""
    theta = np.asarray(theta, dtype=np.float64)
    v, tau, ton, b1, b2, A, R = (float(q) for q in theta[:7])
    PolPos = constant_elongation_sim(v, ton, R + theta[7:], np.asarray(t, dtype=np.float64))
    MS2, PP7 = get_fluor_from_polpos(construct, PolPos, v, tau, b1, b2)
    return A * MS2, PP7


def forward_interp(construct: Construct, t: np.ndarray, theta: np.ndarray):
    """Simulated MS2/PP7 at the acquisition times, through the uniform grid and
    ``interp1`` exactly as inside the SS (``SumofSquares...m:28-56``)."""
    t = np.asarray(t, dtype=np.float64)
    t_interp = interp_grid(t)
    theta = np.asarray(theta, dtype=np.float64)
    v, tau, ton, b1, b2, A, R = (float(q) for q in theta[:7])
    PolPos = constant_elongation_sim(v, ton, R + theta[7:], t_interp)
    MS2, PP7 = get_fluor_from_polpos(construct, PolPos, v, tau, b1, b2)
    return interp1_linear(t_interp, A * MS2, t), interp1_linear(t_interp, PP7, t)
