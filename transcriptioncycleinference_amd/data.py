"""Cell datasets: the reference's ``data`` struct array as a ragged struct-of-arrays.

Reference schema (``README.md:11-16``): a MAT file holding a struct array ``data`` with one
element per cell and fields ``time``, ``MS2``, ``PP7`` (1 x N doubles) and ``name``. The driver
truncates each cell to ``t >= t_start`` and ``t < t_end`` (``TranscriptionCycleMCMC.m:170-175``)
and builds ``data.xdata = t``, ``data.ydata = [MS2, PP7]`` (``:179-181``).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Callable, Optional, Sequence

import numpy as np

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTDATA_NPZ = os.path.join(REPO_ROOT, "tests", "golden", "testdata.npz")


@dataclass
class Cells:
    offsets: np.ndarray  # int64 [C+1]
    t: np.ndarray        # float64
    ms2: np.ndarray
    pp7: np.ndarray
    name: str = "dataset"

    def __post_init__(self):
        self.offsets = np.ascontiguousarray(self.offsets, np.int64)
        self.t = np.ascontiguousarray(self.t, np.float64)
        self.ms2 = np.ascontiguousarray(self.ms2, np.float64)
        self.pp7 = np.ascontiguousarray(self.pp7, np.float64)
        if self.offsets.ndim != 1 or len(self.offsets) < 1 or self.offsets[0] != 0:  # [0]: no cells
            raise ValueError("offsets must be [0, ..., total]")
        if np.any(np.diff(self.offsets) < 0) or self.offsets[-1] != len(self.t):
            raise ValueError("offsets must be non-decreasing and end at len(t)")
        if not (len(self.t) == len(self.ms2) == len(self.pp7)):
            raise ValueError("t, ms2, pp7 must have equal lengths")

    @property
    def n_cells(self) -> int:
        return len(self.offsets) - 1

    @property
    def lengths(self) -> np.ndarray:
        return np.diff(self.offsets)

    def cell(self, c: int):
        o, e = self.offsets[c], self.offsets[c + 1]
        return self.t[o:e], self.ms2[o:e], self.pp7[o:e]

    def data_struct(self, c: int) -> dict:
        """``data.xdata = t; data.ydata = [MS2, PP7]`` (TranscriptionCycleMCMC.m:179-181)."""
        t, m, p = self.cell(c)
        return {"xdata": t.copy(), "ydata": np.concatenate([m, p])}

    def subset(self, ids: Sequence[int]) -> "Cells":
        return from_lists([self.cell(int(c)) for c in ids], self.name)

    def replicate(self, times: int) -> "Cells":
        return self.subset(list(range(self.n_cells)) * times)


def from_lists(cells, name: str = "dataset") -> Cells:
    """Build from ``[(t, ms2, pp7), ...]``."""
    lens = [len(c[0]) for c in cells]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    cat = (lambda i: np.concatenate([np.asarray(c[i], np.float64) for c in cells]) if cells else np.zeros(0))
    return Cells(off, cat(0), cat(1), cat(2), name)


def truncate(t, ms2, pp7, t_start: float = 0.0, t_end: float = math.inf):
    """``indStart = find(t >= t_start,1,'first'); indEnd = find(t < t_end,1,'last')``
    (TranscriptionCycleMCMC.m:170-175)."""
    t = np.asarray(t, np.float64)
    ge = np.nonzero(t >= t_start)[0]
    lt = np.nonzero(t < t_end)[0]
    if len(ge) == 0 or len(lt) == 0 or lt[-1] < ge[0]:
        return t[:0], np.asarray(ms2)[:0], np.asarray(pp7)[:0]
    s, e = ge[0], lt[-1] + 1
    return t[s:e], np.asarray(ms2, np.float64)[s:e], np.asarray(pp7, np.float64)[s:e]


def load_mat(path: str, t_start: float = 0.0, t_end: float = math.inf) -> Cells:
    """Load a reference dataset file (MAT v5 struct array ``data``) with ``scipy.io.loadmat``
    -- a data reader that executes nothing from the file."""
    import scipy.io as sio

    d = sio.loadmat(path, squeeze_me=True, struct_as_record=False)
    if "data" not in d:
        raise ValueError(f"{path}: no struct array named 'data' (README.md:11)")
    arr = np.atleast_1d(d["data"])
    cells = []
    for c in arr:
        t, m, p = truncate(np.atleast_1d(c.time), np.atleast_1d(c.MS2), np.atleast_1d(c.PP7), t_start, t_end)
        cells.append((t, m, p))
    name = str(getattr(arr[0], "name", "dataset")) if len(arr) else "dataset"
    return from_lists(cells, name)


def load_npz(path: str) -> Cells:
    z = np.load(path, allow_pickle=False)
    name = str(z["name"]) if "name" in z.files else os.path.basename(path)
    return Cells(z["offsets"], z["t"], z["ms2"], z["pp7"], name)


def testdata() -> Cells:
    """The reference's 299-cell ``TestScripts/TestData.mat`` (committed as a fixture)."""
    return load_npz(TESTDATA_NPZ)


# ---------------------------------------------------------------------------
# theta helpers (theta order: TranscriptionCycleMCMC.m:210, bounds :242-255)
# ---------------------------------------------------------------------------

THETA_NAMES = ("v", "tau", "ton", "MS2_basal", "PP7_basal", "A", "R")
LOWER = np.array([0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0])
UPPER = np.array([10.0, 20.0, 10.0, 50.0, 50.0, 1.0, 40.0])
DR_BOUNDS = (-30.0, 30.0)


def draw_x0(rng: np.random.Generator, n_points: int, v0: Optional[float] = None) -> np.ndarray:
    """The reference's initial-state distribution (TranscriptionCycleMCMC.m:200-210)."""
    v = 1 + 2 * rng.random() if v0 is None else v0
    ton, A, tau = 4 * rng.random(), rng.random(), 4 * rng.random()
    dR = rng.normal(0.0, 3.0, n_points)
    return np.concatenate([[v, tau, ton, 10.0, 5.0, A, 15.0], dR])


def in_bounds(theta: np.ndarray, n_points: int) -> bool:
    th = np.asarray(theta)
    core = th[:7]
    dR = th[7:7 + n_points]
    return bool(np.all(core >= LOWER) and np.all(core <= UPPER) and np.all(dR >= DR_BOUNDS[0])
                and np.all(dR <= DR_BOUNDS[1]))


def pack_theta(rows: Sequence[np.ndarray], ld: Optional[int] = None) -> np.ndarray:
    """Ragged theta rows -> zero-padded (B, ld) float64 matrix."""
    ld = ld or max(len(r) for r in rows)
    out = np.zeros((len(rows), ld))
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out


# ---------------------------------------------------------------------------
# Synthetic datasets
# ---------------------------------------------------------------------------


def synthetic_times(rng: np.random.Generator, n_points: int) -> np.ndarray:
    """``t_j = 0.2454*j + U(-0.012, 0.012)``, 2 % of gaps widened to ``U(0.34, 0.71)``
    (TestData's dt range 0.2305-0.7103, mean 0.2548)."""
    gaps = 0.2454 + rng.uniform(-0.012, 0.012, n_points - 1)
    wide = rng.random(n_points - 1) < 0.02
    gaps[wide] = rng.uniform(0.34, 0.71, int(wide.sum()))
    return np.concatenate([[0.0], np.cumsum(gaps)])


def synthetic_cells(n_cells: int, n_points: int, seed: int,
                    forward: Callable[[list, np.ndarray], tuple],
                    nan_fraction: float = 0.37):
    """Synthetic cells: times as above, ground-truth theta from the reference's x0
    distribution, data = forward model + N(0,1) on MS2 and N(0,2) on PP7, then i.i.d.
    NaN-masked with probability ``nan_fraction``.

    ``forward(times_list, theta_matrix) -> (ms2, pp7)`` evaluates the noise-free signal
    at the acquisition times (e.g. ``Likelihood.forward`` on a times-only table).
    Returns ``(cells, theta_true)``.
    """
    rng = np.random.default_rng(seed)
    times = [synthetic_times(rng, n_points) for _ in range(n_cells)]
    theta = np.stack([draw_x0(rng, n_points) for _ in range(n_cells)])
    theta[:, 3] = rng.uniform(5, 15, n_cells)
    theta[:, 4] = rng.uniform(2, 8, n_cells)
    theta[:, 5] = rng.uniform(0.2, 1.0, n_cells)
    theta[:, 6] = rng.uniform(8, 20, n_cells)
    ms2, pp7 = forward(times, theta)
    out = []
    for c in range(n_cells):
        m = ms2[c, :n_points] + rng.normal(0, 1, n_points)
        p = pp7[c, :n_points] + rng.normal(0, 2, n_points)
        m[rng.random(n_points) < nan_fraction] = np.nan
        p[rng.random(n_points) < nan_fraction] = np.nan
        out.append((times[c], m, p))
    return from_lists(out, f"synthetic-{n_cells}x{n_points}-seed{seed}"), theta
