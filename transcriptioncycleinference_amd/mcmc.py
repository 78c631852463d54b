"""Fit driver: the reference's per-cell MCMC setup + the GPU-resident batched DRAM + its outputs.

Mirrors ``src/TranscriptionCycleMCMC.m``:

* per-cell setup (``:161-270``): truncation, ``data``, x0 (``:193-210``), the proposal
  covariance J0 (``:214-231``), bounds (``:233-255``), Gaussian priors on dR (``:254``),
  ``model.sigma2 = 1`` (``:212,259``);
* ``mcmcrun`` (``:273``) -> :func:`dram_run` (``tci_dram_run``: all chains at once on the GPU);
* summaries (``:275-303``), the forward model at the means (``:305-309``), the
  ``MCMCchain`` / ``MCMCresults`` / ``MCMCplot`` structs (``:149-157,315-356``), the pruning of
  skipped cells (``:359-369``) and the two result files (``:371-378``).

The reference runs cells in a parfor with independent MATLAB RNG streams (``rand``/``normrnd``).
Here x0 comes from ``numpy.random.default_rng([seed, cell])`` and the chains from Philox streams, so a
fit reproduces the reference's *distribution*, not its exact draws.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import datetime
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Optional, Sequence

import numpy as np

from . import _lib
from .data import Cells, draw_x0

RESULT_FIELDS = ("mean_v", "sigma_v", "mean_ton", "sigma_ton", "mean_A", "sigma_A", "mean_tau", "sigma_tau",
                 "mean_MS2_basal", "sigma_MS2_basal", "mean_PP7_basal", "sigma_PP7_basal", "mean_R", "sigma_R",
                 "mean_dR", "sigma_dR", "mean_sigma", "sigma_sigma", "cell_index", "ApprovedFits")  # :151-155
CHAIN_FIELDS = ("v_chain", "ton_chain", "A_chain", "tau_chain", "MS2_basal_chain", "PP7_basal_chain", "R_chain",
                "dR_chain", "s2chain")  # :149-150
PLOT_FIELDS = ("t_plot", "MS2_plot", "PP7_plot", "simMS2", "simPP7")  # :156-157
THETA_INDEX = {"v": 0, "tau": 1, "ton": 2, "MS2_basal": 3, "PP7_basal": 4, "A": 5, "R": 6}


@dataclass
class DramOptions:
    """``options`` of ``TranscriptionCycleMCMC.m:263-270`` plus mcmcstat's DRAM defaults."""

    n_steps: int = 20000          # options.nsimu = n_steps (:264; default :40)
    burnintime: int = 10000       # options.burnintime = n_burn (:267; default :39)
    adaptint: int = 100           # :268
    ntry: int = 2                 # 'dram' (:269)
    updatesigma: bool = True      # :265
    drscale: float = 5.0
    adascale: float = 0.0         # 0: 2.4/sqrt(npar)
    qcovadj: float = 1e-5
    burnin_scale: float = 10.0
    stats_from: int = 10000       # chain(n_burn:end, :) (:276)
    thin: int = 0
    seed: int = 20201028
    engine: str = "auto"          # "auto" | "fused" | "batched" | "walk" (include/tci.h TCI_DRAM_*): identical chains
    max_chunk: int = 0            # FUSED/WALK rows per draws pass + walk (0 = automatic); identical chains
    adapt_pmax: int = 0           # a shard of a larger fit: that fit's largest P (the adaptation kernel's pick)
    kernel_times: bool = False    # FUSED/WALK: HIP-event device time per kernel class (DramResult.kernel_ms)

    ENGINES = {"auto": 0, "fused": 1, "batched": 2, "walk": 3}

    def to_c(self, chain_keys: Optional[np.ndarray] = None) -> "_lib.tci_dram_options":
        """``chain_keys`` (int64 [n_chains], kept alive by the caller): chain c's RNG stream key."""
        if self.engine not in self.ENGINES:
            raise ValueError(f"engine must be one of {sorted(self.ENGINES)}, got {self.engine!r}")
        return _lib.tci_dram_options(int(self.n_steps), int(self.burnintime), int(self.adaptint), int(self.ntry),
                                     int(bool(self.updatesigma)), float(self.drscale), float(self.adascale),
                                     float(self.qcovadj), float(self.burnin_scale), int(self.stats_from),
                                     int(self.thin), int(self.seed) & 0xFFFFFFFFFFFFFFFF,
                                     self.ENGINES[self.engine], int(self.max_chunk), _lib.ptr(chain_keys, _lib._i64p),
                                     int(self.adapt_pmax), int(bool(self.kernel_times)))


@dataclass
class DramResult:
    mean: np.ndarray
    std: np.ndarray
    final_theta: np.ndarray
    sigma_mean: np.ndarray
    sigma_std: np.ndarray
    accept_rate: np.ndarray
    n_evals: np.ndarray
    chain: Optional[np.ndarray]
    s2chain: Optional[np.ndarray]
    elapsed_ms: float
    qcov_R: Optional[np.ndarray] = None   # final proposal factor (upper, R'R = mcmcstat results.qcov)
    kernel_ms: Optional[np.ndarray] = None        # DramOptions.kernel_times: ms per class (draws, walk, adapt,
    #                                               the split draws' first-chunk launch; include/tci.h)
    kernel_launches: Optional[np.ndarray] = None  # and launches per class


def dram_run(lk, cell_id, theta0, lower, upper, prior_mu, prior_sig, qcov_diag, sigma2_0,
             opts: DramOptions, want_qcov: bool = False, chain_keys=None) -> DramResult:
    """Run one chain per row on the device (``tci_dram_run``). Arrays are (n_chains, ld).
    ``want_qcov``: also return the final proposal factor R (n_chains, ld, ld). ``chain_keys``:
    RNG stream key per chain (default: the row index)."""
    f = lambda a: np.ascontiguousarray(a, np.float64)  # noqa: E731
    theta0, lower, upper, prior_mu, prior_sig, qcov_diag = map(f, (theta0, lower, upper, prior_mu, prior_sig,
                                                                    qcov_diag))
    n, ld = theta0.shape
    cid = np.ascontiguousarray(cell_id, np.int32)
    s20 = f(np.broadcast_to(np.asarray(sigma2_0, np.float64), (n,)))
    mean, std, fin = np.empty((n, ld)), np.empty((n, ld)), np.empty((n, ld))
    smean, sstd, acc = np.empty(n), np.empty(n), np.empty(n)
    nev = np.empty(n, np.int64)
    n_keep = (opts.n_steps + opts.thin - 1) // opts.thin if opts.thin > 0 else 0
    chain = np.empty((n_keep, n, ld)) if n_keep else None
    s2c = np.empty((n_keep, n)) if n_keep else None
    qR = np.empty((n, ld, ld)) if want_qcov else None
    out = _lib.tci_dram_outputs(_lib.ptr(mean, _lib._dp), _lib.ptr(std, _lib._dp), _lib.ptr(fin, _lib._dp),
                                _lib.ptr(smean, _lib._dp), _lib.ptr(sstd, _lib._dp), _lib.ptr(acc, _lib._dp),
                                _lib.ptr(nev, _lib._i64p), _lib.ptr(chain, _lib._dp), _lib.ptr(s2c, _lib._dp),
                                _lib.ptr(qR, _lib._dp), 0.0)   # kernel_ms / kernel_launches: zero-initialised
    keys = None if chain_keys is None else np.ascontiguousarray(chain_keys, np.int64)
    if keys is not None and keys.shape != (n,):
        raise ValueError("chain_keys must have one entry per chain")
    o = opts.to_c(keys)
    P = lambda a: _lib.ptr(a, _lib._dp)  # noqa: E731
    lk._check(lk._lib.tci_dram_run(lk._h, C.byref(o), n, _lib.ptr(cid, _lib._i32p), P(theta0), P(lower), P(upper),
                                   P(prior_mu), P(prior_sig), P(qcov_diag), P(s20), ld, C.byref(out)))
    return DramResult(mean, std, fin, smean, sstd, acc, nev, chain, s2c, float(out.elapsed_ms), qR,
                      np.array(out.kernel_ms[:], np.float64), np.array(out.kernel_launches[:], np.int64))


# ---------------------------------------------------------------------------
# TranscriptionCycleMCMC.m per-cell setup
# ---------------------------------------------------------------------------


def cell_setup(t: np.ndarray, rng: np.random.Generator, ratePriorWidth: float = 50.0,
               v0: Optional[float] = None):
    """x0, lower, upper, prior mu/sig and J0 diagonal for one cell (TranscriptionCycleMCMC.m:193-255).
    ``v0`` given = the hierarchical fit (loadPrevious): v fixed to v0 +- 1e-5 with step 1e-7."""
    n = len(t)
    x0 = draw_x0(rng, n, v0)                                                 # :200-210
    load_prev = v0 is not None
    v_step = 1e-7 if load_prev else 0.05                                      # :217-221
    ton_step = t[-1] - t[-2]                                                  # :222
    J0 = np.concatenate([[v_step, 0.1, ton_step, 1.0, 1.0, 0.05, 0.5], np.full(n, 0.5)])  # :223-231
    v_lo, v_hi = (v0 - 1e-5, v0 + 1e-5) if load_prev else (0.0, 10.0)         # :235-241
    lower = np.concatenate([[v_lo, 0, 0, 0, 0, 0, 0], np.full(n, -30.0)])     # :242-255
    upper = np.concatenate([[v_hi, 20, 10, 50, 50, 1, 40], np.full(n, 30.0)])
    mu = np.zeros(7 + n)
    sig = np.concatenate([np.full(7, np.inf), np.full(n, float(ratePriorWidth))])  # :254
    return x0, lower, upper, mu, sig, J0


@dataclass
class FitResult:
    DatasetName: str
    MCMCresults: List[Dict]
    MCMCplot: List[Dict]
    MCMCchain: List[Dict]
    accept_rate: np.ndarray
    n_evals: int
    elapsed_ms: float
    cell_index: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))   # 0-based, dataset-wide
    final_theta: Optional[np.ndarray] = None   # last chain row per fitted cell (padded), mcmcstat results.theta
    gather_s: float = 0.0                      # parallel.fit_sharded: wall time of the results all-gather
    gather_bytes: int = 0                      # parallel.fit_sharded: bytes every rank receives in it
    local: Optional["FitResult"] = None        # parallel.fit_sharded: this rank's own fit (raw chains, final_theta)
    rows_per_lane_uniform: bool = True         # parallel.fit_sharded: every rank ran the same likelihood variant


@dataclass
class PreviousFit:
    """One ``MCMCresults`` entry of an earlier fit as ``loadPrevious`` keeps it
    (TranscriptionCycleMCMC.m:100-104): the elongation rate and the curation flag."""

    mean_v: Optional[float]
    ApprovedFits: int = 0


def _per_cell(values, c: int):
    """Value for 0-based cell ``c`` of a per-cell input: a mapping keyed by the reference's
    1-based ``cell_index`` (what :func:`load_previous` returns), or a sequence over every cell
    of the dataset (0-based). Missing from a mapping -> None."""
    if values is None:
        return None
    if isinstance(values, Mapping):
        return values.get(c + 1)
    return values[c]


@dataclass
class FitPlan:
    """Per-chain inputs of one fit (TranscriptionCycleMCMC.m:193-255), rows padded to ``ld``."""

    cells: List[int]          # 0-based cell indices that get a chain (skipped cells removed, :196-198)
    x0: np.ndarray
    lower: np.ndarray
    upper: np.ndarray
    prior_mu: np.ndarray
    prior_sig: np.ndarray
    qcov_diag: np.ndarray
    approved: List[int]       # MCMCresults.ApprovedFits per fitted cell (:345-350)


def _previous(v0, approved, g: int):
    """(skip, v0 of the cell or None, ApprovedFits) for dataset-wide 0-based cell ``g`` (:193-198, :345-350)."""
    prev = _per_cell(v0, g)
    a = 0
    if isinstance(prev, PreviousFit):
        a = int(prev.ApprovedFits)
        prev = prev.mean_v
    if v0 is not None and (prev is None or np.size(prev) != 1 or not np.isfinite(float(prev))):
        return True, None, a
    ap = _per_cell(approved, g)
    if ap is not None:
        a = int(ap)
    return False, (None if v0 is None else float(prev)), a


def kept_cells(cl: Cells, ids: Sequence[int], v0=None, cell_offset: int = 0) -> List[int]:
    """The cells of ``ids`` that get a chain: those with a previous entry when ``v0`` is given
    (:196-198), all of them otherwise -- :func:`plan_fit`'s rule, without drawing anything."""
    return [int(c) for c in ids if not _previous(v0, None, int(cell_offset) + int(c))[0]]


def plan_fit(cl: Cells, ids: Sequence[int], seed: int, ratePriorWidth: float = 50.0, v0=None,
             approved=None, cell_offset: int = 0) -> FitPlan:
    """The parfor body's per-cell setup for the cells ``ids`` (host only, no GPU).

    ``v0`` (loadPrevious, :193-198) and ``approved`` are per-cell inputs read by cell, never by
    position in ``ids``: a mapping keyed by 1-based ``cell_index`` (:194 matches
    ``[MCMCresults.cell_index] == cellNum``) or a sequence over all cells. A ``PreviousFit`` value
    carries both. A cell with no previous entry, or an empty/NaN ``mean_v``, is skipped
    (``continue``, :196-198) and so pruned from the outputs (:359-369). ``ApprovedFits`` is the
    previous fit's when v0 came from one (:345-347) unless ``approved`` overrides it; 0 otherwise
    (:349). ``cell_offset``: the dataset-wide index of ``cl``'s cell 0 (``cl`` holds one shard of a
    larger dataset): x0 and the per-cell inputs are keyed by the dataset-wide index."""
    rows, keep, appr = [], [], []
    for c in ids:
        c = int(c)
        t = cl.cell(c)[0]
        g = int(cell_offset) + c
        skip, vv, a = _previous(v0, approved, g)
        if skip:
            continue
        rows.append(cell_setup(t, np.random.default_rng([int(seed), g]), ratePriorWidth, vv))
        keep.append(c)
        appr.append(a)
    ld = max((len(r[0]) for r in rows), default=7)

    def stack(i, fill):
        out = np.full((len(rows), ld), fill, np.float64)
        for k, r in enumerate(rows):
            out[k, :len(r[i])] = r[i]
        return out

    return FitPlan(keep, stack(0, 0.0), stack(1, -np.inf), stack(2, np.inf), stack(3, 0.0), stack(4, np.inf),
                   stack(5, 1.0), appr)


def fit(lk, n_steps: int = 20000, n_burn: int = 10000, ratePriorWidth: float = 50.0, seed: int = 0,
        v0=None, approved=None, thin: int = 0, cells: Optional[Sequence[int]] = None,
        opts: Optional[DramOptions] = None, cell_offset: int = 0) -> FitResult:
    """``TranscriptionCycleMCMC`` for one dataset on the GPU: one DRAM chain per cell.

    ``lk``: a ``Likelihood`` holding the (truncated) cells. ``v0``: the previous fit of a
    hierarchical run (loadPrevious): ``load_previous(path)`` (cell_index -> PreviousFit), a
    mapping cell_index -> mean_v, or a sequence of rates over ALL cells (None/NaN = no entry).
    Cells without an entry are skipped (``continue``, :196-198) and pruned from the outputs
    (:359-369); see :func:`plan_fit`. ``thin``: keep every thin-th raw chain row in ``MCMCchain``
    (the reference keeps all rows from n_burn, :276-283 -- ~193 MB/cell at 200k steps; thin=1
    reproduces that). ``cells``: fit only these cell indices (a shard).

    Everything random is keyed by the cell index -- x0 by ``default_rng([seed, cell])``, the chain
    by RNG stream ``cell`` -- so fitting a subset of the cells (one GPU's shard,
    :func:`parallel.fit_sharded`) reproduces those cells' results of the full fit bit for bit.
    ``cell_offset``: ``lk`` holds only a contiguous block of a larger dataset, starting at this
    dataset-wide cell index; keys, x0, per-cell inputs and ``cell_index`` use the dataset-wide index
    (a rank that loaded only its own shard reproduces the one-GPU fit of the whole dataset)."""
    cl: Cells = lk.cells
    ids = list(range(cl.n_cells)) if cells is None else [int(c) for c in cells]
    off = int(cell_offset)
    plan = plan_fit(cl, ids, seed, ratePriorWidth, v0, approved, cell_offset=off)
    keep = plan.cells
    if not keep:
        return FitResult(cl.name, [], [], [], np.zeros(0), 0, 0.0)
    # a private copy: the caller's options object is never modified
    o = dataclasses.replace(opts) if opts is not None else DramOptions()
    o.n_steps, o.burnintime, o.stats_from, o.thin = int(n_steps), int(n_burn), int(max(n_burn, 1)), int(thin)
    o.seed = int(seed) * 1000003 + 20201028
    res = dram_run(lk, np.array(keep, np.int32), plan.x0, plan.lower, plan.upper, plan.prior_mu, plan.prior_sig,
                   plan.qcov_diag, 1.0, o, chain_keys=np.array(keep, np.int64) + off)
    # forward model at the means on the raw times (:307-309)
    ms2, pp7 = lk.forward(res.mean, np.array(keep, np.int32), grid="raw")
    results, plots, chains = [], [], []
    for k, c in enumerate(keep):
        t, m, p = cl.cell(c)
        n = len(t)
        mean, std = res.mean[k, :7 + n], res.std[k, :7 + n]
        r = {}
        for name in ("v", "ton", "A", "tau", "MS2_basal", "PP7_basal", "R"):
            r["mean_" + name] = float(mean[THETA_INDEX[name]])
            r["sigma_" + name] = float(std[THETA_INDEX[name]])
        r["mean_dR"], r["sigma_dR"] = mean[7:].copy(), std[7:].copy()
        r["mean_sigma"], r["sigma_sigma"] = float(res.sigma_mean[k]), float(res.sigma_std[k])
        r["cell_index"] = off + c + 1                                         # :343 (1-based)
        r["ApprovedFits"] = plan.approved[k]                                  # :345-350
        results.append({f: r[f] for f in RESULT_FIELDS})
        plots.append({"t_plot": t.copy(), "MS2_plot": m.copy(), "PP7_plot": p.copy(),
                      "simMS2": ms2[k, :n].copy(), "simPP7": pp7[k, :n].copy()})
        ch = {}
        if res.chain is not None:
            # rows kept: 1, 1+thin, ...; the reference stores chain(n_burn:end, :) (:276-283)
            rows_idx = 1 + thin * np.arange(res.chain.shape[0])
            sel = rows_idx >= max(n_burn, 1)
            th = res.chain[sel, k, :7 + n]
            for name in ("v", "ton", "A", "tau", "MS2_basal", "PP7_basal", "R"):
                ch[name + "_chain"] = th[:, THETA_INDEX[name]].copy()
            ch["dR_chain"] = th[:, 7:].copy()
            ch["s2chain"] = res.s2chain[:, k].copy()  # s2chain is not sliced by n_burn (:323)
        chains.append(ch)
    return FitResult(cl.name, results, plots, chains, res.accept_rate, int(res.n_evals.sum()), res.elapsed_ms,
                     np.array(keep, np.int64) + off, res.final_theta)


# ---------------------------------------------------------------------------
# Result files (TranscriptionCycleMCMC.m:371-378)
# ---------------------------------------------------------------------------


def _struct_array(items: List[Dict], fields: Sequence[str]) -> np.ndarray:
    arr = np.empty((1, len(items)), dtype=[(f, object) for f in fields])
    for i, it in enumerate(items):
        for f in fields:
            v = it.get(f, np.zeros((0, 0)))
            if isinstance(v, np.ndarray) and v.ndim == 1:
                v = v[None, :]  # MATLAB row vectors
            arr[0, i][f] = v
    return arr


def save_results(fit_result: FitResult, save_loc: str = ".", date: Optional[str] = None):
    """Write ``<date>-<DatasetName>.mat`` (MCMCresults, MCMCplot, DatasetName) and
    ``<date>-<DatasetName>_RawChain.mat`` (MCMCchain), as the reference does (:373-378).
    ``date`` defaults to MATLAB's ``date`` format (dd-Mmm-yyyy). Returns the two paths."""
    import scipy.io as sio

    date = date or datetime.date.today().strftime("%d-%b-%Y")
    base = os.path.join(save_loc, f"{date}-{fit_result.DatasetName}")
    sio.savemat(base + ".mat", {"MCMCresults": _struct_array(fit_result.MCMCresults, RESULT_FIELDS),
                                "MCMCplot": _struct_array(fit_result.MCMCplot, PLOT_FIELDS),
                                "DatasetName": fit_result.DatasetName})
    chains = [c if c else {f: np.zeros((0, 1)) for f in CHAIN_FIELDS} for c in fit_result.MCMCchain]
    for c in chains:  # chains are column vectors in the reference (chain(n_burn:end, k))
        for f in CHAIN_FIELDS:
            if f in c and isinstance(c[f], np.ndarray) and c[f].ndim == 1:
                c[f] = c[f][:, None]
    sio.savemat(base + "_RawChain.mat", {"MCMCchain": _struct_array(chains, CHAIN_FIELDS)})
    return base + ".mat", base + "_RawChain.mat"


def load_previous(results_path: str) -> Dict[int, PreviousFit]:
    """``loadPrevious`` (hierarchical fit, TranscriptionCycleMCMC.m:84-107): the ``MCMCresults``
    of an earlier result file as ``cell_index -> PreviousFit(mean_v, ApprovedFits)``. The fit
    looks each cell up by ``cell_index`` (:194), so cells missing from the file (pruned there,
    :359-369) are skipped, never shifted. A repeated cell_index keeps its first entry (MATLAB's
    ``v0 = MCMCresults(cellToload).mean_v`` takes the first of a comma list). Read with
    scipy.io.loadmat: a data reader, nothing executes."""
    import scipy.io as sio

    d = sio.loadmat(results_path, squeeze_me=True, struct_as_record=False)
    out: Dict[int, PreviousFit] = {}
    for r in np.atleast_1d(d["MCMCresults"]):
        ci = getattr(r, "cell_index", None)
        if ci is None or np.size(ci) != 1:
            continue
        v = getattr(r, "mean_v", None)
        v = float(v) if v is not None and np.size(v) == 1 else None   # [] -> skipped at :196
        a = getattr(r, "ApprovedFits", 0)
        a = int(a) if np.size(a) == 1 else 0
        out.setdefault(int(ci), PreviousFit(v, a))
    return out


def load_previous_v(results_path: str) -> Dict[int, float]:
    """``cell_index -> mean_v`` of an earlier result file (entries with a usable rate only)."""
    return {c: p.mean_v for c, p in load_previous(results_path).items()
            if p.mean_v is not None and math.isfinite(p.mean_v)}
