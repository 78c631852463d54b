"""Multi-GPU layout: cells are independent, so the path shards with no data-path collective.

The reference's only parallelism is ``parfor (cellNum = 1:N, numParPools)``
(``TranscriptionCycleMCMC.m:161``): independent chains, sliced outputs. Here each rank (one
process per GPU, ``torch.distributed`` over RCCL) owns a contiguous cell range balanced by
work, evaluates it on its own GPU, and the per-cell results are gathered once at the end --
the only collective, replacing parfor's sliced-output assembly (``:315-356``).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np


def shard_bounds(weights: Sequence[float], world: int) -> np.ndarray:
    """Contiguous partition of items with the given work weights into ``world`` ranges
    whose weight sums are as even as a prefix split allows. Returns ``bounds[world+1]``;
    rank r owns ``[bounds[r], bounds[r+1])``."""
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if world < 1:
        raise ValueError("world must be >= 1")
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(cum, target, side="left"))
        if k > 0 and abs(cum[k - 1] - target) <= abs(cum[min(k, n)] - target):
            k -= 1
        bounds.append(min(max(k, bounds[-1]), n))
    bounds.append(n)
    return np.asarray(bounds, dtype=np.int64)


# Prior means of the reference's x0 draw (TranscriptionCycleMCMC.m:200-208): v ~ U(1,3), tau ~ U(0,4).
_V_MEAN, _TAU_MEAN = 2.0, 2.0


def cell_weights(cells, L0: float = 6.626, v0=None) -> np.ndarray:
    """Work per cell ~ N_c x W_c: N_c grid rows, each summing over the cohorts
    inside the elongation window, W_c = (L0 + tau*v) / (v * d_c) grid steps (capped at N_c) at
    the prior means of v and tau; d_c = mean(diff(t)) is the cell's grid increment
    (SumofSquares...m:29). ``v0`` (hierarchical fit, a mapping by 1-based cell_index or a
    sequence over all cells) replaces the prior mean of v where given.

    ``cells`` is a :class:`~.data.Cells`, or (the round-1 signature) an array of the cells'
    point counts N_c: without times there is no window, and the weights are N_c alone."""
    from .mcmc import PreviousFit, _per_cell

    if not hasattr(cells, "lengths"):
        lens = np.asarray(cells, dtype=np.float64)
        if lens.ndim != 1:
            raise ValueError("cell_weights: expected a Cells table or a 1-D array of point counts")
        return lens.copy()
    if v0 is not None and not hasattr(v0, "get") and len(v0) != cells.n_cells:
        raise ValueError(f"cell_weights: v0 has {len(v0)} entries for {cells.n_cells} cells "
                         "(a sequence must cover every cell; use a cell_index mapping for a subset)")
    n = cells.lengths.astype(np.float64)
    w = np.empty(cells.n_cells)
    for c in range(cells.n_cells):
        t = cells.cell(c)[0]
        v = _V_MEAN
        p = _per_cell(v0, c)
        if isinstance(p, PreviousFit):
            p = p.mean_v
        if p is not None and np.isfinite(p) and p > 0:
            v = float(p)
        d = (t[-1] - t[0]) / (len(t) - 1) if len(t) > 1 else 1.0
        win = (L0 + _TAU_MEAN * v) / (v * d) if d > 0 else n[c]
        w[c] = n[c] * min(max(win, 1.0), max(n[c], 1.0))
    return w


def gather_rows(local: np.ndarray, group=None, device: Optional[str] = None) -> np.ndarray:
    """All-gather per-rank row blocks (rank order) over ``torch.distributed`` -- RCCL on GPUs
    (backend 'nccl'), gloo on CPU. Rows may differ in count between ranks."""
    import torch
    import torch.distributed as dist

    local = np.ascontiguousarray(local, np.float64)
    if not dist.is_available() or not dist.is_initialized():
        return local.copy()  # one process, no process group: the gather of one rank
    world = dist.get_world_size(group)
    rows = local.shape[0]
    width = int(np.prod(local.shape[1:])) if local.ndim > 1 else 1
    dev = torch.device(device) if device else torch.device("cpu")
    n_t = torch.tensor([rows], dtype=torch.int64, device=dev)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, n_t, group=group)
    counts = [int(c.item()) for c in counts]
    mx = max(counts) if counts else 0
    buf = torch.zeros((mx, width), dtype=torch.float64, device=dev)
    if rows:
        buf[:rows] = torch.from_numpy(local.reshape(rows, width)).to(dev)
    outs = [torch.zeros((mx, width), dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    parts = [o[:c].cpu().numpy() for o, c in zip(outs, counts)]
    res = np.concatenate(parts, axis=0) if parts else np.zeros((0, width))
    return res.reshape((-1,) + local.shape[1:]) if local.ndim > 1 else res.reshape(-1)


# ---------------------------------------------------------------------------
# Sharded fit: the parfor over cells (TranscriptionCycleMCMC.m:161) across GPUs
# ---------------------------------------------------------------------------

_SCALARS = ("mean_v", "sigma_v", "mean_ton", "sigma_ton", "mean_A", "sigma_A", "mean_tau", "sigma_tau",
            "mean_MS2_basal", "sigma_MS2_basal", "mean_PP7_basal", "sigma_PP7_basal", "mean_R", "sigma_R",
            "mean_sigma", "sigma_sigma")


def pack_results(fr, n_max: int) -> np.ndarray:
    """One float64 row per fitted cell: cell_index, ApprovedFits, N, accept rate, the 16 scalar
    summaries, then mean_dR, sigma_dR, simMS2, simPP7 (each padded to ``n_max``): the per-cell
    output of the reference's parfor body (:315-356) as a fixed-width row for one all-gather."""
    k = len(fr.MCMCresults)
    out = np.full((k, 4 + len(_SCALARS) + 4 * n_max), np.nan)
    for i, (r, pl) in enumerate(zip(fr.MCMCresults, fr.MCMCplot)):
        n = len(r["mean_dR"])
        out[i, 0], out[i, 1], out[i, 2], out[i, 3] = r["cell_index"], r["ApprovedFits"], n, fr.accept_rate[i]
        out[i, 4:4 + len(_SCALARS)] = [r[f] for f in _SCALARS]
        base = 4 + len(_SCALARS)
        for j, v in enumerate((r["mean_dR"], r["sigma_dR"], pl["simMS2"], pl["simPP7"])):
            out[i, base + j * n_max:base + j * n_max + n] = v
    return out


def unpack_results(rows: np.ndarray, cells, dataset_name: str, n_evals: int, elapsed_ms: float,
                   cell_offset: int = 0):
    """Inverse of :func:`pack_results` over the gathered rows (any rank order): a ``FitResult``
    sorted by cell, with ``MCMCplot``'s data columns restored from ``cells``. Raw chains are not
    gathered (``MCMCchain`` entries are empty): they stay on the rank that sampled them.
    ``cells`` may hold only a contiguous block of the dataset starting at dataset-wide index
    ``cell_offset`` (a rank that loaded only its shard): cells outside it get empty data columns
    (``t_plot`` / ``MS2_plot`` / ``PP7_plot``) -- the simulated rows are always there."""
    from .mcmc import FitResult

    rows = rows[np.argsort(rows[:, 0], kind="stable")]
    n_max = (rows.shape[1] - 4 - len(_SCALARS)) // 4
    results, plots, chains = [], [], []
    base = 4 + len(_SCALARS)
    for row in rows:
        c, n = int(row[0]) - 1, int(row[2])
        r = {f: float(v) for f, v in zip(_SCALARS, row[4:base])}
        r["mean_dR"] = row[base:base + n].copy()
        r["sigma_dR"] = row[base + n_max:base + n_max + n].copy()
        r["cell_index"], r["ApprovedFits"] = c + 1, int(row[1])
        from .mcmc import RESULT_FIELDS

        results.append({f: r[f] for f in RESULT_FIELDS})
        lc = c - int(cell_offset)
        if 0 <= lc < cells.n_cells:
            t, m, p = (a.copy() for a in cells.cell(lc))
        else:
            t = m = p = np.zeros(0)
        plots.append({"t_plot": t, "MS2_plot": m, "PP7_plot": p,
                      "simMS2": row[base + 2 * n_max:base + 2 * n_max + n].copy(),
                      "simPP7": row[base + 3 * n_max:base + 3 * n_max + n].copy()})
        chains.append({})
    return FitResult(dataset_name, results, plots, chains, rows[:, 3].copy(), int(n_evals), float(elapsed_ms),
                     (rows[:, 0].astype(np.int64) - 1))


def fit_sharded(lk, group=None, device: Optional[str] = None, v0=None, approved=None,
                cell_offset: Optional[int] = None, **fit_kwargs):
    """``TranscriptionCycleMCMC`` over ``torch.distributed`` ranks, one GPU each: rank r fits its
    cells (its own GPU-resident DRAM chains), then ONE all-gather of the packed per-cell results
    (RCCL on GPUs, gloo on CPU) gives every rank the whole dataset's ``MCMCresults`` / ``MCMCplot``
    (the parfor's sliced-output assembly, :315-356). The chains' randomness is keyed by the
    dataset-wide cell index (:func:`mcmc.fit`), and every rank adapts with the kernel the whole fit's
    largest P picks (``DramOptions.adapt_pmax``, all-reduced), so the gathered results equal a
    one-GPU fit of all cells bit for bit -- provided every rank's ``Likelihood`` runs the kernel
    variant the one-GPU one does (``lk.info['rows_per_lane']``, set by the context's longest cell:
    the SS's lane sums follow it). Shards whose longest cells differ in that variant give a valid fit
    whose chains are not bitwise the one-GPU chains; ``rows_per_lane_uniform`` in the result says
    which case a run was.

    Two layouts:
    * ``cell_offset=None``: every rank holds the whole dataset in ``lk`` and fits the contiguous
      range ``shard_bounds`` gives it (balanced by Σ N_c·W̄);
    * ``cell_offset=k``: ``lk`` holds only this rank's contiguous block of the dataset, starting at
      dataset-wide index k (each rank loaded its own shard files); every cell of ``lk`` is fitted.
      A rank with no cells (more ranks than shards) passes ``lk=None``: it fits nothing but takes
      part in every collective, so the other ranks never wait on it.

    ``v0`` / ``approved``: per-cell inputs over ALL cells (by 1-based cell_index in a mapping, or
    0-based in a sequence); ``fit`` reads them by dataset-wide cell, so every shard passes them
    unchanged. The result carries the gather's wall time (``gather_s``), the bytes every rank
    receives in it (``gather_bytes``) and this rank's own ``FitResult`` (``local``: raw chains,
    final states). Without an initialised process group it is the one-rank case."""
    import time

    import torch
    import torch.distributed as dist

    import dataclasses

    from .mcmc import DramOptions, fit, kept_cells

    on = dist.is_available() and dist.is_initialized()
    world, rank = (dist.get_world_size(group), dist.get_rank(group)) if on else (1, 0)
    if lk is None and cell_offset is None:
        raise ValueError("fit_sharded: lk=None (a rank without cells) needs the cell_offset layout")
    cl = lk.cells if lk is not None else None
    if cl is None:
        ids, off = [], int(cell_offset)
    elif cell_offset is None:
        b = shard_bounds(cell_weights(cl, lk.construct.L0, v0), world)
        ids, off = list(range(int(b[rank]), int(b[rank + 1]))), 0
    else:
        ids, off = list(range(cl.n_cells)), int(cell_offset)
    dev = torch.device(device) if device else torch.device("cpu")
    # the whole fit's largest P (over the cells that get a chain) and kernel variant, over the ranks
    kept = kept_cells(cl, ids, v0, off)
    pmax = 7 + int(np.max(cl.lengths[kept])) if kept else 0
    rpl = int(lk.info["rows_per_lane"]) if kept else -1
    rpl_lo, rpl_hi = (rpl, rpl) if kept else (1 << 30, -1)
    if on:
        t = torch.tensor([pmax, rpl_hi, -rpl_lo], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        pmax, rpl_hi, rpl_lo = int(t[0].item()), int(t[1].item()), -int(t[2].item())
    opts = fit_kwargs.pop("opts", None)
    opts = dataclasses.replace(opts) if opts is not None else DramOptions()
    opts.adapt_pmax = max(int(opts.adapt_pmax), pmax)
    fr = fit(lk, cells=ids, v0=v0, approved=approved, cell_offset=off, opts=opts, **fit_kwargs) if ids else None
    n_max = int(np.max(cl.lengths)) if cl is not None and cl.n_cells else 0
    if on and cell_offset is not None:  # shards may differ in their longest cell: one common width
        t = torch.tensor([n_max], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        n_max = int(t.item())
    local = pack_results(fr, n_max) if fr is not None else np.zeros((0, 4 + len(_SCALARS) + 4 * n_max))
    if on:
        dist.barrier(group)
    g0 = time.perf_counter()
    rows = gather_rows(local, group=group, device=device)
    gather_s = time.perf_counter() - g0
    ev, ms = (fr.n_evals, fr.elapsed_ms) if fr else (0, 0.0)
    if on:
        t = torch.tensor([ms, ev], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        ev, ms = int(t[1].item()), float(mx[0].item())
    if cl is None:  # no cells here: the other ranks' rows, without data columns
        from .data import from_lists

        cl = from_lists([], "empty-shard")
    out = unpack_results(rows, cl, cl.name, int(ev), float(ms), cell_offset=off)
    out.gather_s, out.gather_bytes, out.local = gather_s, int(rows.nbytes), fr
    out.rows_per_lane_uniform = rpl_lo >= rpl_hi   # no rank fitted anything, or all ran one variant
    return out
