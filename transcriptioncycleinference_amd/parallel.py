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


def cell_weights(lengths: Sequence[int]) -> np.ndarray:
    """Work per cell ~ rows x elongation window; the window is theta-dependent, rows are not."""
    return np.asarray(lengths, dtype=np.float64)


def gather_rows(local: np.ndarray, group=None, device: Optional[str] = None) -> np.ndarray:
    """All-gather per-rank row blocks (rank order) over ``torch.distributed`` -- RCCL on GPUs
    (backend 'nccl'), gloo on CPU. Rows may differ in count between ranks."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    local = np.ascontiguousarray(local, np.float64)
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
