"""World-size-2 gloo run of the multi-GPU layout on CPU: shard cells, process per rank, one
gather at the end (the RCCL all-gather on GPUs). Compute per rank is a stand-in here (CPU only);
the kernels are covered by tests/test_parity_gpu.py."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from transcriptioncycleinference_amd import testdata
    from transcriptioncycleinference_amd.parallel import cell_weights, gather_rows, shard_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cells = testdata()
    b = shard_bounds(cell_weights(cells), world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    # per-cell "result" rows: (cell index, N, sum of finite data) -- deterministic stand-in
    local = np.array([[c, cells.lengths[c], np.nansum(cells.cell(c)[1])] for c in range(lo, hi)])
    full = gather_rows(local)
    import torch

    t = torch.tensor([float(hi - lo)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((full, b, float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_shard_and_gather():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, bounds, mx = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from transcriptioncycleinference_amd import testdata

    cells = testdata()
    assert full.shape == (299, 3)
    np.testing.assert_array_equal(full[:, 0], np.arange(299))
    np.testing.assert_array_equal(full[:, 1], cells.lengths)
    assert bounds[0] == 0 and bounds[-1] == 299
    assert mx == max(bounds[1] - bounds[0], bounds[2] - bounds[1])


def _pack_worker(rank, world, port, q):
    import torch.distributed as dist

    from transcriptioncycleinference_amd import testdata
    from transcriptioncycleinference_amd.parallel import cell_weights, gather_rows, pack_results, shard_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cells = testdata()
    b = shard_bounds(cell_weights(cells), world)
    fr = _fake_fit(cells, range(int(b[rank]), int(b[rank + 1])))
    rows = gather_rows(pack_results(fr, int(cells.lengths.max())))
    if rank == 0:
        q.put(rows)
    dist.barrier()
    dist.destroy_process_group()


def _fake_fit(cells, ids):
    """A FitResult with deterministic per-cell values (stand-in for the GPU fit)."""
    from transcriptioncycleinference_amd.mcmc import RESULT_FIELDS, FitResult

    res, plots = [], []
    for c in ids:
        n = int(cells.lengths[c])
        r = {f: float(c) + k / 100 for k, f in enumerate(RESULT_FIELDS)}
        r["mean_dR"], r["sigma_dR"] = np.arange(n) + c, np.arange(n) * 0.5 - c
        r["cell_index"], r["ApprovedFits"] = c + 1, c % 2
        res.append(r)
        plots.append({"simMS2": np.full(n, c * 1.5), "simPP7": np.full(n, -c * 1.0)})
    return FitResult(cells.name, res, plots, [{} for _ in ids], np.array([c / 1000 for c in ids]), 0, 0.0)


def test_gloo_world2_sharded_results_gather_round_trip():
    """parallel.fit_sharded's data path on CPU: per-rank packed results, one all-gather, unpacked
    into the whole dataset's MCMCresults/MCMCplot in cell order (the GPU fit itself is covered by
    tests/test_dram_gpu.py::test_sharded_fit_world2_equals_the_one_gpu_fit)."""
    from transcriptioncycleinference_amd import testdata
    from transcriptioncycleinference_amd.parallel import unpack_results

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pack_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rows = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cells = testdata()
    fr = unpack_results(rows[::-1], cells, cells.name, 7, 1.0)  # any row order
    want = _fake_fit(cells, range(299))
    assert [r["cell_index"] for r in fr.MCMCresults] == list(range(1, 300))
    for a, b, pa, pb in zip(fr.MCMCresults, want.MCMCresults, fr.MCMCplot, want.MCMCplot):
        for f in a:
            np.testing.assert_array_equal(a[f], b[f], err_msg=f)
        np.testing.assert_array_equal(pa["simMS2"], pb["simMS2"])
        np.testing.assert_array_equal(pa["simPP7"], pb["simPP7"])
        assert len(pa["t_plot"]) == len(a["mean_dR"])
    np.testing.assert_array_equal(fr.accept_rate, want.accept_rate)


def test_config_shards_are_the_same_dataset_at_every_world_size():
    """bench.py configs 4/5: 10,000 cells as 8 fixed shards of 1,250 (seed
    20201028 + shard); rank r of N owns a contiguous range of whole shards, so the global dataset --
    and with chains keyed by dataset-wide cell index, the fit -- does not depend on N."""
    import bench

    for world in range(1, 11):
        got = [list(bench.config_shards(r, world)) for r in range(world)]
        flat = [s for g in got for s in g]
        assert flat == list(range(bench.CONFIG_SHARDS)), (world, got)
        sizes = [len(g) for g in got]
        assert max(sizes) - min(sizes) <= 1
    assert bench.CONFIG_SHARDS * bench.CONFIG_SHARD_CELLS == 10000


def test_unpack_results_of_a_shard_local_rank():
    """A rank that loaded only its own block of cells (parallel.fit_sharded's cell_offset layout)
    unpacks the gathered rows of every cell: its own cells get their data columns, the others the
    simulated rows only."""
    from transcriptioncycleinference_amd import testdata
    from transcriptioncycleinference_amd.parallel import pack_results, unpack_results

    cells = testdata()
    rows = pack_results(_fake_fit(cells, range(299)), int(cells.lengths.max()))
    block = cells.subset(range(100, 150))
    fr = unpack_results(rows, block, "x", 0, 0.0, cell_offset=100)
    assert [r["cell_index"] for r in fr.MCMCresults] == list(range(1, 300))
    for c, p in enumerate(fr.MCMCplot):
        n = int(cells.lengths[c])
        assert len(p["simMS2"]) == n
        if 100 <= c < 150:
            np.testing.assert_array_equal(p["t_plot"], cells.cell(c)[0])
        else:
            assert len(p["t_plot"]) == 0


class _StubLikelihood:
    """What fit_sharded reads of a Likelihood (cells, construct.L0, info) -- no GPU context."""

    def __init__(self, cells, rpl=2):
        from types import SimpleNamespace

        self.cells = cells
        self.construct = SimpleNamespace(L0=6.626)
        self.info = {"rows_per_lane": rpl}


def _empty_rank_worker(rank, world, port, q, blocks):
    """fit_sharded in the cell_offset layout with the GPU fit replaced by a deterministic stand-in;
    ranks whose block is empty pass lk=None (more ranks than shards: bench.config_shards)."""
    import torch.distributed as dist

    import transcriptioncycleinference_amd.mcmc as M
    from transcriptioncycleinference_amd import testdata
    from transcriptioncycleinference_amd.parallel import fit_sharded, pack_results

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = testdata()
    seen = {}

    def fake_fit(lk, cells=None, cell_offset=0, opts=None, **kw):
        seen["adapt_pmax"] = opts.adapt_pmax
        return _fake_fit(full, [cell_offset + c for c in cells])

    M.fit = fake_fit
    lo, hi = blocks[rank]
    lk = _StubLikelihood(full.subset(range(lo, hi))) if hi > lo else None
    fr = fit_sharded(lk, cell_offset=lo)
    q.put((rank, pack_results(fr, int(full.lengths.max())), seen.get("adapt_pmax"), fr.rows_per_lane_uniform,
           fr.local is None))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world3_fit_sharded_with_a_rank_without_cells():
    """with more ranks than shards some ranks hold no cells. fit_sharded(lk=None) on such a
    rank fits nothing but joins the all-reduce and the all-gather, so no rank waits forever; every rank
    ends with the whole dataset's rows in cell order, and the ranks that fit pass the fit-wide largest
    P (adapt_pmax) to the sampler. Rank 0 is the empty one here, as bench.config_shards gives it at
    N > 8 (3 ranks, 2 shards: config_shards(0, 3, 2) is empty)."""
    import bench
    from transcriptioncycleinference_amd import testdata

    full = testdata()
    shards = [(0, 150), (150, 299)]
    owned = [list(bench.config_shards(r, 3, 2)) for r in range(3)]
    assert owned == [[], [0], [1]]
    blocks = [(shards[o[0]][0], shards[o[-1]][1]) if o else (0, 0) for o in owned]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_rank_worker, args=(r, 3, port, q, blocks)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=240) for _ in range(3)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _fake_fit(full, range(299))
    from transcriptioncycleinference_amd.parallel import pack_results

    rows = pack_results(want, int(full.lengths.max()))
    pmax = 7 + int(full.lengths.max())
    for r in range(3):
        np.testing.assert_array_equal(got[r][0], rows)
        assert got[r][1] == (None if r == 0 else pmax)
        assert got[r][2] is True
    assert got[0][3] and not got[1][3]
