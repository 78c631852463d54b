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
    b = shard_bounds(cell_weights(cells.lengths), world)
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
