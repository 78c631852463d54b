#!/usr/bin/env python3
"""Benchmark: forward-model SS evaluations/sec on the 299-cell TestData (BASELINE.json metric).

One *launch* = one batched ssfun evaluation of the whole per-GPU workload: every TestData cell
(299) x K DRAM-style proposals (default 256), i.e. the evaluations mcmcstat would request from
299 independent chains over K lockstep proposals. One *step* = --launches-per-step (128) such
launches over distinct resident proposal batches, so the timed region is >= 100 ms at the default
--steps 20. Proposals are Gaussian around the
fixture chain states with the reference's proposal variances J0 (TranscriptionCycleMCMC.m:
217-231); proposals outside the parameter box (:242-255) are marked inactive and are NOT
counted (mcmcstat rejects them without calling ssfun). All inputs are resident in HBM before
timing; the kernel is launched on torch's current stream through the C ABI.

Multi-GPU (torchrun, one process per GPU, RCCL): weak scaling -- every rank evaluates its own
replica of the 299-cell workload with a rank-specific seed; there is no data-path collective.
The per-cell results are gathered once after timing (the reference's parfor output assembly),
and the elapsed time is the max over ranks.

Beside `value` (kernel mode, K = 256) the line carries the K in {1, 64, 256, 1024} sweep, the
drop-in's per-call latency, the metric's 200k-step end-to-end fit (BASELINE config 2), configs
3/4/5, and the CPU baseline at all host threads and at one core.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFS = 78.6   # MI355X FP64 dense peak, vector and MFMA alike: 1024 SIMDs x 32 FLOP/clk x 2.4 GHz (a
                       # v_mfma_f64_16x16x4, 2,048 FLOP, issues every 64 cycles: DESIGN.md §7, r05q)
SIMDS = 256 * 4        # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9       # max engine clock (MI355X_MICROARCH.md)
CONSTRUCT = "P2P-MS2v5-LacZ-PP7v4"


def proposal_batch(cells, P: int, seed: int):
    """theta (B, ld), cell_id (B,), active (B,) for 299 cells x P proposals (host, numpy)."""
    from transcriptioncycleinference_amd.data import DR_BOUNDS, LOWER, UPPER

    with np.load(os.path.join(ROOT, "tests", "golden", "chain_theta.npz"), allow_pickle=False) as f:
        z = {k: f[k] for k in f.files}  # materialise once (NpzFile re-reads on every access)
    off = z["theta_offsets"]
    rng = np.random.default_rng(seed)
    C = cells.n_cells
    lens = cells.lengths
    ld = int(7 + lens.max())
    B = C * P
    theta = np.zeros((B, ld))
    cid = np.repeat(np.arange(C, dtype=np.int32), P)
    # current chain state per cell: a random fixture row of that cell
    rows_of = [np.nonzero(z["cell_id"] == c)[0] for c in range(C)]
    for c in range(C):
        n = int(lens[c])
        t = cells.cell(c)[0]
        picks = rng.choice(rows_of[c], P)
        st = np.stack([z["theta"][off[i]:off[i + 1]] for i in picks])
        # proposal variances J0 = diag([v 0.05, tau 0.1, ton dt_last, MS2 1, PP7 1, A 0.05, R 0.5, dR 0.5])
        var = np.concatenate([[0.05, 0.1, t[-1] - t[-2], 1.0, 1.0, 0.05, 0.5], np.full(n, 0.5)])
        theta[c * P:(c + 1) * P, :7 + n] = st + rng.normal(0.0, 1.0, st.shape) * np.sqrt(var)
    core = theta[:, :7]
    active = np.all((core >= LOWER) & (core <= UPPER), axis=1)
    for c in range(C):
        n = int(lens[c])
        dR = theta[c * P:(c + 1) * P, 7:7 + n]
        active[c * P:(c + 1) * P] &= np.all((dR >= DR_BOUNDS[0]) & (dR <= DR_BOUNDS[1]), axis=1)
    return theta, cid, active.astype(np.uint8)


class ProposalRounds:
    """``rounds`` distinct lockstep proposal batches for 299 cells x K proposals, generated and kept
    resident in HBM (one batch = what 299 DRAM chains would hand ssfun at one step if each proposed
    K candidates): theta = a fixture chain state of the cell + N(0, J0) (the reference's proposal
    variances, TranscriptionCycleMCMC.m:217-231); rows outside the parameter box (:242-255) are
    inactive and not counted (mcmcstat rejects them without calling ssfun). Cycling through distinct
    batches keeps every launch's theta reads coming from memory, not from a cache warmed by the
    previous launch of the same batch."""

    def __init__(self, cells, K: int, rounds: int, seed: int, dev):
        import torch

        from transcriptioncycleinference_amd.data import DR_BOUNDS, LOWER, UPPER

        with np.load(os.path.join(ROOT, "tests", "golden", "chain_theta.npz"), allow_pickle=False) as f:
            z = {k: f[k] for k in f.files}
        C, lens = cells.n_cells, cells.lengths.astype(np.int64)
        ld = int(7 + lens.max())
        off = z["theta_offsets"]
        S = np.zeros((len(off) - 1, ld))
        for i in range(len(off) - 1):
            S[i, :off[i + 1] - off[i]] = z["theta"][off[i]:off[i + 1]]
        first = np.searchsorted(z["cell_id"], np.arange(C))            # rows are sorted by cell
        count = np.bincount(z["cell_id"], minlength=C)
        sd = np.zeros((C, ld))
        lo, hi = np.zeros((C, ld)), np.zeros((C, ld))
        for c in range(C):
            n = int(lens[c])
            t = cells.cell(c)[0]
            sd[c, :7 + n] = np.sqrt(np.concatenate([[0.05, 0.1, t[-1] - t[-2], 1.0, 1.0, 0.05, 0.5], np.full(n, 0.5)]))
            lo[c, :7], hi[c, :7] = LOWER, UPPER
            lo[c, 7:], hi[c, 7:] = DR_BOUNDS
        self.B, self.ld, self.K = C * K, ld, K
        cid = np.repeat(np.arange(C, dtype=np.int32), K)
        g = torch.Generator(device=dev)
        g.manual_seed(int(seed))
        S_d, sd_d = torch.from_numpy(S).to(dev), torch.from_numpy(sd).to(dev)
        lo_d, hi_d = torch.from_numpy(lo).to(dev), torch.from_numpy(hi).to(dev)
        cid_l = torch.from_numpy(cid.astype(np.int64)).to(dev)
        first_d, count_d = torch.from_numpy(first).to(dev), torch.from_numpy(count).to(dev)
        self.cid = torch.from_numpy(cid).to(dev)
        self.theta, self.active, self.n_active = [], [], []
        for _ in range(rounds):
            u = torch.rand(self.B, generator=g, device=dev, dtype=torch.float64)
            pick = first_d[cid_l] + torch.clamp((u * count_d[cid_l]).long(), max=int(count.max()) - 1)
            th = S_d[pick] + torch.randn(self.B, ld, generator=g, device=dev, dtype=torch.float64) * sd_d[cid_l]
            act = ((th >= lo_d[cid_l]) & (th <= hi_d[cid_l])).all(dim=1).to(torch.uint8)
            self.theta.append(th.contiguous())
            self.active.append(act)
            self.n_active.append(int(act.sum().item()))
        self.cid_host = cid
        self.out = torch.empty(self.B, dtype=torch.float64, device=dev)


def algorithmic_bytes(cells, cid, active) -> int:
    """per active eval theta 8*(7+N_c) + cell id 4; per row active flag 1 +
    SS write 8; per launch the cell data t/MS2/PP7 24*N_c once per cell."""
    lens = cells.lengths.astype(np.int64)
    act = active.astype(bool)
    per_active = (8 * (7 + lens[cid[act]]) + 4).sum()
    return int(per_active + 9 * len(cid) + 24 * lens.sum())


def load_pmc(workload: str) -> dict:
    """The committed rocprofv3 PMC summary of this workload's kernel (profiles/pmc_traffic.json,
    written by scripts/pmc_summary.py), or {} when there is none."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return d
    except (OSError, ValueError):
        pass
    return {}


def valu_issue(pmc: dict, kernel_ms: float):
    """VALU issue utilisation of the FP64 kernel from the committed PMC passes, priced per class:
    a wave64 FP64 instruction (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64) holds its SIMD for 4 cycles
    (78.6 TF/s FP64 = 1024 SIMDs x 16 lanes x 2 x 2.4 GHz), a 32-bit one for 2 (SIMD-32). The
    instructions in no class (moves, DPP moves, compares, selects, min/max) are priced at 2 cycles
    for `frac` and at 4 for `frac_high`. busy = issue cycles / (1024 SIMDs x 2.4 GHz x launch time)."""
    cnt = pmc.get("counters_mean_per_launch") or {}
    insts = cnt.get("SQ_INSTS_VALU")
    if not insts or kernel_ms <= 0:
        return None
    fp64 = sum(cnt.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS"))
    avail = SIMDS * CLOCK_HZ * kernel_ms * 1e-3
    out = {"valu_insts_per_launch": insts, "fp64_insts_per_launch": fp64 or None, "source": pmc.get("source"),
           "unit": "fraction of SIMD issue cycles"}
    if fp64:
        lo, hi = 4.0 * fp64 + 2.0 * (insts - fp64), 4.0 * insts
        out.update({"frac": lo / avail, "frac_high": hi / avail, "issue_cycles_per_launch": [lo, hi]})
    else:
        out.update({"frac_high": 4.0 * insts / avail})
    return out


def _cpu_rate(cells, cs, th, ci, ac, threads: int, seconds: float):
    from oracle import c_oracle  # cpu_baseline leg only

    n_act = int(ac.sum())
    evals, reps, t0 = 0, 0, time.perf_counter()
    while True:
        c_oracle.ss_batch(cells.offsets, cells.t, cells.ms2, cells.pp7, cs, th, ci, ac, nthreads=threads)
        evals += n_act
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return evals / el, evals, reps, el


def cpu_baseline(cells, theta, cid, active, seconds: float):
    """The C oracle (faithful matrix-form restatement, OpenMP over rows -- the parfor analogue)
    on the host cores, on a bounded sample of the same workload: every cell, its first proposals,
    enough rows to keep every thread busy. Reported at all host threads (the box's CPU share:
    OMP_NUM_THREADS) and at 1 core (BASELINE.md's CPU-baseline plan)."""
    from oracle import c_oracle, oracle as ref  # cpu_baseline leg only

    c_oracle.build()
    cs = ref.builtin_construct(CONSTRUCT)
    threads = c_oracle.max_threads()
    P = len(cid) // cells.n_cells
    per_cell = max(1, min(P, (threads * 8 + cells.n_cells - 1) // cells.n_cells))
    idx = np.concatenate([np.arange(c * P, c * P + per_cell) for c in range(cells.n_cells)])
    th, ci, ac = theta[idx], cid[idx], active[idx]
    rate, evals, reps, el = _cpu_rate(cells, cs, th, ci, ac, threads, seconds)
    one = np.arange(cells.n_cells) * per_cell          # one proposal per cell for the 1-core leg
    rate1, evals1, reps1, el1 = _cpu_rate(cells, cs, th[one], ci[one], ac[one], 1, seconds / 2)
    return {"value": rate, "unit": "SS evals/s", "cores": threads, "kind": "port",
            "sample": f"{len(idx)} rows ({per_cell} proposals x {cells.n_cells} cells, {int(ac.sum())} in-bounds) x "
                      f"{reps} passes = {evals} evals in {el:.1f} s; C matrix-form oracle (oracle/tci_oracle.c), "
                      f"OpenMP {threads} threads",
            "single_core": {"value": rate1, "unit": "SS evals/s", "cores": 1,
                            "sample": f"{len(one)} rows (1 proposal x {cells.n_cells} cells) x {reps1} passes = "
                                      f"{evals1} evals in {el1:.1f} s"}}


def end_to_end(lk, n_steps: int, seed: int, reduce=None):
    """SURVEY §8(d) mode (ii): the reference's whole fit -- one DRAM chain per TestData cell,
    n_steps (200k) steps, n_burn = n_steps/20, GPU-resident sampler (every ssfun evaluation runs
    inside the fused chain kernel). Reported beside `value` (a step there is one batched launch).
    With N ranks every rank fits its own replica (weak scaling, like `value`); `reduce(x, op)`
    combines over ranks: evals are summed, the wall time is the max."""
    from transcriptioncycleinference_amd.mcmc import fit

    t0 = time.perf_counter()
    fr = fit(lk, n_steps=n_steps, n_burn=max(1, n_steps // 20), seed=seed)
    wall = time.perf_counter() - t0
    roof = sampler_roofline(lk, n_steps=2000, label="TestData: ")   # untimed, after the fit
    dev_s, evals, chains = fr.elapsed_ms * 1e-3, int(fr.n_evals), len(fr.MCMCresults)
    if reduce is not None:
        dev_s, wall = reduce(dev_s, "max"), reduce(wall, "max")
        evals, chains = int(reduce(evals, "sum")), int(reduce(chains, "sum"))
    return {"n_steps": n_steps, "chains": chains, "device_s": dev_s, "wall_s": wall,
            "ssfun_evals": evals, "value": evals / wall, "unit": "SS evals/s (wall time, SURVEY §8(d)(ii))",
            "value_basis": "wall",
            "us_per_step": wall * 1e6 / max(n_steps - 1, 1),
            "device_value": evals / dev_s, "device_us_per_step": dev_s * 1e6 / max(n_steps - 1, 1),
            "accept_rate_median_rank0": float(np.median(fr.accept_rate)), "roofline_rank0": roof}


CONFIG_SHARDS = 8            # the 10,000 synthetic cells are 8 shards of 1,250
CONFIG_SHARD_CELLS = 1250


def config_shards(rank: int, world: int, n_shards: int = CONFIG_SHARDS) -> range:
    """The shards rank r of N builds and fits: a contiguous range of the fixed shards (every shard
    once over the ranks; with N > 8 some ranks get none). The dataset is the same at every N."""
    return range(rank * n_shards // world, (rank + 1) * n_shards // world)


def synthetic_config_cells(cfg: int, rank: int, world: int, device_index: int, n_points: int = 200,
                           shard_cells: int = CONFIG_SHARD_CELLS, n_shards: int = CONFIG_SHARDS):
    """this rank's shards of the 10,000 synthetic cells x 200 points
    (shard s: 1,250 cells from data seed 20201028 + s, independent of the GPU count) and the construct
    (config 5: 2 segments per dye, 3x length). Returns (cells, truth, construct, n_total, n_points,
    first cell, end cell) with the rank's cells at dataset-wide indices [first, end)."""
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.construct import builtin_construct, long_two_loop_construct
    from transcriptioncycleinference_amd.data import synthetic_cells

    construct = builtin_construct(CONSTRUCT) if cfg == 4 else long_two_loop_construct()
    n_total = shard_cells * n_shards
    mine = config_shards(rank, world, n_shards)
    lo, hi = mine.start * shard_cells, mine.stop * shard_cells

    def fwd(times, theta):
        nan = [np.full(len(t), np.nan) for t in times]
        tab = from_lists([(t, a, a) for t, a in zip(times, nan)])
        with Likelihood(tab, construct, device=device_index) as L:
            return L.forward(theta, np.arange(len(times), dtype=np.int32), grid="interp")

    parts, truths = [], []
    for s in mine:
        c, th = synthetic_cells(shard_cells, n_points, 20201028 + s, fwd)
        parts.append(c)
        truths.append(th)
    if not parts:
        return from_lists([], "synthetic-empty"), np.zeros((0, 7 + n_points)), construct, n_total, n_points, lo, hi
    cells = from_lists([p.cell(k) for p in parts for k in range(p.n_cells)],
                       f"synthetic-{n_total}x{n_points}-shards{mine.start}-{mine.stop - 1}")
    return cells, np.concatenate(truths), construct, n_total, n_points, lo, hi


def synthetic_kernel(cfg: int, rank: int, world: int, device_index: int, proposals: int, warmup: int, steps: int,
                     reduce):
    """SURVEY.md §8(d) configs 4/5 in kernel mode: 10,000 synthetic cells x 200 points in 8 fixed
    shards, this rank's shards on its GPU, `proposals` Gaussian proposals per cell around the ground
    truth with the reference's J0 variances (proposal seed 7 + shard; bounds-rejected rows inactive,
    not counted). Config 5 runs the 2-segment, 3x-length construct. Strong scaling: the total is fixed."""
    import torch

    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.data import DR_BOUNDS, LOWER, UPPER

    cells, truth, construct, n_total, n_points, lo, hi = synthetic_config_cells(cfg, rank, world, device_index)
    C, ld = truth.shape
    out = {"workload": f"config{cfg}: synthetic {n_total} cells x {n_points} points in {CONFIG_SHARDS} shards, "
                       f"{proposals} proposals/cell, construct {construct.name}, {hi - lo} cells on rank 0",
           "unit": "SS evals/s", "scaling": "strong"}
    n_act, kernel_ms, alg, ok, rpl = 0, 0.0, 0, True, None
    if C:
        cid = np.repeat(np.arange(C, dtype=np.int32), proposals)
        theta = np.empty((len(cid), ld))
        for k, s in enumerate(config_shards(rank, world)):  # proposals keyed by shard: N-independent
            rng = np.random.default_rng(7 + s)
            rows = slice(k * CONFIG_SHARD_CELLS * proposals, (k + 1) * CONFIG_SHARD_CELLS * proposals)
            theta[rows] = rng.normal(0.0, 1.0, (CONFIG_SHARD_CELLS * proposals, ld))
        dtl = np.array([cells.cell(c)[0][-1] - cells.cell(c)[0][-2] for c in range(C)])
        sd = np.sqrt(np.concatenate([np.tile([0.05, 0.1, 0.0, 1.0, 1.0, 0.05, 0.5], (C, 1)), np.full((C, ld - 7), 0.5)], 1))
        sd[:, 2] = np.sqrt(dtl)
        theta = truth[cid] + theta * sd[cid]
        active = np.all((theta[:, :7] >= LOWER) & (theta[:, :7] <= UPPER), axis=1)
        active &= np.all((theta[:, 7:] >= DR_BOUNDS[0]) & (theta[:, 7:] <= DR_BOUNDS[1]), axis=1)
        active = active.astype(np.uint8)
        dev = torch.device("cuda", device_index)
        lk = Likelihood(cells, construct, device=device_index)
        th_d, cid_d = torch.from_numpy(theta).to(dev), torch.from_numpy(cid).to(dev)
        act_d, out_d = torch.from_numpy(active).to(dev), torch.empty(len(cid), dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev)
        for _ in range(warmup):
            lk.ss_batch_device(th_d, cid_d, out_d, act_d, stream=stream)
        torch.cuda.synchronize(dev)
    reduce(0.0, "max")  # barrier
    t0 = time.perf_counter()
    if C:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            lk.ss_batch_device(th_d, cid_d, out_d, act_d, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
    elapsed = reduce(time.perf_counter() - t0, "max")
    if C:
        kernel_ms = e0.elapsed_time(e1) / steps
        ss = out_d.cpu().numpy()
        n_act = int(active.sum())
        alg = algorithmic_bytes(cells, cid, active)
        ok = bool(np.all(np.isfinite(ss[active.astype(bool)])))
        rpl = lk.info["rows_per_lane"]
        lk.close()
        out.update({"rows_per_launch_rank0": len(cid), "in_bounds_rank0": n_act})
    out.update({"value": reduce(n_act, "sum") * steps / elapsed, "kernel_ms_rank0": kernel_ms,
                "hbm_frac_rank0": alg / max(kernel_ms * 1e-3, 1e-30) / 1e9 / HBM_PEAK_GBS,
                "kernel_rows_per_lane": rpl, "results_finite": bool(reduce(0.0 if ok else 1.0, "sum") == 0.0)})
    return out


def synthetic_end_to_end(cfg: int, rank: int, world: int, device_index: int, n_steps: int, reduce,
                         engine: str = "auto", n_points: int = 200, coll_device: str = None,
                         shard_cells: int = CONFIG_SHARD_CELLS, n_shards: int = CONFIG_SHARDS):
    """SURVEY.md §8(d) configs 4/5 end to end, as `parallel.fit_sharded` runs a sharded fit: 10,000
    synthetic cells in 8 fixed shards, rank r fits its shards (one GPU-resident DRAM chain per cell,
    n_burn = n_steps/20, chains keyed by the dataset-wide cell index, so the fit is the same at every
    GPU count), then ONE all-gather of the packed per-cell results (RCCL over xGMI on a multi-GPU node)
    -- inside the timed region, and timed on its own too. Strong scaling: 10,000 cells in total.
    BASELINE configs 4/5 name n_steps = 200000 (the default); a smaller n_steps is labelled a sample.
    With more ranks than shards a rank holds no cells: it builds no context and fits nothing, but joins
    every collective (fit_sharded with lk=None)."""
    import contextlib

    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.mcmc import DramOptions
    from transcriptioncycleinference_amd.parallel import fit_sharded

    cells, _, construct, n_total, n_points, lo, hi = synthetic_config_cells(cfg, rank, world, device_index, n_points,
                                                                            shard_cells=shard_cells,
                                                                            n_shards=n_shards)
    with (Likelihood(cells, construct, device=device_index) if cells.n_cells else contextlib.nullcontext()) as lk:
        reduce(0.0, "max")  # barrier
        t0 = time.perf_counter()
        fr = fit_sharded(lk, device=coll_device, cell_offset=lo, n_steps=n_steps, n_burn=max(1, n_steps // 20),
                         seed=cfg, opts=DramOptions(engine=engine))
        wall = reduce(time.perf_counter() - t0, "max")
        # output checks (untimed): every gathered cell's summaries finite, every local final state finite,
        # and the GPU SS of a sample of this rank's final states, which the cpu_baseline leg re-evaluates
        # on the oracle
        ok = len(fr.MCMCresults) == n_total and [r["cell_index"] for r in fr.MCMCresults] == list(range(1, n_total + 1))
        ok = ok and bool(np.all([np.isfinite(r["mean_v"]) and np.isfinite(r["mean_sigma"]) and
                                 np.all(np.isfinite(r["mean_dR"])) for r in fr.MCMCresults]))
        loc = fr.local
        s_theta, s_cid, s_ss = np.zeros((0, 7 + n_points)), np.zeros(0, np.int32), np.zeros(0)
        if loc is not None:
            fin = loc.final_theta
            lens = cells.lengths[loc.cell_index - lo]
            ok = ok and all(np.all(np.isfinite(fin[k, :7 + n])) for k, n in enumerate(lens))
            sample = np.linspace(0, len(loc.cell_index) - 1, min(256, len(loc.cell_index))).astype(np.int64)
            s_theta = np.ascontiguousarray(fin[sample])
            s_cid = (loc.cell_index[sample] - lo).astype(np.int32)
            s_ss = lk.ss_batch(s_theta, s_cid)
            ok = ok and bool(np.all(np.isfinite(s_ss)))
        else:
            ok = ok and cells.n_cells == 0   # only a rank without cells has no local fit
        # untimed: the sampler kernels' roofline on this rank's chains (rank 0's in the line)
        roof = sampler_roofline(lk, cell_offset=lo, label=f"config{cfg} rank {rank}: ") if cells.n_cells else None
    dev_s = fr.elapsed_ms * 1e-3     # max over ranks (fit_sharded)
    evals = int(fr.n_evals)          # summed over ranks (fit_sharded)
    gather_s = reduce(fr.gather_s, "max")
    acc = float(np.median([r for r in fr.accept_rate])) if len(fr.accept_rate) else float("nan")
    out = {"workload": f"config{cfg}: synthetic {n_total} cells x {n_points} points in {n_shards} shards "
                       f"(seed 20201028 + shard), construct {construct.name}, {hi - lo} chains on rank 0, "
                       f"{n_steps} steps, results all-gathered" + ("" if n_steps >= 200000 else
                                                                    " (bounded sample of the configured 200k)"),
           "n_steps": n_steps, "engine": engine, "chains": len(fr.MCMCresults), "device_s": dev_s,
           "wall_s": wall, "ssfun_evals": evals, "value": evals / wall, "unit": "SS evals/s (wall time)",
           "value_basis": "wall",
           "scaling": "strong", "us_per_step": wall * 1e6 / max(n_steps - 1, 1),
           "device_value": evals / dev_s, "device_us_per_step": dev_s * 1e6 / max(n_steps - 1, 1),
           "gather_s": gather_s, "gather_bytes_per_rank": fr.gather_bytes,
           "gather_collective": "RCCL all-gather" if coll_device and str(coll_device).startswith("cuda") and world > 1
           else ("gloo all-gather" if world > 1 else "none (one rank)"),
           "accept_rate_median": acc,
           "outputs_finite": bool(reduce(0.0 if ok else 1.0, "sum") == 0.0),
           "roofline": roof}
    spot = {"cells": cells, "construct": construct, "theta": s_theta, "cid": s_cid, "ss_gpu": s_ss}
    return out, spot


def _tri_stride(ld: int) -> int:
    """Doubles per chain of the packed FP64 R (csrc/tci_dram_internal.h dram_tri_stride)."""
    return (ld * (ld + 1) // 2 + 127) // 128 * 128


def sampler_roofline(lk, cell_offset: int = 0, n_steps: int = 1000, seed: int = 9, label: str = ""):
    """Roofline of the sampler's three kernel classes: a short fit of every cell of
    ``lk`` (all chains of the timed fit, burn-in 100 rows so that every later window is a full covupd +
    Cholesky, as in 95 % of a 200k-step fit) with HIP events around each launch (tci_dram_options.
    kernel_times), and the ALGORITHMIC bytes / FLOP per launch of each class from the shapes:
      draws (k_draws): R read once per chain and launch (dram_tri_stride(ld) doubles) + every row's draws
        written, (2P + 4) doubles; FLOP: z*R for both stages, 2 x P(P+1) per row (upper-triangular matvec);
        the split form (k_chain's engine) reads the row's 2P normals too and writes 2P;
      walk (k_walk / k_chain): per row the draws row read ((2P + 4) doubles), the window-log row written (P
        doubles + s2 + the run flag), and the cell's data (24 N bytes) once per launch; no FLOP count (the
        SS evaluations are a dependent VALU chain); the split form's k_chain launch also
        writes the next chunk's normals and scalar draws, (2P + 4) doubles per row;
      adapt (k_adapt_*): per chain the window (adaptint rows of P doubles + run flags), the covariance tiles
        read and written (2 x NT(NT+1)/2 x 256 doubles), the means (3P doubles) and R written; FLOP: one
        symmetric rank-1 update per run of equal rows, P(P+1) each (runs ~ 1 + accept rate x adaptint),
        plus the Cholesky, P^3/3.
    Fractions of 8 TB/s and of the 78.6 TFLOP/s FP64 peak."""
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run, plan_fit

    cl = lk.cells
    plan = plan_fit(cl, list(range(cl.n_cells)), seed, cell_offset=cell_offset)
    n, ld = plan.x0.shape
    o = DramOptions(n_steps=n_steps, burnintime=100, adaptint=100, stats_from=1, seed=seed, kernel_times=True)
    r = dram_run(lk, np.array(plan.cells, np.int32), plan.x0, plan.lower, plan.upper, plan.prior_mu, plan.prior_sig,
                 plan.qcov_diag, 1.0, o, chain_keys=np.array(plan.cells, np.int64) + cell_offset)
    P = 7 + cl.lengths[plan.cells].astype(np.float64)
    N = cl.lengths[plan.cells].astype(np.float64)
    rows = n_steps - 1
    acc = float(np.mean(r.accept_rate))
    NT = np.ceil(P / 16)
    split = int(r.kernel_launches[3]) > 0  # the split draws (its first-chunk launch is class 3)
    out = {"workload": f"{label}{n} chains, {n_steps} steps (burn-in 100, adaptint 100), HIP events per launch",
           "peaks": {"hbm_GBs": HBM_PEAK_GBS, "fp64_TFs": FP64_PEAK_TFS}, "accept_rate_mean": acc,
           "split_draws": split}
    names = ("draws", "walk", "adapt")
    for k, name in enumerate(names):
        launches = int(r.kernel_launches[k])
        if launches == 0:
            continue
        us = float(r.kernel_ms[k]) * 1e3 / launches
        if name == "draws":
            byts = (8 * _tri_stride(ld) * n * launches + rows * 8 * ((4 * P) if split else (2 * P + 4)).sum()) / launches
            flop = rows * 2 * (P * (P + 1)).sum() / launches
        elif name == "walk":
            per_row = 8 * (2 * P + 4) + 8 * P + 9 + (8 * (2 * P + 4) if split else 0)
            byts = (rows * per_row.sum() + launches * 24 * N.sum()) / launches
            flop = None
        else:
            runs = 1 + acc * 100
            byts = (100 * 8 * P + 100 + 2 * 8 * 256 * NT * (NT + 1) / 2 + 3 * 8 * P + 8 * P * (P + 1) / 2).sum()
            flop = (runs * P * (P + 1) + P ** 3 / 3).sum()
        d = {"launches": launches, "avg_us": us, "alg_bytes_per_launch": float(byts),
             "achieved_GBs": float(byts) / (us * 1e-6) / 1e9}
        d["hbm_frac"] = d["achieved_GBs"] / HBM_PEAK_GBS
        if flop is not None:
            d["alg_flop_per_launch"] = float(flop)
            d["achieved_TFs"] = float(flop) / (us * 1e-6) / 1e12
            d["fp64_frac"] = d["achieved_TFs"] / FP64_PEAK_TFS
        d["bound"] = ("fp64" if flop is not None and d["fp64_frac"] > d["hbm_frac"] else "hbm")
        out[name] = d
    return out


def cpu_baseline_synth(cfg: int, spot: dict, seconds: float):
    """cpu_baseline leg on a BASELINE config-4/5 workload (BASELINE.md CPU plan): the C
    oracle on the host cores (all threads, then 1 core) over a sample of the 10,000-chain fit's final
    states (one row per sampled chain), which doubles as the oracle spot check of that fit's
    outputs: the GPU SS of the same rows (synthetic_end_to_end) against the oracle's."""
    from oracle import c_oracle  # cpu_baseline leg only

    cells, cs = spot["cells"], spot["construct"]
    th, ci = spot["theta"], spot["cid"]
    if len(ci) == 0:  # rank 0 holds no shard (more ranks than shards)
        return {"value": None, "unit": "SS evals/s", "kind": "port", "sample": "none: rank 0 fitted no cells"}
    c_oracle.build()
    ac = np.ones(len(ci), np.uint8)
    threads = c_oracle.max_threads()
    want, st = c_oracle.ss_batch(cells.offsets, cells.t, cells.ms2, cells.pp7, cs, th, ci)
    rel = float(np.max(np.abs(spot["ss_gpu"] - want) / np.maximum(np.abs(want), 1e-300))) if np.all(st == 0) \
        else float("nan")
    rate, evals, reps, el = _cpu_rate(cells, cs, th, ci, ac, threads, seconds)
    one = np.arange(min(len(ci), 64))
    rate1, evals1, reps1, el1 = _cpu_rate(cells, cs, th[one], ci[one], ac[one], 1, seconds / 2)
    return {"value": rate, "unit": "SS evals/s", "cores": threads, "kind": "port",
            "sample": f"config{cfg}: {len(ci)} final chain states of the DRAM fit x {reps} passes = {evals} evals in "
                      f"{el:.1f} s; C matrix-form oracle, OpenMP {threads} threads",
            "single_core": {"value": rate1, "unit": "SS evals/s", "cores": 1,
                            "sample": f"{len(one)} rows x {reps1} passes = {evals1} evals in {el1:.1f} s"},
            "oracle_spot_check": {"rows": int(len(ci)), "max_rel_err_gpu_vs_oracle": rel,
                                  "ok": bool(rel <= 1e-6), "tolerance": 1e-6}}


def cpu_fit_config1(lk, n_steps: int = 10000, n_burn: int = 1000, seed: int = 1):
    """BASELINE config 1 as written: TestData cell 1, n_steps = 10,000,
    n_burn = 1,000, fitted on the host -- mcmcstat's DRAM restated in C with the C oracle as ssfun
    (oracle/tci_dram_oracle.c, one chain, one core: mcmcstat's loop is serial) -- the CPU counterpart
    of mode (ii). The same cell is fitted on the GPU with the same inputs (x0, bounds, J0, seed, RNG
    streams: mcmc.fit), and the posterior summaries of v and R are compared: the two samplers take
    the same decisions on the same streams, so they agree far inside the posterior sd."""
    from oracle import c_oracle, oracle as ref  # cpu_baseline leg only
    from transcriptioncycleinference_amd.mcmc import DramOptions, fit, plan_fit

    c_oracle.build()
    cell = 0
    g0 = time.perf_counter()
    fr = fit(lk, n_steps=n_steps, n_burn=n_burn, seed=seed, cells=[cell])
    g_wall = time.perf_counter() - g0
    plan = plan_fit(lk.cells, [cell], seed)
    o = DramOptions(n_steps=n_steps, burnintime=n_burn, stats_from=max(n_burn, 1), seed=seed * 1000003 + 20201028)
    t0 = time.perf_counter()
    r = c_oracle.dram_run(lk.cells, ref.builtin_construct(CONSTRUCT), np.array(plan.cells, np.int32), plan.x0,
                          plan.lower, plan.upper, plan.prior_mu, plan.prior_sig, plan.qcov_diag, 1.0, o,
                          keys=np.array(plan.cells, np.int64), nthreads=1)
    wall = time.perf_counter() - t0
    evals = int(r["n_evals"][0])
    g = fr.MCMCresults[0]
    cmp = {}
    for name, j in (("v", 0), ("R", 6)):
        mc, sc, mg, sg = float(r["mean"][0, j]), float(r["std"][0, j]), g["mean_" + name], g["sigma_" + name]
        cmp[name] = {"cpu_mean": mc, "gpu_mean": mg, "cpu_sd": sc, "gpu_sd": sg,
                     "mean_diff_in_sd": abs(mc - mg) / max(sc, 1e-300), "sd_rel_diff": abs(sc - sg) / max(sc, 1e-300)}
    ok = all(c["mean_diff_in_sd"] < 3.0 and c["sd_rel_diff"] < 0.5 for c in cmp.values())
    return {"value": evals / wall, "unit": "SS evals/s (wall time, one chain)", "cores": 1, "kind": "port",
            "sample": f"BASELINE config 1 in full: TestData cell 1, {n_steps} steps, n_burn {n_burn}, {evals} ssfun "
                      f"evals in {wall:.2f} s; mcmcstat's DRAM restated in C (oracle/tci_dram_oracle.c) with the C "
                      f"matrix-form oracle as ssfun, one core",
            "us_per_step": wall * 1e6 / max(n_steps - 1, 1), "wall_s": wall,
            "gpu_same_fit": {"wall_s": g_wall, "us_per_step": g_wall * 1e6 / max(n_steps - 1, 1),
                             "ssfun_evals": int(fr.n_evals), "note": "one chain on the GPU: latency-bound, the "
                             "GPU's throughput needs many chains (end_to_end_dram)"},
            "posterior_check": cmp, "posterior_check_ok": bool(ok)}


def hierarchical_end_to_end(lk, n_steps: int, seed: int, reduce):
    """the 299-cell fit with loadPrevious, v fixed to v0 +- 1e-5 (proposal
    variance 1e-7, TranscriptionCycleMCMC.m:218,236-237), v0 = the reference's MCMCresults.mean_v
    (28-Oct-2020-TestData.mat, committed in tests/golden/forward_means.npz)."""
    from transcriptioncycleinference_amd.mcmc import fit

    with np.load(os.path.join(ROOT, "tests", "golden", "forward_means.npz"), allow_pickle=False) as f:
        th, off = f["theta"], f["theta_offsets"]
    v0 = [float(th[off[c]]) for c in range(len(off) - 1)]
    t0 = time.perf_counter()
    fr = fit(lk, n_steps=n_steps, n_burn=max(1, n_steps // 20), seed=seed, v0=v0)
    wall = reduce(time.perf_counter() - t0, "max")
    dev_s, evals = reduce(fr.elapsed_ms * 1e-3, "max"), int(reduce(fr.n_evals, "sum"))
    return {"n_steps": n_steps, "chains": int(reduce(len(fr.MCMCresults), "sum")), "device_s": dev_s, "wall_s": wall,
            "ssfun_evals": evals, "value": evals / wall, "unit": "SS evals/s (wall time)", "value_basis": "wall",
            "us_per_step": wall * 1e6 / max(n_steps - 1, 1),
            "device_value": evals / dev_s, "device_us_per_step": dev_s * 1e6 / max(n_steps - 1, 1),
            "v_fixed": bool(all(abs(r["mean_v"] - v0[int(r["cell_index"]) - 1]) <= 1e-5 + 1e-12
                                for r in fr.MCMCresults))}


def kernel_mode(lk, rounds: ProposalRounds, launches: int, stream, sync_ranks=None):
    """``launches`` back-to-back batched launches cycling over the resident proposal rounds, timed
    with HIP events on the launch stream (per-launch kernel time) and the wall clock (whole job).
    Returns (wall seconds, kernel ms per launch, in-bounds evals)."""
    import torch

    R = len(rounds.theta)
    torch.cuda.synchronize()
    if sync_ranks:
        sync_ranks()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for i in range(launches):
        r = i % R
        lk.ss_batch_device(rounds.theta[r], rounds.cid, rounds.out, rounds.active[r], stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    if sync_ranks:
        sync_ranks()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    evals = sum(rounds.n_active[i % R] for i in range(launches))
    return wall, e0.elapsed_time(e1) / launches, evals


def rounds_algorithmic_bytes(cells, rounds: ProposalRounds) -> float:
    """Mean algorithmic bytes per launch over the rounds (see algorithmic_bytes)."""
    return float(np.mean([algorithmic_bytes(cells, rounds.cid_host, a.cpu().numpy()) for a in rounds.active]))


def kernel_sweep(lk, cells, dev, stream, seed: int, Ks=(1, 64, 256, 1024), target_s: float = 0.05):
    """kernel throughput at K proposals per cell per launch (B = 299 K rows).
    K = 1 is the reference's own per-step batch (one ssfun per parfor cell)."""
    out = []
    for K in Ks:
        rounds = ProposalRounds(cells, K, 4, seed + K, dev)
        kernel_mode(lk, rounds, 4, stream)                                  # warm-up
        _, ms, _ = kernel_mode(lk, rounds, 8, stream)
        n = int(max(16, min(20000, target_s / max(ms * 1e-3, 1e-7))))
        wall, ms, evals = kernel_mode(lk, rounds, n, stream)
        alg = rounds_algorithmic_bytes(cells, rounds)
        ach = alg / (ms * 1e-3) / 1e9
        out.append({"K": K, "rows_per_launch": rounds.B, "in_bounds_per_launch": float(np.mean(rounds.n_active)),
                    "launches": n, "kernel_us": ms * 1e3, "value": evals / wall, "unit": "SS evals/s",
                    "kernel_evals_per_s": float(np.mean(rounds.n_active)) / (ms * 1e-3),
                    "algorithmic_bytes_per_launch": alg, "achieved_GBs": ach, "hbm_frac": ach / HBM_PEAK_GBS})
        del rounds
    return out


def x0_theta_kernel(lk, cells, dev, stream, K: int = 256, seed: int = 1, target_s: float = 0.1):
    """SURVEY §8(d)(6) kernel-mode theta set: every row drawn from the reference's initial-state
    distribution (TranscriptionCycleMCMC.m:200-210: v ~ 1+2U, ton ~ 4U, A ~ U, tau ~ 4U, MS2_basal 10,
    PP7_basal 5, R 15, dR ~ N(0, 3)), numpy seed 1, K rows per cell (all inside the box, so all
    counted). The same kernel as `value`; only the theta distribution differs."""
    import torch

    rng = np.random.default_rng(seed)
    C, lens = cells.n_cells, cells.lengths.astype(np.int64)
    ld = int(7 + lens.max())
    theta = np.zeros((C * K, ld))
    for c in range(C):
        n = int(lens[c])
        u = rng.random((K, 4))
        blk = theta[c * K:(c + 1) * K]
        blk[:, 0], blk[:, 2], blk[:, 5], blk[:, 1] = 1 + 2 * u[:, 0], 4 * u[:, 1], u[:, 2], 4 * u[:, 3]
        blk[:, 3], blk[:, 4], blk[:, 6] = 10.0, 5.0, 15.0
        blk[:, 7:7 + n] = rng.normal(0.0, 3.0, (K, n))
    cid = np.repeat(np.arange(C, dtype=np.int32), K)
    act = np.ones(C * K, np.uint8)
    th_d, cid_d = torch.from_numpy(theta).to(dev), torch.from_numpy(cid).to(dev)
    act_d, out_d = torch.from_numpy(act).to(dev), torch.empty(C * K, dtype=torch.float64, device=dev)
    for _ in range(8):
        lk.ss_batch_device(th_d, cid_d, out_d, act_d, stream=stream)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 64
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(n):
        lk.ss_batch_device(th_d, cid_d, out_d, act_d, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / n
    ss = out_d.cpu().numpy()
    alg = algorithmic_bytes(cells, cid, act)
    return {"workload": f"TestData-299cells-x{K}-x0-distribution-theta (seed {seed})", "rows_per_launch": C * K,
            "in_bounds_per_launch": C * K, "kernel_us": ms * 1e3, "value": C * K * n / wall, "unit": "SS evals/s",
            "kernel_evals_per_s": C * K / (ms * 1e-3), "algorithmic_bytes_per_launch": alg,
            "hbm_frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "results_finite": bool(np.all(np.isfinite(ss)))}


def drop_in_latency(lk, cells, theta, cid, calls: int = 2000):
    """Per-call latency of the literal drop-in: ``tci_ssfun`` (one ssfun(theta, data) with its H2D
    copy, launch, D2H copy and synchronisation -- what mcmcstat's DRAM loop calls once or twice per
    step, TranscriptionCycleMCMC.m:186,258), and ``tci_ss_batch`` on host pointers with one row per
    cell (the lockstep driver's per-step call for all 299 chains, K = 1)."""
    rows = [np.ascontiguousarray(theta[np.nonzero(cid == c)[0][0], :7 + int(cells.lengths[c])]) for c in range(8)]
    for k in range(50):
        lk.ssfun(rows[k % 8], k % 8)
    t0 = time.perf_counter()
    for k in range(calls):
        lk.ssfun(rows[k % 8], k % 8)
    one = (time.perf_counter() - t0) / calls
    first = np.array([np.nonzero(cid == c)[0][0] for c in range(cells.n_cells)])
    th, ci = np.ascontiguousarray(theta[first]), np.ascontiguousarray(cid[first])
    for _ in range(20):
        lk.ss_batch(th, ci)
    n_b = max(200, calls // 4)
    t0 = time.perf_counter()
    for _ in range(n_b):
        lk.ss_batch(th, ci)
    batch = (time.perf_counter() - t0) / n_b
    return {"tci_ssfun_us_per_call": one * 1e6, "tci_ssfun_calls_per_s": 1.0 / one,
            "ss_batch_299_rows_us_per_call": batch * 1e6, "ss_batch_299_rows_evals_per_s": cells.n_cells / batch,
            "note": "host pointers, synchronous, PCIe round trip included; Python ctypes call overhead included"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--proposals", type=int, default=256, help="DRAM-style proposals per cell per launch (K)")
    ap.add_argument("--launches-per-step", type=int, default=128,
                    help="batched launches per step: one step = this many lockstep proposal rounds")
    ap.add_argument("--distinct-rounds", type=int, default=8, help="distinct resident proposal batches cycled")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true", help="skip the K in {1, 64, 256, 1024} kernel sweep")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the drop-in latency and host-pointer legs (profiling runs: only the K launch)")
    ap.add_argument("--dram-steps", type=int, default=200000,
                    help="end-to-end mode: one DRAM chain per TestData cell for this many steps (0 = skip)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other BASELINE configs (3: hierarchical fit; 4/5: 10k synthetic cells)")
    ap.add_argument("--synth-dram-steps", type=int, default=200000,
                    help="configs 4/5 end to end: DRAM steps of the 10,000-chain fit (BASELINE: 200k; 0 = skip)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    # Rehearsal switch (never used by the driver): several ranks on ONE GPU over gloo.
    rehearsal = os.environ.get("TCI_BENCH_REHEARSAL") == "1"
    device_index = 0 if rehearsal else local
    backend = "gloo" if rehearsal else "nccl"  # "nccl" is RCCL on ROCm
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(device_index)
        if backend == "nccl":
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=torch.device("cuda", device_index))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    if not rehearsal and local >= visible_devices():
        print(f"bench.py: rank {rank} has LOCAL_RANK {local} but only {visible_devices()} GPU(s) are visible",
              file=sys.stderr)
        sys.exit(2)
    dev = torch.device("cuda", device_index)
    torch.cuda.set_device(dev)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    ident = dict(device_identity(device_index), rank=rank, local_rank=local)
    if distributed:
        idents = [None] * world
        dist.all_gather_object(idents, ident)
        pcis = [d["pci"] for d in idents]
        if not rehearsal and len(set(pcis)) != world:
            raise RuntimeError(f"bench.py: {world} ranks share {len(set(pcis))} GPU(s): {pcis}")
    else:
        idents = [ident]

    def reduce(x, op):
        if not distributed:
            return x
        t = torch.tensor([float(x)], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return float(t.item())

    barrier = dist.barrier if distributed else None

    from transcriptioncycleinference_amd import Likelihood, testdata

    cells = testdata()
    lk = Likelihood(cells, CONSTRUCT, device=device_index)
    stream = torch.cuda.current_stream(dev)
    rounds = ProposalRounds(cells, args.proposals, args.distinct_rounds, 20201028 + rank, dev)
    L = args.launches_per_step
    kernel_mode(lk, rounds, max(1, args.warmup) * L, stream)                         # untimed warm-up steps
    wall, kernel_ms, evals = kernel_mode(lk, rounds, args.steps * L, stream, sync_ranks=barrier)
    elapsed = reduce(wall, "max")
    total_active = int(reduce(evals, "sum"))
    ss = rounds.out.cpu().numpy()
    act_last = rounds.active[(args.steps * L - 1) % len(rounds.theta)].cpu().numpy().astype(bool)
    finite_ok = bool(np.all(np.isfinite(ss[act_last])))
    if distributed:
        # the one results collective: per-cell SS of the last proposal of every cell (RCCL)
        from transcriptioncycleinference_amd.parallel import gather_rows

        per_cell = ss.reshape(cells.n_cells, -1)[:, -1].copy()
        gathered = gather_rows(per_cell, device=str(coll_dev))
        assert len(gathered) == cells.n_cells * world

    workload = f"TestData-299cells-x{args.proposals}proposals"
    alg = rounds_algorithmic_bytes(cells, rounds)
    achieved = alg / (kernel_ms * 1e-3) / 1e9
    pmc = load_pmc(workload)
    traffic = pmc.get("hbm_bytes_per_launch")
    res = {
        "metric": "forward-model SS evals/sec, 299-cell TestData, 200k-step chains @1/2/4/8 GPU",
        "value": total_active / elapsed,
        "unit": "SS evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "reference TestData.mat (299 cells) + synthetic DRAM-style proposals around the fixture chain states",
        "config": {
            "workload": workload,
            "step": f"{L} batched launches, each one lockstep round of {args.proposals} proposals for each of the "
                    f"{cells.n_cells} cells ({args.distinct_rounds} distinct resident proposal batches cycled)",
            "cells_per_gpu": cells.n_cells,
            "proposals_per_cell": args.proposals,
            "launches_per_step": L,
            "rows_per_launch_per_gpu": rounds.B,
            "in_bounds_evals_per_launch_per_gpu": float(np.mean(rounds.n_active)),
            "timed_region_s": elapsed,
            "construct": CONSTRUCT,
            "parallelism": f"replica-per-gpu x{world} (cells independent" + (
                f"; 1 {'RCCL' if backend == 'nccl' else 'gloo'} gather after timing)" if distributed else ")"),
            "launcher": os.environ.get("TCI_BENCH_LAUNCHER") or ("torch.distributed.run" if distributed else "none"),
            "kernel_rows_per_lane": lk.info["rows_per_lane"],
            "devices": idents,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel_ms": kernel_ms,
            "algorithmic_bytes_per_launch": alg,
            "note": "FP64 path bound by each wave's dependent chain under issue contention, no unit saturated "
                    "(see 'valu'; DESIGN.md §3); HBM fraction reported as the north star asks",
            "valu": valu_issue(pmc, kernel_ms),
        },
        "results_finite": finite_ok,
    }
    if not args.no_sweep:
        res["kernel_sweep"] = kernel_sweep(lk, cells, dev, stream, seed=77 + rank)
        res["kernel_x0_theta"] = x0_theta_kernel(lk, cells, dev, stream)
    theta_h = rounds.theta[0].cpu().numpy()
    act_h = rounds.active[0].cpu().numpy()
    if rank == 0 and world == 1 and not args.no_latency:
        res["drop_in_latency"] = drop_in_latency(lk, cells, theta_h, rounds.cid_host)
        # PCIe-inclusive rate of the host-pointer entry point for the whole K-proposal batch
        # (theta H2D + SS D2H per call): reported beside, never as, `value`.
        lk.ss_batch(theta_h, rounds.cid_host, act_h)
        h0 = time.perf_counter()
        for _ in range(5):
            lk.ss_batch(theta_h, rounds.cid_host, act_h)
        h_el = (time.perf_counter() - h0) / 5
        res["host_api_pcie_inclusive"] = {"value": int(act_h.sum()) / h_el, "unit": "SS evals/s",
                                          "ms_per_call": h_el * 1e3, "bytes_h2d": int(theta_h.nbytes + rounds.B * 5)}
    del rounds
    if args.dram_steps > 1:
        if distributed:
            dist.barrier()
        e2e = end_to_end(lk, args.dram_steps, seed=1 + rank, reduce=reduce)
        e2e["workload"] = (f"the metric's named workload (BASELINE config 2): 299-cell TestData, one GPU-resident DRAM "
                           f"chain per cell, {args.dram_steps} steps, every ssfun evaluation counted")
        res["end_to_end_dram"] = e2e
        if not args.no_configs:
            res["config3_hierarchical_dram"] = hierarchical_end_to_end(lk, args.dram_steps, seed=3 + rank, reduce=reduce)
    spots = {}
    if not args.no_configs:
        for cfg in (4, 5):
            res[f"config{cfg}_kernel"] = synthetic_kernel(cfg, rank, world, device_index, 8, args.warmup,
                                                          max(args.steps, 20), reduce)
            if args.synth_dram_steps > 1:
                res[f"config{cfg}_dram"], spots[cfg] = synthetic_end_to_end(cfg, rank, world, device_index,
                                                                            args.synth_dram_steps, reduce,
                                                                            coll_device=str(coll_dev))
    if distributed:
        dist.barrier()   # every GPU leg of every rank is done before the host cores are timed
    cpu_legs(res, rank, world, args, cells, theta_h, act_h, lk, spots)
    if rank == 0:
        print(json.dumps(res), flush=True)
    lk.close()
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def cpu_legs(res: dict, rank: int, world: int, args, cells, theta_h, act_h, lk, spots: dict):
    """The CPU baselines beside the GPU numbers (BASELINE.md CPU plan), at EVERY world
    size: on rank 0 only, after the last GPU leg of every rank (the caller's barrier), on the host
    cores of the GPU box; the other ranks wait in the final barrier. With N ranks on one node the N
    processes share those cores, which the `host` entry states."""
    if rank != 0 or args.no_cpu_baseline:
        return
    host = {"os_cpu_count": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "ranks_on_this_host": world,
            "note": "rank 0 times the CPU path after every rank's GPU legs; the other ranks idle in a barrier"
            if world > 1 else "one rank"}
    res["cpu_baseline"] = cpu_baseline(cells, theta_h, rounds_cid(cells, args.proposals), act_h, args.cpu_seconds)
    res["cpu_baseline"]["host"] = host
    res["cpu_fit_config1"] = cpu_fit_config1(lk)
    for cfg, spot in spots.items():
        res[f"cpu_baseline_config{cfg}"] = cpu_baseline_synth(cfg, spot, args.cpu_seconds / 2)


def rounds_cid(cells, K: int) -> np.ndarray:
    return np.repeat(np.arange(cells.n_cells, dtype=np.int32), K)


# ---------------------------------------------------------------------------
# --gpus N without a launcher: one child process per GPU (the reference's parfor workers,
# TranscriptionCycleMCMC.m:161), spawned before anything touches the GPU
# ---------------------------------------------------------------------------


class LaunchError(ValueError):
    pass


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_devices() -> int:
    """GPUs this process may use, counted WITHOUT initialising the GPU (torch.cuda.device_count()
    reads the device list without creating a HIP context on this image), so the parent can refuse
    a --gpus N it cannot honour before any child touches a GPU."""
    forced = os.environ.get("TCI_BENCH_DEVICES")  # CPU tests of the launcher only
    if forced:
        return int(forced)
    import torch

    return int(torch.cuda.device_count())


def check_devices(gpus: int, visible: int, rehearsal: bool):
    """A run on N GPUs needs N visible devices (one rank per GPU); the one-GPU rehearsal needs 1.
    Raises LaunchError instead of silently running several ranks on one device."""
    need = 1 if rehearsal else gpus
    if visible < need:
        raise LaunchError(f"--gpus {gpus} needs {need} visible GPU(s), found {visible} "
                          f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES', '<unset>')})")


def device_identity(device_index: int) -> dict:
    """This rank's device as the driver's record can check it: PCI domain:bus:device and name."""
    import torch

    pr = torch.cuda.get_device_properties(device_index)
    return {"device_index": device_index, "pci": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}",
            "name": pr.name, "gcn_arch": getattr(pr, "gcnArchName", "")}


def launch_plan(gpus: int, env: dict, port: int = 0):
    """How this invocation runs. None: in this process (a launcher such as torch.distributed.run set
    WORLD_SIZE, or one GPU). Otherwise one environment per rank for ``gpus`` child processes:
    RANK = LOCAL_RANK = r, WORLD_SIZE = gpus, rendezvous on 127.0.0.1. An inherited WORLD_SIZE that
    disagrees with --gpus is an error (LaunchError), never silently the smaller run."""
    if gpus < 1:
        raise LaunchError(f"--gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is not None and ws != "":
        if int(ws) != gpus:
            raise LaunchError(f"--gpus {gpus} disagrees with the launcher's WORLD_SIZE={ws}")
        return None
    if gpus == 1:
        return None
    port = port or _free_port()
    return [dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TCI_BENCH_LAUNCHER="bench.py --gpus")
            for r in range(gpus)]


def run_ranks(plan, argv) -> int:
    """Start one child per rank (this parent never touches the GPU) and wait for all of them. Rank 0
    prints the JSON line on the inherited stdout. If a rank fails, the others are stopped (their
    collectives would wait forever) and its exit status is returned."""
    import subprocess

    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=e) for e in plan]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                r = p.poll()
                if r is None:
                    continue
                procs.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in procs:
                        q.terminate()
            time.sleep(0.2)
    finally:
        for q in procs:
            q.kill()
    return rc


def entry() -> int:
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    known, _ = ap.parse_known_args()
    try:
        plan = launch_plan(known.gpus, dict(os.environ))
        if not {"-h", "--help"} & set(sys.argv[1:]) and (plan is not None or int(os.environ.get("WORLD_SIZE", "1")) == 1):
            # the parent (or a lone process) refuses before anything initialises a GPU; a rank
            # started by an outside launcher checks its own LOCAL_RANK in main()
            check_devices(known.gpus, visible_devices(), os.environ.get("TCI_BENCH_REHEARSAL") == "1")
    except LaunchError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        return 2
    if plan is not None:
        return run_ranks(plan, sys.argv[1:])
    main()
    return 0


if __name__ == "__main__":
    sys.exit(entry())
