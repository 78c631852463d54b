"""GPU-resident batched DRAM -- statistical and structural checks (MI355X).

Chain-level parity with MATLAB is impossible (mcmcstat is unpinned and MATLAB's RNG cannot be
reproduced); what is checked instead:
* the sigma^2 Gibbs draw obeys the same law the reference's fixtures pin
  (s2 * N / SS(theta) has mean N/(N-2), sd sqrt(2/N), as in tests/test_oracle_golden.py);
* determinism per seed, bounds (incl. the hierarchical fixed-v fit), bookkeeping (n_steps=1);
* recovery of ground truth on synthetic cells; the reference's output structs round-trip.
"""
import dataclasses

import numpy as np
import pytest

from conftest import pack

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lk(cells):
    from transcriptioncycleinference_amd import Likelihood

    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4", device=0) as L:
        yield L


def setup_rows(cells, ids, seed=0, v0=None):
    from transcriptioncycleinference_amd.mcmc import cell_setup

    rng = np.random.default_rng(seed)
    rows = [cell_setup(cells.cell(c)[0], rng, 50.0, None if v0 is None else v0[k]) for k, c in enumerate(ids)]
    ld = max(len(r[0]) for r in rows)
    out = []
    for i, fill in enumerate((0.0, -np.inf, np.inf, 0.0, np.inf, 1.0)):
        a = np.full((len(rows), ld), fill)
        for k, r in enumerate(rows):
            a[k, :len(r[i])] = r[i]
        out.append(a)
    return out


def run(lk, ids, opts, seed=0, v0=None):
    from transcriptioncycleinference_amd.mcmc import dram_run

    x0, lo, hi, mu, sg, J0 = setup_rows(lk.cells, ids, seed, v0)
    return dram_run(lk, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, opts), (x0, lo, hi)


def test_single_row_chain_is_the_initial_state(lk):
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(8))
    res, (x0, _, _) = run(lk, ids, DramOptions(n_steps=1, stats_from=1, thin=1))
    n = lk.cells.lengths[ids]
    for k in range(len(ids)):
        np.testing.assert_array_equal(res.mean[k, :7 + n[k]], x0[k, :7 + n[k]])
        assert np.all(res.std[k, :7 + n[k]] == 0)
    assert np.all(res.sigma_mean == 1.0) and np.all(res.n_evals == 1)
    np.testing.assert_array_equal(res.chain[0], x0)


def test_deterministic_per_seed(lk):
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(0, 299, 13))
    o = DramOptions(n_steps=400, burnintime=200, stats_from=100, thin=50, seed=7)
    a, _ = run(lk, ids, o)
    b, _ = run(lk, ids, o)
    np.testing.assert_array_equal(a.mean, b.mean)
    np.testing.assert_array_equal(a.chain, b.chain)
    o.seed = 8
    c, _ = run(lk, ids, o)
    assert not np.array_equal(a.mean, c.mean)


def test_chain_stays_in_bounds_and_moves(lk):
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(0, 299, 7))
    res, (x0, lo, hi) = run(lk, ids, DramOptions(n_steps=600, burnintime=300, stats_from=300, thin=1, seed=3))
    n = lk.cells.lengths[ids]
    for k in range(len(ids)):
        P = 7 + n[k]
        rows = res.chain[:, k, :P]
        assert np.all(rows >= lo[k, :P]) and np.all(rows <= hi[k, :P])
    assert np.all(res.accept_rate > 0.02) and np.all(res.accept_rate < 0.95), res.accept_rate
    # every accepted move changes the state; the row-to-row change count matches accept_rate
    moved = np.any(res.chain[1:] != res.chain[:-1], axis=2).mean(axis=0)
    np.testing.assert_allclose(moved, res.accept_rate, atol=1e-12)
    # ssfun is called once at start and once per in-bounds proposal (at most 2 per step)
    assert np.all(res.n_evals >= 1 + res.accept_rate * 599 - 1e-9) and np.all(res.n_evals <= 1 + 2 * 599)


def test_hierarchical_fit_keeps_v_fixed(lk):
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(10))
    v0 = [1.0 + 0.2 * k for k in range(10)]
    res, _ = run(lk, ids, DramOptions(n_steps=400, burnintime=200, stats_from=1, thin=1, seed=5), v0=v0)
    v = res.chain[:, :, 0]
    assert np.all(np.abs(v - np.array(v0)[None, :]) <= 1e-5 + 1e-12)


def test_sigma2_gibbs_law_matches_the_reference_fixture_statistic(lk):
    """1/s2 ~ Gamma(N/2, 2/SS(theta)): s2 * N / SS has mean N/(N-2) and sd sqrt(2/N) (N = 2 N_c)."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(0, 299, 3))
    res, _ = run(lk, ids, DramOptions(n_steps=1000, burnintime=500, stats_from=500, thin=5, seed=11))
    n = lk.cells.lengths[ids]
    rows, cid, s2, nobs = [], [], [], []
    for r in range(1, res.chain.shape[0]):  # skip row 1 (sigma2_0 is not a Gibbs draw)
        for k, c in enumerate(ids):
            rows.append(res.chain[r, k, :7 + n[k]])
            cid.append(c)
            s2.append(res.s2chain[r, k])
            nobs.append(2 * n[k])
    ss = lk.ss_batch(pack(rows), np.array(cid, np.int32))
    ratio = np.array(s2) * np.array(nobs) / ss
    nobs = np.array(nobs, np.float64)
    assert abs(ratio.mean() - np.mean(nobs / (nobs - 2))) < 0.01, ratio.mean()
    assert abs(ratio.std() - np.mean(np.sqrt(2 / nobs))) < 0.01, ratio.std()


def _synthetic(n_cells, n_points, noise, seed):
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.data import synthetic_cells

    def fwd(times, theta):
        nan = [np.full(len(t), np.nan) for t in times]
        with Likelihood(from_lists([(t, a, a) for t, a in zip(times, nan)])) as L:
            return L.forward(theta, np.arange(len(times), dtype=np.int32), grid="interp")

    cells, truth = synthetic_cells(n_cells, n_points, seed, fwd, nan_fraction=0.0)
    truth[:, 7:] = 0.0
    ms2, pp7 = fwd([cells.cell(c)[0] for c in range(n_cells)], truth)
    rng = np.random.default_rng(seed + 1)
    cells = from_lists([(cells.cell(c)[0], ms2[c, :n_points] + rng.normal(0, noise, n_points),
                         pp7[c, :n_points] + rng.normal(0, noise, n_points)) for c in range(n_cells)])
    return cells, truth


def test_stays_at_the_truth_on_synthetic_cells():
    """Started near the generating parameters, the chains stay at the mode: posterior means of v
    and the mean rate land on the truth and the SS stays at the noise level. (From the
    reference's random x0 this 127-parameter posterior is multimodal and chains can stick in
    local modes for 10^5 steps -- the reason the reference runs 200k steps and curates fits.)"""
    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    cells, truth = _synthetic(64, 120, 0.3, 99)
    with Likelihood(cells) as L:
        ids = np.arange(64, dtype=np.int32)
        x0, lo, hi, mu, sg, J0 = setup_rows(cells, list(ids), seed=2)
        x0[:, :127] = truth[:, :127]
        x0[:, 0] *= 1.02
        res = dram_run(L, ids, x0, lo, hi, mu, sg, J0, 1.0,
                       DramOptions(n_steps=6000, burnintime=2000, stats_from=3000, seed=4))
        ss_fin = L.ss_batch(res.final_theta, ids)
        ss_true = L.ss_batch(truth[:, :127], ids)
    err_v = np.abs(res.mean[:, 0] - truth[:, 0]) / truth[:, 0]
    err_R = np.abs(res.mean[:, 6] + res.mean[:, 7:126].mean(axis=1) - truth[:, 6]) / truth[:, 6]
    assert np.median(err_v) < 0.01, np.median(err_v)
    assert np.median(err_R) < 0.02, np.median(err_R)
    assert np.median(ss_fin / ss_true) < 1.5


@pytest.mark.parametrize("ntry", [1, 2])
def test_samples_the_exact_posterior_of_a_two_parameter_slice(ntry):
    """Free (v, R), every other parameter pinned: with sigma^2 integrated out under mcmcstat's
    Gibbs update (N0 = 0) the marginal target is p(v, R | y) ∝ SS(v, R)^(-N/2) on the box.
    Posterior mean/sd from a dense grid (the GPU likelihood) must match the pooled chains of 64
    independent samplers -- Metropolis (ntry=1) and delayed rejection (ntry=2) alike."""
    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    cells, truth = _synthetic(1, 120, 3.0, 5)
    P = 127
    N = 2 * 120
    t0 = truth[0, :P].copy()
    vlo, vhi, Rlo, Rhi = t0[0] - 0.6, t0[0] + 0.6, t0[6] - 6.0, t0[6] + 6.0
    with Likelihood(cells) as L:
        gv, gR = np.linspace(vlo, vhi, 1201), np.linspace(Rlo, Rhi, 1201)  # 0.05 sd spacing: the density is jagged
        V, RR = np.meshgrid(gv, gR, indexing="ij")
        grid = np.tile(t0, (V.size, 1))
        grid[:, 0], grid[:, 6] = V.ravel(), RR.ravel()
        ss = L.ss_batch(grid, np.zeros(V.size, np.int32)).reshape(V.shape)
        logw = -0.5 * N * np.log(ss)
        w = np.exp(logw - logw.max())
        w /= w.sum()
        mv, mR = (w * V).sum(), (w * RR).sum()
        sv, sR = np.sqrt((w * (V - mv) ** 2).sum()), np.sqrt((w * (RR - mR) ** 2).sum())
        # the posterior must sit well inside the box for the comparison to be exact
        assert vlo + 5 * sv < mv < vhi - 5 * sv and Rlo + 5 * sR < mR < Rhi - 5 * sR
        C = 64
        x0 = np.tile(t0, (C, 1))
        x0[:, 0], x0[:, 6] = mv, mR
        lo, hi = x0 - 1e-6, x0 + 1e-6
        lo[:, 0], hi[:, 0], lo[:, 6], hi[:, 6] = vlo, vhi, Rlo, Rhi
        mu, sg = np.zeros_like(x0), np.full_like(x0, np.inf)
        J0 = np.full_like(x0, 1e-20)
        J0[:, 0], J0[:, 6] = (1.7 * sv) ** 2, (1.7 * sR) ** 2
        res = dram_run(L, np.zeros(C, np.int32), x0, lo, hi, mu, sg, J0, 1.0,
                       DramOptions(n_steps=12000, adaptint=0, ntry=ntry, stats_from=2001, thin=4, seed=17 + ntry))
    rows = res.chain[500:]  # chain rows >= 2001
    v, R = rows[:, :, 0].ravel(), rows[:, :, 6].ravel()
    assert abs(v.mean() - mv) < 0.05 * sv, (v.mean(), mv, sv)
    assert abs(R.mean() - mR) < 0.05 * sR, (R.mean(), mR, sR)
    assert abs(v.std() / sv - 1) < 0.05, (v.std(), sv)
    assert abs(R.std() / sR - 1) < 0.05, (R.std(), sR)


def test_fit_driver_and_result_files(lk, tmp_path):
    import scipy.io as sio

    from transcriptioncycleinference_amd.mcmc import RESULT_FIELDS, fit, save_results

    fr = fit(lk, n_steps=300, n_burn=100, seed=3, thin=1, cells=[0, 5, 17])
    assert len(fr.MCMCresults) == 3 and [r["cell_index"] for r in fr.MCMCresults] == [1, 6, 18]
    for r, c in zip(fr.MCMCresults, [0, 5, 17]):
        assert set(r) == set(RESULT_FIELDS) and len(r["mean_dR"]) == lk.cells.lengths[c]
    ch = fr.MCMCchain[0]
    assert ch["v_chain"].shape == (201,) and ch["dR_chain"].shape == (201, lk.cells.lengths[0])
    assert ch["s2chain"].shape == (300,)
    np.testing.assert_allclose(fr.MCMCresults[0]["mean_v"], ch["v_chain"].mean(), rtol=1e-12)
    np.testing.assert_allclose(fr.MCMCresults[0]["sigma_v"], ch["v_chain"].std(), rtol=1e-9, atol=1e-15)
    a, b = save_results(fr, str(tmp_path), date="15-Oct-2026")
    d = sio.loadmat(a, squeeze_me=True, struct_as_record=False)
    assert d["DatasetName"] == fr.DatasetName
    m = d["MCMCresults"]
    assert len(m) == 3 and m[1].cell_index == 6 and abs(m[2].mean_v - fr.MCMCresults[2]["mean_v"]) == 0
    p = d["MCMCplot"][0]
    np.testing.assert_array_equal(p.t_plot, lk.cells.cell(0)[0])
    raw = sio.loadmat(b, squeeze_me=True, struct_as_record=False)["MCMCchain"]
    assert raw[0].dR_chain.shape == (201, lk.cells.lengths[0])


def test_fit_skips_cells_without_previous_v(lk):
    from transcriptioncycleinference_amd.mcmc import fit

    fr = fit(lk, n_steps=50, n_burn=10, cells=[0, 1, 2, 3], v0=[1.5, None, float("nan"), 2.0])
    assert [r["cell_index"] for r in fr.MCMCresults] == [1, 4]
    assert all(abs(r["mean_v"] - v) <= 1e-5 for r, v in zip(fr.MCMCresults, [1.5, 2.0]))


@pytest.mark.parametrize("ntry", [2, 1])
def test_fused_and_batched_engines_give_identical_chains(lk, ntry):
    """The fused engine (one workgroup per chain, ssfun inside the step loop) and the batched
    engine (one launch per stage, graph-replayed) share RNG keys, reductions and operation order:
    every output must be bitwise equal, through burn-in scaling, covariance adaptation and a
    tail shorter than adaptint."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(0, 299, 5))
    o = DramOptions(n_steps=650, burnintime=300, adaptint=100, stats_from=200, thin=7, seed=11, ntry=ntry)
    o.engine = "fused"
    a, _ = run(lk, ids, o)
    o.engine = "batched"
    b, _ = run(lk, ids, o)
    o.engine = "walk"  # one wavefront per chain
    c, _ = run(lk, ids, o)
    for f in ("chain", "s2chain", "mean", "std", "final_theta", "sigma_mean", "sigma_std", "accept_rate", "n_evals"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
        np.testing.assert_array_equal(getattr(c, f), getattr(b, f), err_msg="walk " + f)
    assert np.median(a.accept_rate) > 0.01


STATS_CASES = {  # (n_steps, adaptint, burnintime, stats_from, max_chunk)
    "stats_from_mid_window_partial_last": (437, 100, 200, 150, 0),
    "no_adaptation": (300, 0, 100, 77, 0),
    "window_spans_chunks": (437, 100, 200, 150, 30),
    "every_row": (250, 100, 100, 1, 0),
    "stats_from_last_row": (305, 100, 100, 305, 0),
}


@pytest.mark.parametrize("engine", ["fused", "walk", "batched"])
@pytest.mark.parametrize("case", sorted(STATS_CASES))
def test_posterior_summaries_equal_the_chain_rows(lk, engine, case):
    """The on-device summaries (window sums merged pairwise, carried across chunks) against the raw
    rows (thin = 1): mean(chain(stats_from:end, :)) and std(., 1) (TranscriptionCycleMCMC.m:284-301),
    sqrt(mean(s2chain)) and std(sqrt(s2chain), 1) (:302-303) over every row -- with stats_from inside
    a window, a partial last window, no adaptation (window = chunk), a window split over several
    chain-kernel launches (max_chunk < adaptint) and a one-row statistics range."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    n_steps, ai, burn, sf, mc = STATS_CASES[case]
    ids = list(range(3, 299, 23))
    o = DramOptions(n_steps=n_steps, adaptint=ai, burnintime=burn, stats_from=sf, thin=1, seed=41, engine=engine,
                    max_chunk=mc)
    res, _ = run(lk, ids, o)
    n = lk.cells.lengths[ids]
    assert res.chain.shape[0] == n_steps
    for k in range(len(ids)):
        P = 7 + int(n[k])
        X = res.chain[sf - 1:, k, :P]
        scale = np.abs(X).max(axis=0) + 1.0
        np.testing.assert_allclose(res.mean[k, :P], X.mean(axis=0), rtol=0, atol=1e-12 * scale.max(), err_msg=case)
        np.testing.assert_allclose(res.std[k, :P], X.std(axis=0), rtol=0, atol=1e-10 * scale.max(), err_msg=case)
        q = np.sqrt(res.s2chain[:, k])
        np.testing.assert_allclose(res.sigma_mean[k], np.sqrt(res.s2chain[:, k].mean()), rtol=1e-12, err_msg=case)
        np.testing.assert_allclose(res.sigma_std[k], q.std(), rtol=1e-9, atol=1e-12 * q.max(), err_msg=case)
    assert np.median(res.accept_rate) > 0.01


@pytest.mark.parametrize("engine", ["fused", "walk"])
def test_chunk_size_does_not_change_the_chains(lk, engine):
    """The fused engines' chunking (draws pass + walk per chunk) is invisible in the chains: a run
    whose windows span several chunks equals the one-chunk-per-window run bit for bit."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(0, 299, 29))
    o = DramOptions(n_steps=437, burnintime=200, adaptint=100, stats_from=150, thin=3, seed=5, engine=engine)
    a, _ = run(lk, ids, o)
    o.max_chunk = 17
    b, _ = run(lk, ids, o)
    for f in ("chain", "s2chain", "mean", "std", "final_theta", "sigma_mean", "sigma_std", "accept_rate", "n_evals"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)


@pytest.mark.parametrize("ntry,updatesigma,max_chunk", [(2, True, 0), (1, True, 23), (2, False, 9)])
def test_split_draws_equal_the_one_launch_draws(lk, monkeypatch, ntry, updatesigma, max_chunk):
    """The fused engine's split draws (the next chunk's normals and scalar draws by extra k_chain
    workgroups into the other draws buffer, k_draws multiplying by R in place) against
    the one-launch draws pass (TCI_DRAWS_SPLIT=0): every output bitwise equal -- stage-2 normals
    zeroed (ntry = 1), no Gamma draws (updatesigma off), chunks shorter than a window and a short
    last chunk."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(1, 299, 13))
    o = DramOptions(n_steps=377, burnintime=150, adaptint=100, stats_from=120, thin=4, seed=23, ntry=ntry,
                    updatesigma=updatesigma, engine="fused", max_chunk=max_chunk)
    monkeypatch.setenv("TCI_DRAWS_SPLIT", "1")
    a, _ = run(lk, ids, o)
    monkeypatch.setenv("TCI_DRAWS_SPLIT", "0")
    b, _ = run(lk, ids, o)
    for f in ("chain", "s2chain", "mean", "std", "final_theta", "sigma_mean", "sigma_std", "accept_rate", "n_evals"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    assert np.median(a.accept_rate) > 0.01


@pytest.mark.parametrize("engine", ["fused", "batched"])
def test_adapted_proposal_is_the_scaled_chain_covariance(lk, engine):
    """mcmcstat's adaptation: after the last adaptation row n (n >= burnintime), the proposal
    factor satisfies R'R = (2.4/sqrt(P))^2 (cov(chain rows 1..n) + qcovadj I) with the sample
    covariance of every row so far (covupd's recurrence). R is FP64, as mcmcstat's double chol:
    the factorisation agrees to 1e-12 (round 2 kept R float-representable and needed 1e-6)."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = list(range(0, 299, 37))
    o = DramOptions(n_steps=700, burnintime=300, adaptint=100, stats_from=1, thin=1, seed=21, engine=engine)
    x0, lo, hi, mu, sg, J0 = setup_rows(lk.cells, ids, 0)
    from transcriptioncycleinference_amd.mcmc import dram_run

    res = dram_run(lk, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o, want_qcov=True)
    n = lk.cells.lengths[ids]
    for k in range(len(ids)):
        P = 7 + int(n[k])
        X = res.chain[:700, k, :P]
        C = np.cov(X.T, ddof=1) + 1e-5 * np.eye(P)
        R = res.qcov_R[k, :P, :P]
        assert np.all(np.tril(R, -1) == 0)
        assert not np.array_equal(R, R.astype(np.float32).astype(np.float64))  # no fp32 rounding
        Q = R.T @ R
        want = (2.4 ** 2 / P) * C
        np.testing.assert_allclose(Q, want, rtol=1e-12, atol=1e-12 * np.abs(want).max())


@pytest.mark.parametrize("engine", ["fused", "batched", "walk"])
def test_chain_keys_let_a_shard_reproduce_the_full_run(lk, engine):
    """chains keyed by their global index reproduce, on a shard (a subset of the
    chains run alone, as one GPU of a sharded fit would), the rows of the unsharded run bitwise."""
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    ids = list(range(40, 100))
    o = DramOptions(n_steps=450, burnintime=200, adaptint=100, stats_from=100, thin=9, seed=5, engine=engine)
    x0, lo, hi, mu, sg, J0 = setup_rows(lk.cells, ids, 0)
    keys = np.array(ids, np.int64)
    full = dram_run(lk, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o, chain_keys=keys)
    for a, b in ((0, 25), (25, 60)):
        sl = slice(a, b)
        part = dram_run(lk, np.array(ids[sl], np.int32), x0[sl], lo[sl], hi[sl], mu[sl], sg[sl], J0[sl], 1.0, o,
                        chain_keys=keys[sl])
        for f in ("mean", "std", "final_theta", "sigma_mean", "accept_rate", "n_evals"):
            np.testing.assert_array_equal(getattr(part, f), getattr(full, f)[sl], err_msg=f)
        np.testing.assert_array_equal(part.chain, full.chain[:, sl])
    # no keys = keyed by row index
    d0 = dram_run(lk, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o)
    d1 = dram_run(lk, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o,
                  chain_keys=np.arange(len(ids), dtype=np.int64))
    np.testing.assert_array_equal(d0.chain, d1.chain)


def _previous_for_shards():
    """A hierarchical-fit input over all 299 cells with gaps and curation flags (by cell_index)."""
    from transcriptioncycleinference_amd.mcmc import PreviousFit

    return {c + 1: PreviousFit(1.0 + (c % 17) * 0.1, c % 3 - 1) for c in range(299) if c % 11 != 5}


def _sharded_worker(rank, world, port, q, backend="gloo", hierarchical=False):
    import os

    import torch
    import torch.distributed as dist

    from transcriptioncycleinference_amd import Likelihood, testdata
    from transcriptioncycleinference_amd.parallel import fit_sharded, pack_results

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":  # RCCL, as on a multi-GPU node (here world 1 on this GPU)
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        dev = "cuda:0"
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = None
    cells = testdata()
    kw = dict(v0=_previous_for_shards()) if hierarchical else {}
    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4", device=0) as L:
        fr = fit_sharded(L, device=dev, n_steps=400, n_burn=150, seed=4, **kw)
    if rank == 0:
        q.put(pack_results(fr, int(cells.lengths.max())))
    dist.barrier()
    dist.destroy_process_group()


def _run_sharded(world, backend, hierarchical):
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, backend, hierarchical))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("hierarchical", [False, True])
def test_sharded_fit_world2_equals_the_one_gpu_fit(lk, hierarchical):
    """parallel.fit_sharded over 2 ranks (gloo, both on this GPU; RCCL on a multi-GPU node): each
    rank fits its cell range, one all-gather assembles MCMCresults/MCMCplot -- equal bitwise to
    fitting every cell in one process. The hierarchical case passes loadPrevious inputs with gaps
    and ApprovedFits over all cells: every rank reads them by cell, not by shard position."""
    from transcriptioncycleinference_amd.mcmc import fit
    from transcriptioncycleinference_amd.parallel import pack_results

    got = _run_sharded(2, "gloo", hierarchical)
    kw = dict(v0=_previous_for_shards()) if hierarchical else {}
    want = pack_results(fit(lk, n_steps=400, n_burn=150, seed=4, **kw), int(lk.cells.lengths.max()))
    n = 299 - (len(range(5, 299, 11)) if hierarchical else 0)
    assert got.shape == want.shape == (n, want.shape[1])
    np.testing.assert_array_equal(got, want)
    if hierarchical:
        prev = _previous_for_shards()
        for row in got:
            p = prev[int(row[0])]
            assert row[1] == p.ApprovedFits and abs(row[4] - p.mean_v) <= 1e-5 + 1e-12


def test_sharded_fit_over_rccl_world1(lk):
    """The RCCL branch of parallel.fit_sharded / gather_rows on hardware: backend 'nccl' (RCCL)
    with device_id, world size 1 (the 8-GPU run is the driver's): equal bitwise to the plain fit."""
    from transcriptioncycleinference_amd.mcmc import fit
    from transcriptioncycleinference_amd.parallel import pack_results

    got = _run_sharded(1, "nccl", True)
    want = pack_results(fit(lk, n_steps=400, n_burn=150, seed=4, v0=_previous_for_shards()),
                        int(lk.cells.lengths.max()))
    np.testing.assert_array_equal(got, want)


def test_config3_hierarchical_fit_from_a_results_file(lk, tmp_path, means, c_oracle, construct):
    """BASELINE config 3 at full size, through the file: a results file in the reference's schema
    holding the reference's own MCMCresults.mean_v (28-Oct-2020-TestData.mat, tests/golden) with
    two entries removed and curation flags set, read by load_previous, then the 299-cell fixed-v
    fit (TranscriptionCycleMCMC.m:84-107,193-198,218,236-237,345-350). Checks: cells missing from
    the file are skipped and pruned, v stays within v0 +- 1e-5, ApprovedFits is carried, and the
    SS at every chain's final state equals the oracle's."""
    from transcriptioncycleinference_amd.mcmc import RESULT_FIELDS, FitResult, fit, load_previous, save_results

    cl = lk.cells
    v_ref = np.array([r[0] for r in means["rows"]])
    drop = {17, 230}                                        # 1-based cell_index missing from the file
    res, plots = [], []
    for c in range(cl.n_cells):
        if c + 1 in drop:
            continue
        n = int(cl.lengths[c])
        r = {f: 0.0 for f in RESULT_FIELDS}
        r.update(mean_v=float(v_ref[c]), mean_dR=np.zeros(n), sigma_dR=np.zeros(n), cell_index=c + 1,
                 ApprovedFits=(1 if c % 4 == 0 else -1 if c % 4 == 1 else 0))
        res.append(r)
        t, m, p = cl.cell(c)
        plots.append({"t_plot": t, "MS2_plot": m, "PP7_plot": p, "simMS2": m, "simPP7": p})
    path = save_results(FitResult("InitialRise", res, plots, [{} for _ in res], np.zeros(len(res)), 0, 0.0),
                        str(tmp_path), date="28-Oct-2020")[0]
    fr = fit(lk, n_steps=2000, n_burn=500, seed=9, v0=load_previous(path))
    ci = [r["cell_index"] for r in fr.MCMCresults]
    assert ci == [c + 1 for c in range(cl.n_cells) if c + 1 not in drop]
    for r in fr.MCMCresults:
        c = r["cell_index"] - 1
        assert abs(r["mean_v"] - v_ref[c]) <= 1e-5 + 1e-12
        assert r["ApprovedFits"] == (1 if c % 4 == 0 else -1 if c % 4 == 1 else 0)
        assert np.isfinite(r["mean_sigma"]) and np.all(np.isfinite(r["mean_dR"]))
    assert np.all(np.abs(fr.final_theta[:, 0] - v_ref[fr.cell_index]) <= 1e-5 + 1e-12)
    cid = fr.cell_index.astype(np.int32)
    ss = lk.ss_batch(fr.final_theta, cid)
    want, st = c_oracle.ss_batch(cl.offsets, cl.t, cl.ms2, cl.pp7, construct, fr.final_theta, cid)
    assert np.all(st == 0)
    np.testing.assert_allclose(ss, want, rtol=1e-10)
    assert np.median(fr.accept_rate) > 0.01


@pytest.fixture(scope="module")
def lk_long():
    """Synthetic cells of 150 and 200 points (P = 157, 207): the adaptation runs on the 8-wave
    matrix-core kernel (k_adapt_mfma<8, 13>, P <= 208), as for BASELINE configs 4/5."""
    from transcriptioncycleinference_amd import Likelihood, from_lists

    rng = np.random.default_rng(11)
    cells = []
    for k in range(12):
        n = 200 if k % 3 else 150
        t = 0.2454 * np.arange(n) + rng.uniform(-0.012, 0.012, n)
        ms2 = rng.normal(20.0, 5.0, n)
        pp7 = rng.normal(10.0, 3.0, n)
        ms2[rng.random(n) < 0.37] = np.nan
        cells.append((t, ms2, pp7))
    with Likelihood(from_lists(cells), "P2P-MS2v5-LacZ-PP7v4", device=0) as L:
        yield L


@pytest.mark.parametrize("engine", ["fused", "batched"])
def test_long_cells_adapted_proposal_is_the_scaled_chain_covariance(lk_long, engine):
    """As test_adapted_proposal_is_the_scaled_chain_covariance, for P in (144, 208] (the 8-wave
    adaptation kernel); the fused and batched engines agree bitwise."""
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    ids = list(range(12))
    o = DramOptions(n_steps=500, burnintime=200, adaptint=100, stats_from=1, thin=1, seed=4, engine=engine)
    x0, lo, hi, mu, sg, J0 = setup_rows(lk_long.cells, ids, 0)
    res = dram_run(lk_long, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o, want_qcov=True)
    n = lk_long.cells.lengths[ids]
    for k in range(len(ids)):
        P = 7 + int(n[k])
        X = res.chain[:500, k, :P]
        C = np.cov(X.T, ddof=1) + 1e-5 * np.eye(P)
        R = res.qcov_R[k, :P, :P]
        assert np.all(np.tril(R, -1) == 0)
        assert not np.array_equal(R, R.astype(np.float32).astype(np.float64))  # FP64 R
        want = (2.4 ** 2 / P) * C
        np.testing.assert_allclose(R.T @ R, want, rtol=1e-12, atol=1e-12 * np.abs(want).max())
    if engine == "batched":
        for other in ("fused", "walk"):
            o.engine = other
            res_f = dram_run(lk_long, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o, want_qcov=True)
            np.testing.assert_array_equal(res_f.chain, res.chain, err_msg=other)
            np.testing.assert_array_equal(res_f.qcov_R, res.qcov_R, err_msg=other)


def test_engines_agree_on_the_two_segment_construct():
    """BASELINE config 5's construct (2 segments per dye, 3x length): the fused, walk and batched
    engines give bitwise-equal chains (the walk re-reads bounds and priors per evaluation there)."""
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.construct import long_two_loop_construct
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    rng = np.random.default_rng(12)
    cells = []
    for k in range(10):
        n = 120 + 8 * k
        t = 0.2454 * np.arange(n) + rng.uniform(-0.012, 0.012, n)
        cells.append((t, rng.normal(20.0, 5.0, n), rng.normal(10.0, 3.0, n)))
    with Likelihood(from_lists(cells), long_two_loop_construct(), device=0) as L:
        ids = list(range(10))
        x0, lo, hi, mu, sg, J0 = setup_rows(L.cells, ids, 0)
        out = {}
        for eng in ("batched", "fused", "walk"):
            o = DramOptions(n_steps=400, burnintime=150, adaptint=100, stats_from=100, thin=3, seed=8, engine=eng)
            out[eng] = dram_run(L, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o)
    for eng in ("fused", "walk"):
        for f in ("chain", "s2chain", "mean", "std", "final_theta", "accept_rate", "n_evals"):
            np.testing.assert_array_equal(getattr(out[eng], f), getattr(out["batched"], f), err_msg=f"{eng} {f}")
    assert np.median(out["walk"].accept_rate) > 0.01


@pytest.mark.parametrize("n", [293, 600])
def test_very_long_cells_sample_and_adapt(n):
    """Cells past the fused engine's LDS budget (P = 300: the batched engine; N = 600: the
    long-cell likelihood kernel too, R read from global memory in the proposal products and the
    generic adaptation): the chains stay in bounds, are deterministic per seed, and the adapted
    proposal is the scaled chain covariance (ConstantElongationSim.m:39-50 has no length cap)."""
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    rng = np.random.default_rng(n)
    cl = []
    for _ in range(3):
        t = 0.2454 * np.arange(n) + rng.uniform(-0.012, 0.012, n)
        ms2 = rng.normal(20.0, 5.0, n)
        pp7 = rng.normal(10.0, 3.0, n)
        ms2[rng.random(n) < 0.37] = np.nan
        cl.append((t, ms2, pp7))
    with Likelihood(from_lists(cl), "P2P-MS2v5-LacZ-PP7v4", device=0) as L:
        assert L.info["rows_per_lane"] == (8 if n <= 513 else 0)
        ids = [0, 1, 2]
        o = DramOptions(n_steps=300, burnintime=100, adaptint=100, stats_from=1, thin=1, seed=9)
        x0, lo, hi, mu, sg, J0 = setup_rows(L.cells, ids, 0)
        res = dram_run(L, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o, want_qcov=True)
        res2 = dram_run(L, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o, want_qcov=True)
        others = {}
        if n <= 513:  # the fused and walk engines (R read from global memory in the draws pass)
            for eng in ("batched", "fused", "walk"):
                o.engine = eng
                others[eng] = dram_run(L, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o, want_qcov=True)
    np.testing.assert_array_equal(res.chain, res2.chain)
    for eng, r in others.items():
        np.testing.assert_array_equal(r.chain, res.chain, err_msg=eng)
        np.testing.assert_array_equal(r.qcov_R, res.qcov_R, err_msg=eng)
    P = 7 + n
    for k in range(3):
        X = res.chain[:300, k, :P]
        assert np.all(X >= lo[k, :P]) and np.all(X <= hi[k, :P])
        assert len(np.unique(X[:, 0])) > 5  # the chain moves
        C = np.cov(X.T, ddof=1) + 1e-5 * np.eye(P)
        R = res.qcov_R[k, :P, :P]
        assert np.all(np.tril(R, -1) == 0)
        want = (2.4 ** 2 / P) * C
        np.testing.assert_allclose(R.T @ R, want, rtol=1e-10, atol=1e-10 * np.abs(want).max())  # FP64 R, P <= 520


@pytest.mark.parametrize("cfg", [4, 5])
def test_walk_at_10000_chains_equals_fused_and_batched(cfg, c_oracle):
    """BASELINE configs 4 and 5 at their full chain count (10,000 synthetic cells x 200 points, one chain
    per cell; config 5 on the two-segment, 3x-length construct, whose WALK instance keeps its bounds in
    registers): WALK -- what AUTO runs there -- against FUSED and the batched engine, bit for bit, over
    two adaptation windows; every output finite, and the SS of 256 of the 10,000 final states equal to
    the C oracle's (SumofSquares...m:28-64 restated) within 1e-10."""
    import bench
    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.mcmc import DramOptions, fit

    cells, _, construct = bench.synthetic_config_cells(cfg, 0, 1, 0)[:3]
    assert cells.n_cells == 10000 and construct.n_seg == (1 if cfg == 4 else 2)
    out = {}
    with Likelihood(cells, construct, device=0) as L:
        for eng in ("walk", "fused", "batched"):
            fr = fit(L, n_steps=240, n_burn=120, seed=5, opts=DramOptions(engine=eng))
            out[eng] = fr
    w = out["walk"]
    assert np.all(np.isfinite(w.final_theta)) and np.all(np.isfinite([r["mean_v"] for r in w.MCMCresults]))
    assert np.median(w.accept_rate) > 0.01
    for eng in ("fused", "batched"):
        o = out[eng]
        np.testing.assert_array_equal(o.final_theta, w.final_theta, err_msg=eng)
        np.testing.assert_array_equal(o.accept_rate, w.accept_rate, err_msg=eng)
        np.testing.assert_array_equal(o.n_evals, w.n_evals, err_msg=eng)
        np.testing.assert_array_equal([r["mean_v"] for r in o.MCMCresults], [r["mean_v"] for r in w.MCMCresults],
                                      err_msg=eng)
    sample = np.linspace(0, 9999, 256).astype(np.int64)
    th = np.ascontiguousarray(w.final_theta[sample])
    with Likelihood(cells, construct, device=0) as L:
        got = L.ss_batch(th, sample.astype(np.int32))
    want, st = c_oracle.ss_batch(cells.offsets, cells.t, cells.ms2, cells.pp7, construct, th, sample.astype(np.int32))
    assert np.all(st == 0)
    np.testing.assert_allclose(got, want, rtol=1e-10, atol=0)


@pytest.mark.parametrize("engine", ["fused", "walk", "batched"])
def test_gpu_chains_follow_the_cpu_restatement(lk, c_oracle, construct, engine):
    """The GPU sampler against the CPU restatement of mcmcstat's DRAM (oracle/tci_dram_oracle.c, the
    C oracle as ssfun, mcmcstat's own MATLAB-form expressions: divisions by sigma2, the alpha13
    quotient, R./drscale, covupd's row recurrence, a textbook Cholesky) on the same Philox streams:
    both chains take the same accept / reject decisions at every step, through burn-in scaling and
    covariance adaptation, and their rows agree to the rounding of the continuous arithmetic."""
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run, plan_fit

    ids = [0, 41, 97, 150, 222, 298]
    plan = plan_fit(lk.cells, ids, 3)
    o = DramOptions(n_steps=600, burnintime=300, adaptint=100, stats_from=200, thin=1, seed=77, engine=engine)
    keys = np.array(plan.cells, np.int64)
    g = dram_run(lk, np.array(plan.cells, np.int32), plan.x0, plan.lower, plan.upper, plan.prior_mu, plan.prior_sig,
                 plan.qcov_diag, 1.0, o, chain_keys=keys)
    c = c_oracle.dram_run(lk.cells, construct, np.array(plan.cells, np.int32), plan.x0, plan.lower, plan.upper,
                          plan.prior_mu, plan.prior_sig, plan.qcov_diag, 1.0, o, keys=keys, want_chain=True)
    n = lk.cells.lengths[ids]
    for k in range(len(ids)):
        P = 7 + int(n[k])
        G, Cc = g.chain[:, k, :P], c["chain"][:, k, :P]
        moved_g = np.any(G[1:] != G[:-1], axis=1)
        moved_c = np.any(Cc[1:] != Cc[:-1], axis=1)
        np.testing.assert_array_equal(moved_g, moved_c, err_msg=f"chain {k}: accept/reject decisions differ")
        np.testing.assert_allclose(G, Cc, rtol=1e-9, atol=1e-9, err_msg=f"chain {k}")
        np.testing.assert_allclose(g.s2chain[:, k], c["s2chain"][:, k], rtol=1e-9)
        assert g.n_evals[k] == c["n_evals"][k]
        np.testing.assert_allclose(g.mean[k, :P], c["mean"][k, :P], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(g.std[k, :P], c["std"][k, :P], rtol=1e-7, atol=1e-9)
    assert np.median(g.accept_rate) > 0.02


# BASELINE configs 4/5 shapes for the restatement check, and one past the
# 8-wave adaptation kernel: (chains, points per cell, construct, data seed).
#   config4: N = 200, P = 207, the built-in construct -- k_adapt_mfma<8, 13>, WALK / FUSED / batched;
#   config5: N = 200, the two-segment 3x-length construct (BASELINE config 5);
#   long:    N = 210, P = 217 > 208 -- the generic adaptation kernel k_adapt_gt;
#   mid:     N = 145 / 160 / 180 (P = 152 / 167 / 187: 10, 11 and 12 tiles per dimension), the tile
#            ownership maps of k_adapt_mfma<8, 13> no BASELINE config reaches (tci_adapt_map.h).
RESTATEMENT_SHAPES = {
    "config4": (24, 200, "builtin", 20201028),
    "config5": (16, 200, "two_segment", 20201029),
    "long": (8, 210, "builtin", 20201030),
    "mid": (4, (145, 160, 180), "builtin", 20201031),
}
_restatement_cache = {}


def _restatement_case(shape, c_oracle):
    """Synthetic cells of the shape (SURVEY §8(d) item 4's generator), the reference's per-cell setup
    (plan_fit) and the CPU restatement's chains -- computed once per shape for every engine."""
    if shape in _restatement_cache:
        return _restatement_cache[shape]
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.construct import builtin_construct, long_two_loop_construct
    from transcriptioncycleinference_amd.data import synthetic_cells
    from transcriptioncycleinference_amd.mcmc import DramOptions, plan_fit

    n_cells, n_points, cname, seed = RESTATEMENT_SHAPES[shape]
    cs = builtin_construct("P2P-MS2v5-LacZ-PP7v4") if cname == "builtin" else long_two_loop_construct()

    def fwd(times, theta):
        nan = [np.full(len(t), np.nan) for t in times]
        with Likelihood(from_lists([(t, a, a) for t, a in zip(times, nan)]), cs, device=0) as L:
            return L.forward(theta, np.arange(len(times), dtype=np.int32), grid="interp")

    if isinstance(n_points, tuple):  # n_cells cells of each length
        parts = []
        for i, npts in enumerate(n_points):
            cc, _ = synthetic_cells(n_cells, npts, seed + 7919 * i, fwd)
            o_ = cc.offsets
            parts += [(cc.t[o_[k]:o_[k + 1]], cc.ms2[o_[k]:o_[k + 1]], cc.pp7[o_[k]:o_[k + 1]]) for k in range(n_cells)]
        cells = from_lists(parts, f"synthetic-mixed-{shape}")
        n_cells = len(parts)
    else:
        cells, _ = synthetic_cells(n_cells, n_points, seed, fwd)
    plan = plan_fit(cells, list(range(n_cells)), 5)
    o = DramOptions(n_steps=700, burnintime=300, adaptint=100, stats_from=200, thin=1, seed=91)
    keys = np.array(plan.cells, np.int64)
    want = c_oracle.dram_run(cells, cs, np.array(plan.cells, np.int32), plan.x0, plan.lower, plan.upper,
                             plan.prior_mu, plan.prior_sig, plan.qcov_diag, 1.0, o, keys=keys, want_chain=True,
                             want_R=True)
    _restatement_cache[shape] = (cells, cs, plan, o, keys, want)
    return _restatement_cache[shape]


@pytest.mark.parametrize("engine", ["fused", "walk", "batched"])
@pytest.mark.parametrize("shape", sorted(RESTATEMENT_SHAPES))
def test_gpu_chains_follow_the_cpu_restatement_at_config_shapes(c_oracle, shape, engine):
    """As test_gpu_chains_follow_the_cpu_restatement, at the shapes BASELINE configs 4/5 run
    (TranscriptionCycleMCMC.m:263-273): 700 steps, burn-in scaling at rows 100-300, then four covariance
    updates (rows 400-700) on the P <= 208 matrix-core adaptation (k_adapt_mfma<8, 13>) or, for P = 217,
    on k_adapt_gt, and on cells of 10-12 tiles per dimension (the "mid" shape); every engine. Same accept / reject decision at every step; rows, s2chain, summaries
    and the final proposal factor R within 1e-9."""
    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.mcmc import dram_run

    cells, cs, plan, o, keys, c = _restatement_case(shape, c_oracle)
    o = dataclasses.replace(o, engine=engine)
    with Likelihood(cells, cs, device=0) as L:
        g = dram_run(L, np.array(plan.cells, np.int32), plan.x0, plan.lower, plan.upper, plan.prior_mu,
                     plan.prior_sig, plan.qcov_diag, 1.0, o, chain_keys=keys, want_qcov=True)
    n = cells.lengths[plan.cells]
    assert int(7 + n.max()) == {"config4": 207, "config5": 207, "long": 217, "mid": 187}[shape]
    if shape == "mid":
        assert sorted(set(((7 + n + 15) // 16).tolist())) == [10, 11, 12]
    for k in range(len(plan.cells)):
        P = 7 + int(n[k])
        G, Cc = g.chain[:, k, :P], c["chain"][:, k, :P]
        moved_g = np.any(G[1:] != G[:-1], axis=1)
        moved_c = np.any(Cc[1:] != Cc[:-1], axis=1)
        np.testing.assert_array_equal(moved_g, moved_c, err_msg=f"{shape} chain {k}: accept/reject decisions differ")
        np.testing.assert_allclose(G, Cc, rtol=1e-9, atol=1e-9, err_msg=f"{shape} chain {k}")
        np.testing.assert_allclose(g.s2chain[:, k], c["s2chain"][:, k], rtol=1e-9)
        assert g.n_evals[k] == c["n_evals"][k]
        np.testing.assert_allclose(g.mean[k, :P], c["mean"][k, :P], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(g.std[k, :P], c["std"][k, :P], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(g.sigma_mean[k], c["sigma_mean"][k], rtol=1e-9)
        R, Rc = g.qcov_R[k, :P, :P], c["R"][k, :P, :P]
        np.testing.assert_allclose(R, Rc, rtol=1e-9, atol=1e-9 * np.abs(Rc).max(), err_msg=f"{shape} chain {k}: R")
    moved = np.any(g.chain[1:] != g.chain[:-1], axis=2).mean(axis=0)
    assert np.median(moved) > 0.01, moved


def test_output_padding_is_the_documented_contract(c_oracle):
    """include/tci.h (tci_dram_outputs): past a chain's P, mean/std are NaN, final_theta keeps theta0's
    padding, chain rows and qcov_R are 0 -- on the GPU and in the CPU restatement alike (two cell
    lengths in one run, so the shorter chain's rows are padded)."""
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run, plan_fit

    cells, cs = _restatement_case("config4", c_oracle)[:2]
    two = from_lists([cells.cell(0), tuple(a[:150] for a in cells.cell(1))])
    p = plan_fit(two, [0, 1], 5)
    p.x0[1, 157:] = 3.25                                    # theta0 padding the outputs must keep
    o = DramOptions(n_steps=250, burnintime=100, adaptint=100, stats_from=50, thin=1, seed=4)
    with Likelihood(two, cs, device=0) as L:
        g = dram_run(L, np.array([0, 1], np.int32), p.x0, p.lower, p.upper, p.prior_mu, p.prior_sig, p.qcov_diag,
                     1.0, o, want_qcov=True)
    c = c_oracle.dram_run(two, cs, np.array([0, 1], np.int32), p.x0, p.lower, p.upper, p.prior_mu, p.prior_sig,
                          p.qcov_diag, 1.0, o, want_chain=True, want_R=True)
    for name, got, want in (("mean", g.mean, c["mean"]), ("std", g.std, c["std"])):
        assert np.all(np.isnan(got[1, 157:])) and np.all(np.isnan(want[1, 157:])), name
        assert np.all(np.isfinite(got[:, :157])) and np.all(np.isfinite(got[0])), name
    np.testing.assert_array_equal(g.final_theta[1, 157:], 3.25)
    np.testing.assert_array_equal(c["final_theta"][1, 157:], 3.25)
    assert np.all(g.chain[:, 1, 157:] == 0) and np.all(c["chain"][:, 1, 157:] == 0)
    assert np.all(g.qcov_R[1, 157:, :] == 0) and np.all(g.qcov_R[1, :, 157:] == 0)
    assert np.all(c["R"][1, 157:, :] == 0)
    # no statistics rows at all: every mean / std entry is NaN
    o.stats_from = 251
    with Likelihood(two, cs, device=0) as L:
        g = dram_run(L, np.array([0, 1], np.int32), p.x0, p.lower, p.upper, p.prior_mu, p.prior_sig, p.qcov_diag,
                     1.0, o)
    c = c_oracle.dram_run(two, cs, np.array([0, 1], np.int32), p.x0, p.lower, p.upper, p.prior_mu, p.prior_sig,
                          p.qcov_diag, 1.0, o)
    assert np.all(np.isnan(g.mean)) and np.all(np.isnan(c["mean"])) and np.all(np.isnan(g.std))


def _config_shard_worker(rank, world, port, q, n_shards, shard_cells):
    """One rank of a config-4-shaped sharded fit: builds ONLY its own shards of the synthetic dataset
    (bench.synthetic_config_cells: shard s from seed 20201028 + s), fits them with chains keyed by the
    dataset-wide cell index, then the one all-gather (parallel.fit_sharded, cell_offset layout)."""
    import os

    import torch.distributed as dist

    import bench
    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.parallel import fit_sharded, pack_results

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cells, _, cs, n_total, _, lo, hi = bench.synthetic_config_cells(4, rank, world, 0, shard_cells=shard_cells,
                                                                    n_shards=n_shards)
    assert cells.n_cells == hi - lo
    with Likelihood(cells, cs, device=0) as L:
        fr = fit_sharded(L, cell_offset=lo, n_steps=300, n_burn=150, seed=4)
    if rank == 0:
        q.put((pack_results(fr, 200), fr.gather_bytes, fr.n_evals))
    dist.barrier()
    dist.destroy_process_group()


def test_config4_sharded_fit_is_the_same_at_every_world_size():
    """BASELINE config 4's layout -- fixed shards seeded 20201028 + shard, rank r of N
    builds only its own shards -- fitted over 2 ranks (gloo, both on this GPU; RCCL on a multi-GPU node)
    gathers to rows bitwise equal to the one-rank fit of the same shards (4 shards x 48 cells x 200
    points, 300 steps)."""
    import socket

    import torch.multiprocessing as mp

    import bench
    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.parallel import fit_sharded, pack_results

    n_shards, shard_cells = 4, 48
    cells, _, cs, n_total, _, lo, hi = bench.synthetic_config_cells(4, 0, 1, 0, shard_cells=shard_cells,
                                                                    n_shards=n_shards)
    assert (lo, hi, n_total) == (0, 192, 192)
    with Likelihood(cells, cs, device=0) as L:
        one = fit_sharded(L, cell_offset=0, n_steps=300, n_burn=150, seed=4)
    want = pack_results(one, 200)
    assert want.shape[0] == 192 and one.gather_bytes == want.nbytes
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_config_shard_worker, args=(r, 2, port, q, n_shards, shard_cells)) for r in range(2)]
    for p in procs:
        p.start()
    got, nbytes, n_evals = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(got, want)
    assert nbytes == want.nbytes and n_evals == one.n_evals
    assert np.median(got[:, 3]) > 0.01  # accept rates


def test_adaptint_past_the_adaptation_lds_is_refused_before_any_launch(c_oracle):
    """the adaptation kernel's run table grows with adaptint (4 bytes per window row);
    an adaptint whose table no longer fits a CU's LDS is refused with TCI_ERANGE up front (nothing
    launched), and one that fits runs. ADVICE r05: the check counts the kernel's static LDS too -- at
    config 4's P = 207 (k_adapt_mfma<8, 13, 12>) adaptint 26,815 fills the 160 KiB with dynamic LDS
    alone ((13 * 512 + 2 * 208) * 8 + 4 * 26,816 bytes), so the kernel's own __shared__ words make it
    one that cannot launch: refused; 26,751 leaves 256 bytes for them and runs."""
    from transcriptioncycleinference_amd import Likelihood, _lib
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    cells, cs, plan = _restatement_case("config4", c_oracle)[:3]
    sl = slice(0, 2)
    with Likelihood(cells, cs, device=0) as L:
        args = (np.array(plan.cells[:2], np.int32), plan.x0[sl], plan.lower[sl], plan.upper[sl], plan.prior_mu[sl],
                plan.prior_sig[sl], plan.qcov_diag[sl], 1.0)
        with pytest.raises(_lib.TciError) as ei:
            dram_run(L, *args, DramOptions(n_steps=50, burnintime=10, adaptint=40000, stats_from=1))
        assert ei.value.code == _lib.TCI_ERANGE and "LDS" in str(ei.value)
        ok = dram_run(L, *args, DramOptions(n_steps=3000, burnintime=10, adaptint=1500, stats_from=1))
        assert np.all(np.isfinite(ok.mean[:, :207]))
        dyn = (13 * 512 + 2 * 208) * 8 + (26815 + 1) * 4
        assert dyn == 160 * 1024
        with pytest.raises(_lib.TciError) as ei:
            dram_run(L, *args, DramOptions(n_steps=50, burnintime=10, adaptint=26815, stats_from=1))
        assert ei.value.code == _lib.TCI_ERANGE and "LDS" in str(ei.value)
        edge = dram_run(L, *args, DramOptions(n_steps=26760, burnintime=10, adaptint=26751, stats_from=1))
        assert np.all(np.isfinite(edge.mean[:, :207])) and np.all(edge.n_evals > 0)


def test_shard_without_long_cells_adapts_like_the_unsharded_fit():
    """the adaptation kernel is picked by the largest P of a run (k_adapt_gt past 208), and the
    two kernels scatter in different orders. A shard whose cells are all P = 207 passes the whole fit's
    largest P (DramOptions.adapt_pmax, as parallel.fit_sharded all-reduces it) and then equals the
    unsharded fit -- which holds two P = 217 cells -- bit for bit."""
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.construct import builtin_construct
    from transcriptioncycleinference_amd.data import synthetic_cells
    from transcriptioncycleinference_amd.mcmc import DramOptions, fit

    cs = builtin_construct("P2P-MS2v5-LacZ-PP7v4")

    def fwd(times, theta):
        nan = [np.full(len(t), np.nan) for t in times]
        with Likelihood(from_lists([(t, a, a) for t, a in zip(times, nan)]), cs, device=0) as L:
            return L.forward(theta, np.arange(len(times), dtype=np.int32), grid="interp")

    a, _ = synthetic_cells(6, 200, 11, fwd)
    b, _ = synthetic_cells(2, 210, 12, fwd)
    full = from_lists([a.cell(k) for k in range(6)] + [b.cell(k) for k in range(2)])
    kw = dict(n_steps=450, n_burn=150, seed=4)
    with Likelihood(full, cs, device=0) as L:
        assert L.info["rows_per_lane"] == 4
        one = fit(L, **kw)
    with Likelihood(full.subset(range(6)), cs, device=0) as L:
        assert L.info["rows_per_lane"] == 4
        shard = fit(L, opts=DramOptions(adapt_pmax=217), **kw)
        own = fit(L, **kw)                                          # picks k_adapt_mfma for its own P = 207
    np.testing.assert_array_equal(shard.final_theta[:, :207], one.final_theta[:6, :207])
    for k in range(6):
        for f in ("mean_v", "sigma_v", "mean_R", "mean_sigma", "mean_dR", "sigma_dR"):
            np.testing.assert_array_equal(shard.MCMCresults[k][f], one.MCMCresults[k][f], err_msg=f)
    assert np.all(np.isfinite(own.final_theta[:, :207]))


def _empty_rank_bench_worker(rank, world, port, q):
    """bench.synthetic_end_to_end with more ranks than shards (gloo, every rank on this GPU): rank 0
    owns no shard, builds no context, and still joins every collective."""
    import os

    import torch
    import torch.distributed as dist

    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def reduce(x, op):
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return float(t.item())

    out, spot = bench.synthetic_end_to_end(4, rank, world, 0, 200, reduce, coll_device="cpu", shard_cells=16,
                                           n_shards=2)
    q.put((rank, out["chains"], out["outputs_finite"], out["ssfun_evals"], len(spot["cid"])))
    dist.barrier()
    dist.destroy_process_group()


def test_config_end_to_end_with_more_ranks_than_shards():
    """bench.py's config-4/5 DRAM leg at N > 8 gave some ranks no shard; such a
    rank raised building a 0-cell context while the others waited in the collectives. Here 3 ranks over
    2 shards of 16 cells: every rank finishes, and every rank reports the 32 gathered chains."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_empty_rank_bench_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=300) for _ in range(3)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(3):
        chains, finite, evals, n_spot = got[r]
        assert chains == 32 and finite and evals == got[0][2]
        assert n_spot == (0 if r == 0 else 16)
