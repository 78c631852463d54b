"""The CPU restatement of the sampler (oracle/tci_dram_oracle.c: mcmcstat's DRAM as
TranscriptionCycleMCMC.m:263-273 calls it, with the C oracle as ssfun) -- CPU only.

mcmcstat is not vendored (README.md:5, version unpinned), so the restatement is pinned by what is
published: the generator's known-answer vectors (Random123's Philox4x32-10 KAT), and the algorithm's
defining properties on TestData cells -- bounds, the acceptance bookkeeping, mcmcstat's adapted
proposal R'R = (2.4^2/P) (cov(chain rows) + qcovadj I), the sigma^2 Gibbs law the reference's own
raw-chain fixture satisfies (tests/test_oracle_golden.py), and the posterior summaries against the
rows. The GPU sampler is compared with it chain for chain in tests/test_dram_gpu.py."""
import numpy as np
import pytest

from conftest import pack

KAT = [  # Random123 kat_vectors: philox4x32 10 rounds (counter, key) -> output
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_known_answers(c_oracle, ctr, key, want):
    assert c_oracle.philox(ctr, key) == want


def _plan(cells, ids, seed=0):
    from transcriptioncycleinference_amd.mcmc import plan_fit

    return plan_fit(cells, ids, seed)


def _run(c_oracle, cells, construct, ids, opts, **kw):
    p = _plan(cells, ids)
    return p, c_oracle.dram_run(cells, construct, np.array(p.cells, np.int32), p.x0, p.lower, p.upper, p.prior_mu,
                                p.prior_sig, p.qcov_diag, 1.0, opts, keys=np.array(p.cells, np.int64), **kw)


def test_chain_bookkeeping_and_bounds(c_oracle, cells, construct):
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = [0, 57, 298]
    o = DramOptions(n_steps=300, burnintime=150, adaptint=50, stats_from=100, seed=9)
    p, r = _run(c_oracle, cells, construct, ids, o, want_chain=True)
    n = cells.lengths[ids]
    for k in range(len(ids)):
        P = 7 + int(n[k])
        rows = r["chain"][:, k, :P]
        np.testing.assert_array_equal(rows[0], p.x0[k, :P])
        assert np.all(rows >= p.lower[k, :P]) and np.all(rows <= p.upper[k, :P])
        moved = np.any(rows[1:] != rows[:-1], axis=1).mean()
        assert moved == pytest.approx(r["accept_rate"][k], abs=1e-12)
        assert 1 + moved * 299 - 1e-9 <= r["n_evals"][k] <= 1 + 2 * 299
        np.testing.assert_array_equal(r["final_theta"][k, :P], rows[-1])
        X = rows[o.stats_from - 1:]
        np.testing.assert_allclose(r["mean"][k, :P], X.mean(0), rtol=0, atol=1e-12 * np.abs(X).max())
        np.testing.assert_allclose(r["std"][k, :P], X.std(0), rtol=0, atol=1e-10 * np.abs(X).max())
        q = np.sqrt(r["s2chain"][:, k])
        assert r["sigma_mean"][k] == pytest.approx(np.sqrt(r["s2chain"][:, k].mean()), rel=1e-12)
        assert r["sigma_std"][k] == pytest.approx(q.std(), rel=1e-9, abs=1e-12)
    assert np.median(r["accept_rate"]) > 0.02
    # deterministic per seed, different for another seed
    _, r2 = _run(c_oracle, cells, construct, ids, o, want_chain=True)
    np.testing.assert_array_equal(r["chain"], r2["chain"])
    o.seed = 10
    _, r3 = _run(c_oracle, cells, construct, ids, o, want_chain=True)
    assert not np.array_equal(r["chain"], r3["chain"])


def test_adapted_proposal_is_the_scaled_chain_covariance(c_oracle, cells, construct):
    """mcmcstat's covupd + chol: after the last adaptation row n >= burnintime, R'R =
    (2.4/sqrt(P))^2 (cov(chain rows 1..n) + qcovadj I) with the sample covariance of every row."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = [3, 150]
    o = DramOptions(n_steps=400, burnintime=200, adaptint=100, stats_from=1, seed=21)
    p, r = _run(c_oracle, cells, construct, ids, o, want_chain=True, want_R=True)
    n = cells.lengths[ids]
    for k in range(len(ids)):
        P = 7 + int(n[k])
        X = r["chain"][:400, k, :P]
        want = (2.4 ** 2 / P) * (np.cov(X.T, ddof=1) + 1e-5 * np.eye(P))
        R = r["R"][k, :P, :P]
        assert np.all(np.tril(R, -1) == 0)
        np.testing.assert_allclose(R.T @ R, want, rtol=1e-10, atol=1e-10 * np.abs(want).max())


def test_sigma2_gibbs_law(c_oracle, cells, construct):
    """1/s2 ~ Gamma(N/2, 2/SS(theta)): s2 N / SS has mean N/(N-2) (N = 2 N_c), the statistic the
    reference's raw-chain fixture satisfies (test_oracle_golden.py)."""
    from transcriptioncycleinference_amd.mcmc import DramOptions

    ids = [1, 100, 200, 250]
    o = DramOptions(n_steps=1500, burnintime=500, adaptint=100, stats_from=500, seed=4)
    p, r = _run(c_oracle, cells, construct, ids, o, want_chain=True)
    n = cells.lengths[ids]
    rows, cid, s2, nobs = [], [], [], []
    for row in range(1, 1500, 3):
        for k, c in enumerate(ids):
            rows.append(r["chain"][row, k, :7 + n[k]])
            cid.append(c)
            s2.append(r["s2chain"][row, k])
            nobs.append(2 * n[k])
    ss, st = c_oracle.ss_batch(cells.offsets, cells.t, cells.ms2, cells.pp7, construct, pack(rows),
                               np.array(cid, np.int32))
    assert np.all(st == 0)
    ratio = np.array(s2) * np.array(nobs) / ss
    nobs = np.array(nobs, np.float64)
    assert abs(ratio.mean() - np.mean(nobs / (nobs - 2))) < 0.012, ratio.mean()
    assert abs(ratio.std() - np.sqrt(np.mean(2 / nobs))) < 0.015, ratio.std()


def test_box_muller_pair_accuracy(c_oracle):
    """The normals' transcendental pair (the GPU's bm_neg2log / bm_sincospi, restated bit for bit):
    -2 log u within 2 ulp of libm's on 53-bit uniforms including both ends, sin / cos(2 pi u)
    within 3e-16 of a long-double reference (0 <= |.| <= 1), quarter turns exact."""
    import math

    rng = np.random.default_rng(1)
    n = 20000
    u = (np.floor(rng.random(n) * 2.0 ** 53) + 0.5) * 2.0 ** -53
    u1 = np.concatenate([u, 1 - np.arange(1, 200) * 2.0 ** -53, np.arange(1, 200) * 2.0 ** -53 + 2.0 ** -54])
    quarter = np.arange(1, 8) / 8.0
    u2 = np.concatenate([u[::-1], quarter, [2.0 ** -53, 1 - 2.0 ** -53]])
    lg, _, _ = c_oracle.box_muller_pair(u1, u1[:1])
    ref = np.array([-2.0 * math.log(v) for v in u1])
    assert np.max(np.abs(lg - ref) / np.spacing(np.abs(ref))) <= 2.0
    _, sn, cs = c_oracle.box_muller_pair(u2[:1], u2)
    pil = np.longdouble("3.14159265358979323846264338327950288")
    th = 2 * pil * u2.astype(np.longdouble)
    assert np.max(np.abs((sn - np.sin(th)).astype(np.float64))) < 3e-16
    assert np.max(np.abs((cs - np.cos(th)).astype(np.float64))) < 3e-16
    k = len(u)
    np.testing.assert_array_equal(sn[k + 1:k + 7:2], [1.0, 0.0, -1.0])  # quarter turns: r = 0
    np.testing.assert_array_equal(cs[k + 1:k + 7:2], [0.0, -1.0, 0.0])
