"""Pin the CPU oracle to the reference's own data before trusting it (CPU only).

Known-answer vectors: ``28-Oct-2020-TestData.mat`` holds ``MCMCplot(c).simMS2/simPP7``, the
reference's forward model at the posterior means (``TranscriptionCycleMCMC.m:307-309``), for
all 299 cells. Statistical pin of the full SS (grid + interp1 + nansum): mcmcstat draws
``1/s2 ~ Gamma(N/2, 2/SS)`` with N = length(ydata) = 2 N_c (``:260``), so over the 2,691
post-initial chain rows ``s2 * 2N_c / SS(theta)`` must have mean N/(N-2) ~ 1.008 and sd
sqrt(2/N) ~ 0.091.
"""
import numpy as np
import pytest

from conftest import pack
from oracle import oracle as O


def test_forward_at_means_matches_reference_exactly(cells, means, construct):
    off = cells.offsets
    worst = 0.0
    for c in range(cells.n_cells):
        t = cells.t[off[c]:off[c + 1]]
        ms2, pp7 = O.forward_raw(construct, t, means["rows"][c])
        exp_m = means["sim_ms2"][off[c]:off[c + 1]]
        exp_p = means["sim_pp7"][off[c]:off[c + 1]]
        worst = max(worst, np.max(np.abs(ms2 - exp_m) / np.abs(exp_m)), np.max(np.abs(pp7 - exp_p) / np.abs(exp_p)))
    assert worst <= 1e-12, worst  # observed: 0 (bit-exact)


def test_c_oracle_matches_reference_goldens_and_numpy(cells, means, construct, c_oracle):
    off = cells.offsets
    for c in range(0, cells.n_cells, 7):
        t = cells.t[off[c]:off[c + 1]]
        m, p = c_oracle.forward(t, construct, means["rows"][c], mode=0)
        np.testing.assert_array_equal(m, means["sim_ms2"][off[c]:off[c + 1]])
        np.testing.assert_array_equal(p, means["sim_pp7"][off[c]:off[c + 1]])
        mi, pi = c_oracle.forward(t, construct, means["rows"][c], mode=1)
        mn, pn = O.forward_interp(construct, t, means["rows"][c])
        np.testing.assert_array_equal(mi, mn)
        np.testing.assert_array_equal(pi, pn)


def test_grid_length_equals_data_length(cells, c_oracle):
    """t(1):mean(diff(t)):t(end) has N points ending at t(end) for every TestData cell."""
    for c in range(cells.n_cells):
        t = cells.cell(c)[0]
        g = O.interp_grid(t)
        assert len(g) == len(t) and g[0] == t[0] and g[-1] == t[-1]
        np.testing.assert_array_equal(c_oracle.interp_grid(t), g)


def test_committed_ss_goldens_reproduce(cells, chain, construct, c_oracle):
    theta = pack(chain["rows"])
    ss, st = c_oracle.ss_batch(cells.offsets, cells.t, cells.ms2, cells.pp7, construct, theta, chain["cell_id"])
    assert np.all(st == 0)
    np.testing.assert_array_equal(ss, chain["ss"])
    # numpy restatement on a subset (slow path)
    for b in range(0, len(theta), 97):
        c = int(chain["cell_id"][b])
        assert O.sum_of_squares(construct, cells.data_struct(c), chain["rows"][b]) == chain["ss"][b]


def test_s2chain_statistical_pin(cells, chain):
    lens = cells.lengths
    post = chain["step"] > 0
    ratio = chain["s2"][post] * 2 * lens[chain["cell_id"][post]] / chain["ss"][post]
    assert len(ratio) == 2691
    n2 = 2 * lens[chain["cell_id"][post]]
    assert abs(ratio.mean() - np.mean(n2 / (n2 - 2))) < 0.01, ratio.mean()  # 1.0075 observed
    assert abs(ratio.std() - np.mean(np.sqrt(2 / n2))) < 0.01, ratio.std()  # 0.0911 observed


def _gibbs_loglik(s2, ss, n_obs, N0, S20=1.0):
    """Log-density of the precisions 1/s2 under mcmcstat's sigma^2 Gibbs update with the prior
    (N0, S20): 1/s2 ~ Gamma((N0 + N)/2, scale 2/(N0 S20 + SS)) (the Jacobian of 1/s2 is the same
    under every hypothesis, so ratios of this are likelihood ratios of the draws)."""
    from scipy.special import gammaln

    y = 1.0 / s2
    k, th = (N0 + n_obs) / 2.0, 2.0 / (N0 * S20 + ss)
    return float(np.sum((k - 1) * np.log(y) - y / th - gammaln(k) - k * np.log(th)))


def test_sigma2_prior_weight_is_pinned_by_the_reference_draws(cells, chain):
    """mcmcstat's N0 / S20 defaults are not vendored (README.md:5); the reference sets only
    model.sigma2 = 1 and model.N (TranscriptionCycleMCMC.m:259-260). The 2,691 post-initial s2chain
    draws of the reference's own run, with the SS of the state they were drawn at, decide between
    the two candidate priors: the exact Gamma log-likelihood favours N0 = 0 (what the sampler and its
    restatement implement, oracle/tci_dram_oracle.c) over N0 = 1, S20 = sigma2_0 = 1 by 1.77 nats
    (likelihood ratio ~5.9), and excludes N0 >= 2 (>= 9 nats). The maximum over N0 on a grid lies in
    [0, 0.5]. DESIGN.md §5 records the decision."""
    lens = cells.lengths
    post = chain["step"] > 0
    s2, ss = chain["s2"][post], chain["ss"][post]
    n_obs = 2.0 * lens[chain["cell_id"][post]]          # model.N = length(ydata), NaNs counted (:260)
    l0 = _gibbs_loglik(s2, ss, n_obs, 0.0)
    l1 = _gibbs_loglik(s2, ss, n_obs, 1.0)
    assert l0 - l1 > 1.5, l0 - l1                         # 1.77 observed
    assert l0 - _gibbs_loglik(s2, ss, n_obs, 2.0) > 8.0   # 9.08 observed
    grid = np.arange(-2.0, 4.01, 0.25)
    best = grid[int(np.argmax([_gibbs_loglik(s2, ss, n_obs, g) for g in grid]))]
    assert 0.0 <= best <= 0.5, best


def test_colon_rule_properties():
    v = O.matlab_colon(0.0, 0.1, 1.0)
    assert len(v) == 11 and v[-1] == 1.0 and v[0] == 0.0
    assert len(O.matlab_colon(1.0, 1.0, 5.5)) == 5
    assert len(O.matlab_colon(2.0, 3.0, 11.0)) == 4
    assert len(O.matlab_colon(1.0, -1.0, 5.0)) == 0
    assert np.isnan(O.matlab_colon(0.0, np.nan, 1.0)[0])


def test_oracle_quirks(construct):
    """Semantics the kernels must reproduce."""
    t = np.linspace(0, 10, 41)
    th = np.concatenate([[2.0, 1.0, 0.0, 0.0, 0.0, 1.0, 5.0], np.zeros(41)])
    # dR_N never enters the SS
    th2 = th.copy()
    th2[-1] = 29.0
    d = {"xdata": t, "ydata": np.concatenate([np.ones(41), np.ones(41)])}
    assert O.sum_of_squares(construct, d, th) == O.sum_of_squares(construct, d, th2)
    # basal is a floor, not an offset: a huge basal dominates everything
    th3 = th.copy()
    th3[3] = 49.0
    m, _ = O.forward_raw(construct, t, th3)
    assert np.all(m >= 49.0 * th3[5]) and np.min(m) == 49.0
    # onset after the last time point: nothing is loaded, signal == floor
    th4 = th.copy()
    th4[2] = 10.0
    m, p = O.forward_raw(construct, t, th4)
    assert np.all(m == 0) and np.all(p == 0)


def test_position_matrix_shape_and_forward_accumulation():
    """x is m x floor(sum(R.*dt)); loaded columns advance by v*dt(i) per step (ConstantElongationSim.m:47-64)."""
    t = np.array([0.0, 1.0, 2.0, 3.5])
    x = O.constant_elongation_sim(1.0, 0.5, np.array([1.5, 1.5, 2.0, -7.0]), t)
    assert x.shape == (4, 6)  # floor(1.5 + 1.5 + 3.0)
    # step 1 (t=0 < ton) skipped; step 2 loads floor(1.5)=1; step 3 loads floor(4.5)=4
    np.testing.assert_array_equal(x[2], [1.0, 0, 0, 0, 0, 0])
    np.testing.assert_array_equal(x[3], [2.5, 1.5, 1.5, 1.5, 0, 0])


def test_counter_never_passes_the_column_count():
    """MATLAB errors ("Index exceeds matrix dimensions", ConstantElongationSim.m:61-64) if
    floor(counter) > n = floor(sum(R.*dt)) (:47). With sum taken left to right -- the oracle's
    restatement of :47 -- that cannot happen: the products are >= 0 and rounding is monotone, so
    every partial sum of ALL steps is >= the ton-gated counter after the same step.
    Checked here on adversarial sequences: tiny leading terms that the gate removes, terms that
    accumulate to just below / above integers (0.1 steps), huge-then-tiny mixes."""
    rng = np.random.default_rng(47)
    for trial in range(4000):
        m = int(rng.integers(2, 200))
        kind = trial % 4
        if kind == 0:
            p = np.full(m, 0.1)
        elif kind == 1:
            p = rng.random(m) * 10.0 ** rng.integers(-18, 3, m)
        elif kind == 2:
            p = np.where(rng.random(m) < 0.5, 1e-16, rng.random(m) * 3)
        else:
            p = rng.integers(0, 4, m) * 0.1 + rng.choice([0.0, 2.0 ** -52, 2.0 ** -50], m)
        gate = int(rng.integers(0, m))          # steps before `gate` are t(i) < ton
        s, c = 0.0, 0.0
        for i in range(m):
            s = s + p[i]
            if i >= gate:
                c = c + p[i]
            assert s >= c
        assert np.floor(c) <= np.floor(s)


def test_oracle_never_raises_the_index_error(construct, c_oracle):
    """The same property through the oracle's own check (OR_EIDX = -2, tci_oracle.c): rates that
    clamp to 0 or to tiny values before the onset, 0.1-min steps, onsets on and between grid points."""
    n = 121
    t = np.arange(n) * 0.1
    off = np.array([0, n])
    y = np.ones(n)
    rng = np.random.default_rng(61)
    rows = []
    for k in range(400):
        dR = rng.choice([-15.0, -10.0 + 1e-13, 0.0, 0.5], n) + (rng.random(n) < 0.3) * rng.normal(0, 2, n)
        rows.append(np.concatenate([[2.0, 1.0, (k % 40) * 0.05, 1.0, 1.0, 0.5, 10.0], np.clip(dR, -30, 30)]))
    ss, st = c_oracle.ss_batch(off, t, y, y, construct, pack(rows), np.zeros(len(rows), np.int32))
    assert np.all(st == 0), np.unique(st)
    assert np.all(np.isfinite(ss))


@pytest.mark.parametrize("n", [2, 3, 65, 66, 129, 200])
def test_oracles_agree_on_random_theta(n, construct, c_oracle):
    rng = np.random.default_rng(n)
    from transcriptioncycleinference_amd.data import draw_x0, synthetic_times

    t = synthetic_times(rng, n)
    y1 = rng.normal(3, 2, n)
    y2 = rng.normal(6, 3, n)
    y1[rng.random(n) < 0.3] = np.nan
    off = np.array([0, n])
    rows = [draw_x0(rng, n) for _ in range(6)]
    ss, st = c_oracle.ss_batch(off, t, y1, y2, construct, pack(rows), np.zeros(6, np.int32))
    assert np.all(st == 0)
    d = {"xdata": t, "ydata": np.concatenate([y1, y2])}
    for i, r in enumerate(rows):
        assert ss[i] == O.sum_of_squares(construct, d, r)
