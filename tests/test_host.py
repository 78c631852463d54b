"""Host-side logic: dataset ingestion, truncation, constructs, theta helpers, sharding (CPU)."""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN


def test_testdata_fixture_shape(cells):
    assert cells.n_cells == 299
    assert int(cells.lengths.sum()) == 35928
    assert cells.lengths.min() == 113 and cells.lengths.max() == 129
    assert np.isnan(cells.ms2).sum() + np.isnan(cells.pp7).sum() == 26645
    for c in range(cells.n_cells):
        t = cells.cell(c)[0]
        assert t[0] == 0 and np.all(np.diff(t) > 0)


def test_data_struct_matches_reference_layout(cells):
    d = cells.data_struct(5)
    t, m, p = cells.cell(5)
    np.testing.assert_array_equal(d["xdata"], t)
    np.testing.assert_array_equal(d["ydata"], np.concatenate([m, p]))


def test_truncation_rule():
    from transcriptioncycleinference_amd.data import truncate

    t = np.array([0.0, 1.0, 2.0, 3.0, 4.0])
    y = t * 10
    tt, m, _ = truncate(t, y, y, 1.0, 3.0)  # t >= 1 and t < 3
    np.testing.assert_array_equal(tt, [1.0, 2.0])
    np.testing.assert_array_equal(m, [10.0, 20.0])
    tt, _, _ = truncate(t, y, y, 0.0, math.inf)
    assert len(tt) == 5
    tt, _, _ = truncate(t, y, y, 10.0, math.inf)
    assert len(tt) == 0


def test_load_mat_roundtrip(tmp_path, cells):
    import scipy.io as sio

    from transcriptioncycleinference_amd.data import load_mat

    recs = np.empty(3, dtype=[("time", object), ("MS2", object), ("PP7", object), ("name", object)])
    for c in range(3):
        t, m, p = cells.cell(c)
        recs[c] = (t[None, :], m[None, :], p[None, :], "TestData")
    path = os.path.join(tmp_path, "ds.mat")
    sio.savemat(path, {"data": recs})
    got = load_mat(path)
    assert got.n_cells == 3 and got.name == "TestData"
    for c in range(3):
        for a, b in zip(got.cell(c), cells.cell(c)):
            np.testing.assert_array_equal(a, b)
    got2 = load_mat(path, t_start=5.0, t_end=20.0)
    t = got2.cell(0)[0]
    assert t.min() >= 5.0 and t.max() < 20.0


def test_construct_validation():
    from transcriptioncycleinference_amd.construct import Construct, builtin_construct, long_two_loop_construct

    c = builtin_construct("P2P-MS2v5-LacZ-PP7v4")
    c.validate()
    assert c.n_seg == 1 and c.L0 == 6.626
    long_two_loop_construct().validate()
    with pytest.raises(ValueError):
        builtin_construct("unknown")
    with pytest.raises(ValueError):
        Construct(6.0, [1.0], [0.5], [24], [2.0], [3.0], [24]).validate()
    with pytest.raises(ValueError):
        Construct(6.0, [-0.1], [0.5], [24], [2.0], [3.0], [24]).validate()
    with pytest.raises(ValueError):
        Construct(6.0, [0.1] * 5, [0.5] * 5, [24] * 5, [2.0] * 5, [3.0] * 5, [24] * 5).validate()


def test_x0_and_bounds():
    from transcriptioncycleinference_amd.data import draw_x0, in_bounds

    rng = np.random.default_rng(0)
    for _ in range(50):
        x0 = draw_x0(rng, 120)
        assert len(x0) == 127
        assert 1 <= x0[0] <= 3 and 0 <= x0[1] <= 4 and 0 <= x0[2] <= 4
        assert list(x0[3:5]) == [10.0, 5.0] and x0[6] == 15.0
    x = draw_x0(rng, 10)
    x[7:] = 0
    assert in_bounds(x, 10)
    x[0] = 10.5
    assert not in_bounds(x, 10)


def test_synthetic_times_match_survey_spec():
    from transcriptioncycleinference_amd.data import synthetic_times

    rng = np.random.default_rng(20201028)
    t = synthetic_times(rng, 200)
    d = np.diff(t)
    assert len(t) == 200 and t[0] == 0 and np.all(d > 0.23) and np.all(d < 0.72)
    assert abs(np.median(d) - 0.2454) < 0.01


def test_shard_bounds_cover_and_balance():
    from transcriptioncycleinference_amd.parallel import shard_bounds

    for n, world in [(299, 1), (299, 2), (299, 8), (10000, 8), (5, 8), (0, 3)]:
        w = np.random.default_rng(n).integers(100, 200, n)
        b = shard_bounds(w, world)
        assert b[0] == 0 and b[-1] == n and np.all(np.diff(b) >= 0) and len(b) == world + 1
        if n >= 8 * world:
            loads = [w[b[r]:b[r + 1]].sum() for r in range(world)]
            assert max(loads) <= w.sum() / world + w.max()


def test_golden_files_are_plain_arrays():
    for f in ("testdata.npz", "forward_means.npz", "chain_theta.npz"):
        z = np.load(os.path.join(GOLDEN, f), allow_pickle=False)
        for k in z.files:
            assert z[k].dtype != object


def test_product_package_never_imports_oracle():
    import pathlib

    pkg = pathlib.Path(__file__).resolve().parent.parent / "transcriptioncycleinference_amd"
    for p in pkg.rglob("*.py"):
        src = p.read_text()
        assert "import oracle" not in src and "from oracle" not in src, p


def test_missing_library_fails_loudly(tmp_path):
    from transcriptioncycleinference_amd import _lib

    with pytest.raises(_lib.TciLibraryMissing):
        _lib.load(str(tmp_path / "libtci.so"))


def _schema():
    import json

    with open(os.path.join(GOLDEN, "result_schema.json")) as f:
        return json.load(f)


def test_result_field_lists_are_the_reference_files_own():
    """RESULT/PLOT/CHAIN_FIELDS equal, in order, the field lists of the reference's own result files
    (28-Oct-2020-TestData*.mat, extracted by tests/golden/make_golden.py --schema)."""
    from transcriptioncycleinference_amd.mcmc import CHAIN_FIELDS, PLOT_FIELDS, RESULT_FIELDS

    sc = _schema()
    assert list(RESULT_FIELDS) == sc["results_file"]["MCMCresults"]
    assert list(PLOT_FIELDS) == sc["results_file"]["MCMCplot"]
    assert list(CHAIN_FIELDS) == sc["rawchain_file"]["MCMCchain"]


def test_result_files_match_reference_schema(tmp_path, cells):
    """The two files the writer makes hold the variables and struct fields (in order) of the
    reference's own files (TranscriptionCycleMCMC.m:149-157,373-378; tests/golden/result_schema.json)."""
    import scipy.io as sio

    from transcriptioncycleinference_amd.mcmc import CHAIN_FIELDS, RESULT_FIELDS, FitResult, save_results

    sc = _schema()
    n = int(cells.lengths[0])
    t, m, p = cells.cell(0)
    res = {f: 1.0 for f in RESULT_FIELDS}
    res.update(mean_dR=np.zeros(n), sigma_dR=np.ones(n), cell_index=1, ApprovedFits=0)
    plot = {"t_plot": t, "MS2_plot": m, "PP7_plot": p, "simMS2": np.ones(n), "simPP7": np.ones(n)}
    chain = {f: np.arange(5.0) for f in CHAIN_FIELDS}
    chain["dR_chain"] = np.zeros((5, n))
    fr = FitResult("TestData", [res], [plot], [chain], np.zeros(1), 0, 0.0)
    a, b = save_results(fr, str(tmp_path), date="28-Oct-2020")
    assert a.endswith("28-Oct-2020-TestData.mat") and b.endswith("28-Oct-2020-TestData_RawChain.mat")
    d = sio.loadmat(a, struct_as_record=False, squeeze_me=True)
    assert sorted(k for k in d if not k.startswith("__")) == sc["results_file"]["variables"]
    assert list(d["MCMCresults"]._fieldnames) == sc["results_file"]["MCMCresults"]
    assert list(d["MCMCplot"]._fieldnames) == sc["results_file"]["MCMCplot"]
    assert d["DatasetName"] == "TestData"
    raw = sio.loadmat(b, struct_as_record=False, squeeze_me=True)
    assert sorted(k for k in raw if not k.startswith("__")) == sc["rawchain_file"]["variables"]
    assert list(raw["MCMCchain"]._fieldnames) == sc["rawchain_file"]["MCMCchain"]
    assert raw["MCMCchain"].dR_chain.shape == (5, n)


def _previous_file(tmp_path, cells, entries):
    """A results file in the reference's schema holding MCMCresults entries
    {cell_index: (mean_v, ApprovedFits)} (mean_v None -> MATLAB [])."""
    from transcriptioncycleinference_amd.mcmc import RESULT_FIELDS, FitResult, save_results

    res, plots = [], []
    for ci, (v, ap) in entries.items():
        n = int(cells.lengths[ci - 1])
        r = {f: 0.5 for f in RESULT_FIELDS}
        r.update(mean_v=np.zeros((0, 0)) if v is None else v, mean_dR=np.zeros(n), sigma_dR=np.zeros(n),
                 cell_index=ci, ApprovedFits=ap)
        res.append(r)
        t, m, p = cells.cell(ci - 1)
        plots.append({"t_plot": t, "MS2_plot": m, "PP7_plot": p, "simMS2": m, "simPP7": p})
    fr = FitResult("Prev", res, plots, [{} for _ in res], np.zeros(len(res)), 0, 0.0)
    return save_results(fr, str(tmp_path), date="01-Jan-2021")[0]


def test_load_previous_keys_by_cell_index_and_skips_gaps(tmp_path, cells):
    """loadPrevious (TranscriptionCycleMCMC.m:84-107,193-198,345-350): each cell takes the mean_v of
    the entry whose cell_index matches it; cells with no entry, or an empty mean_v, are skipped;
    ApprovedFits is carried over. Entries out of order and with gaps, read by cell, never by position."""
    from transcriptioncycleinference_amd.mcmc import PreviousFit, load_previous, load_previous_v, plan_fit

    entries = {5: (2.5, 1), 1: (1.25, 0), 2: (None, 1), 4: (1.75, -1), 7: (2.0, 1)}   # 3 and 6 missing
    path = _previous_file(tmp_path, cells, entries)
    prev = load_previous(path)
    assert set(prev) == {1, 2, 4, 5, 7}
    assert prev[5] == PreviousFit(2.5, 1) and prev[4] == PreviousFit(1.75, -1) and prev[2].mean_v is None
    assert load_previous_v(path) == {1: 1.25, 4: 1.75, 5: 2.5, 7: 2.0}
    for ids in (range(8), [4, 5, 6, 3]):          # the whole dataset, and one shard of it
        plan = plan_fit(cells, list(ids), seed=3, v0=prev)
        want = [c for c in ids if c + 1 in (1, 4, 5, 7)]
        assert plan.cells == want
        for k, c in enumerate(plan.cells):
            v = entries[c + 1][0]
            assert plan.x0[k, 0] == v
            assert plan.lower[k, 0] == v - 1e-5 and plan.upper[k, 0] == v + 1e-5 and plan.qcov_diag[k, 0] == 1e-7
            assert plan.approved[k] == entries[c + 1][1]
    # the mean_v-only mapping, and an explicit ApprovedFits override by cell_index
    plan = plan_fit(cells, range(8), seed=3, v0=load_previous_v(path), approved={5: 7})
    assert plan.cells == [0, 3, 4, 6] and plan.approved == [0, 0, 7, 0]
    # a sequence over ALL cells is read by 0-based cell index (also inside a shard)
    seq = [None, 1.5, float("nan"), 2.0, None, None]
    plan = plan_fit(cells, [3, 1, 2], seed=3, v0=seq)
    assert plan.cells == [3, 1] and list(plan.x0[:, 0]) == [2.0, 1.5]
    # x0 of a cell does not depend on which other cells are fitted (keyed by cell)
    a = plan_fit(cells, [3], seed=3, v0=seq)
    np.testing.assert_array_equal(a.x0[0], plan.x0[0, :a.x0.shape[1]])


class _FakeLk:
    """Stands in for a Likelihood on CPU: fit()'s host logic only (the sampler is monkeypatched)."""

    def __init__(self, cells):
        self.cells = cells

    def forward(self, theta, cid, grid="raw"):
        n = theta.shape[1]
        return np.zeros((len(cid), n)), np.zeros((len(cid), n))


def test_fit_with_load_previous_end_to_end_host_logic(tmp_path, cells, monkeypatch):
    """The documented call fit(lk, v0=load_previous(path)) builds one chain per cell found in the
    file, at v0 +- 1e-5, carries ApprovedFits into MCMCresults, prunes the rest, and leaves the
    caller's DramOptions untouched (the sampler itself is stubbed: it runs on the GPU)."""
    from transcriptioncycleinference_amd import mcmc

    seen = {}

    def fake_dram_run(lk, cell_id, x0, lo, hi, mu, sg, J0, s20, o, want_qcov=False, chain_keys=None):
        seen.update(cell_id=cell_id.copy(), lo=lo.copy(), hi=hi.copy(), opts=o, keys=chain_keys.copy())
        n, ld = x0.shape
        z = np.zeros((n, ld))
        return mcmc.DramResult(x0.copy(), z, x0.copy(), np.ones(n), z[:, 0], np.full(n, 0.3),
                               np.ones(n, np.int64), None, None, 1.0)

    monkeypatch.setattr(mcmc, "dram_run", fake_dram_run)
    path = _previous_file(tmp_path, cells, {2: (1.5, 1), 4: (2.25, 0), 9: (1.0, -1)})
    opts = mcmc.DramOptions(engine="walk")
    before = dict(vars(opts))
    sub = cells.subset(range(10))
    fr = mcmc.fit(_FakeLk(sub), n_steps=50, n_burn=10, seed=1, v0=mcmc.load_previous(path), opts=opts)
    assert vars(opts) == before
    assert seen["opts"].engine == "walk" and seen["opts"].n_steps == 50
    assert list(seen["cell_id"]) == [1, 3, 8] and list(seen["keys"]) == [1, 3, 8]
    np.testing.assert_array_equal(seen["lo"][:, 0], np.array([1.5, 2.25, 1.0]) - 1e-5)
    assert [r["cell_index"] for r in fr.MCMCresults] == [2, 4, 9]
    assert [r["ApprovedFits"] for r in fr.MCMCresults] == [1, 0, -1]
    assert [r["mean_v"] for r in fr.MCMCresults] == [1.5, 2.25, 1.0]
    # a results file written from this fit can seed the next round (the reference's hierarchy)
    a, _ = mcmc.save_results(fr, str(tmp_path / ".."), date="02-Jan-2021")
    assert {c: (p.mean_v, p.ApprovedFits) for c, p in mcmc.load_previous(a).items()} == \
        {2: (1.5, 1), 4: (2.25, 0), 9: (1.0, -1)}


def test_cell_weights_follow_rows_times_window(cells):
    """Shard weights ~ N_c x W_c: W_c = (L0 + tau v)/(v d_c) at the prior means."""
    from transcriptioncycleinference_amd.parallel import cell_weights

    w = cell_weights(cells)
    for c in (0, 17, 298):
        t = cells.cell(c)[0]
        n = len(t)
        d = (t[-1] - t[0]) / (n - 1)
        assert w[c] == pytest.approx(n * min((6.626 + 2.0 * 2.0) / (2.0 * d), n))
    wv = cell_weights(cells, v0={1: 4.0})   # a faster previous rate: shorter window
    assert wv[0] < w[0] and np.all(wv[1:] == w[1:])
    # the round-1 signature (an array of point counts) still works: weights N_c
    np.testing.assert_array_equal(cell_weights(cells.lengths), cells.lengths.astype(np.float64))
    with pytest.raises(ValueError):
        cell_weights(cells, v0=[2.0] * 10)   # a sequence must cover every cell


def test_cell_setup_matches_reference_initialisation():
    from transcriptioncycleinference_amd.mcmc import cell_setup

    t = np.linspace(0, 30, 120)
    x0, lo, hi, mu, sig, J0 = cell_setup(t, np.random.default_rng(0), 50.0)
    assert len(x0) == 127 and np.all(x0 >= lo) and np.all(x0 <= hi)
    assert list(lo[:7]) == [0, 0, 0, 0, 0, 0, 0] and list(hi[:7]) == [10, 20, 10, 50, 50, 1, 40]
    assert np.all(lo[7:] == -30) and np.all(hi[7:] == 30)
    assert np.all(np.isinf(sig[:7])) and np.all(sig[7:] == 50) and np.all(mu == 0)
    np.testing.assert_allclose(J0[:7], [0.05, 0.1, t[-1] - t[-2], 1, 1, 0.05, 0.5])
    x0, lo, hi, _, _, J0 = cell_setup(t, np.random.default_rng(0), 50.0, v0=2.5)
    assert x0[0] == 2.5 and lo[0] == 2.5 - 1e-5 and hi[0] == 2.5 + 1e-5 and J0[0] == 1e-7
