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


def test_result_files_match_reference_schema(tmp_path, cells):
    """MCMCresults/MCMCplot/MCMCchain field sets and file names (TranscriptionCycleMCMC.m:149-157,373-378)."""
    import scipy.io as sio

    from transcriptioncycleinference_amd.mcmc import (CHAIN_FIELDS, PLOT_FIELDS, RESULT_FIELDS, FitResult,
                                                      save_results)

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
    assert set(d["MCMCresults"]._fieldnames) == set(RESULT_FIELDS)
    assert set(d["MCMCplot"]._fieldnames) == set(PLOT_FIELDS)
    raw = sio.loadmat(b, struct_as_record=False, squeeze_me=True)["MCMCchain"]
    assert set(raw._fieldnames) == set(CHAIN_FIELDS) and raw.dR_chain.shape == (5, n)


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
