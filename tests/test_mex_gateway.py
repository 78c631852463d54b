"""The MATLAB MEX gateway (matlab/tci_mex.cpp) executed through the stand-in MATLAB API
(matlab/mexstub/, MATLAB itself is absent): argument checks and error identifiers on CPU; on the
GPU the SS / forward results of `tci_mex` against the Python binding of the same C ABI, bit for bit,
with MATLAB's conventions -- column-major P x B theta, 1-based cells, logical or double `active`.
The gateway stands in for the reference's ssfun hook (TranscriptionCycleMCMC.m:186,258)."""
import os

import numpy as np
import pytest

from conftest import ROOT, pack
from mexharness import Mex, MexError, MxPtr

DATA_FIELDS = ["time", "MS2", "PP7", "name"]


@pytest.fixture(scope="module")
def mex():
    from transcriptioncycleinference_amd.build import MEX_STUB, build_library, build_mex_stub

    build_library()
    srcs = [os.path.join(ROOT, "matlab", "tci_mex.cpp")] + [
        os.path.join(ROOT, "matlab", "mexstub", f) for f in ("mex.h", "matrix.h", "mexstub.cpp")]
    if not os.path.exists(MEX_STUB) or any(os.path.getmtime(s) > os.path.getmtime(MEX_STUB) for s in srcs):
        build_mex_stub()
    m = Mex(MEX_STUB)
    yield m
    m.clear()


def data_struct(mex, cells, ids):
    rows = []
    for c in ids:
        t, m, p = cells.cell(c)
        rows.append({"time": t, "MS2": m, "PP7": p, "name": "TestData"})
    return MxPtr(mex, mex.struct(rows, DATA_FIELDS))


def expect(ident, fn, *a, **k):
    with pytest.raises(MexError) as e:
        fn(*a, **k)
    assert e.value.ident == ident, (e.value.ident, e.value.msg)
    return e.value


# ---- CPU: everything the gateway checks before a pointer reaches the C ABI -------------------


def test_commands_and_handles_are_checked(mex):
    expect("tci:arg", mex.call, 3.0)                        # first argument must be a command
    expect("tci:arg", mex.call, "no_such_command")
    expect("tci:handle", mex.call, "ss", MxPtr(mex, mex.handle(12345)), 1.0, np.zeros(130))
    expect("tci:handle", mex.call, "ss", 7.0, 1.0, np.zeros(130))   # a double is not a handle
    expect("tci:handle", mex.call, "destroy", MxPtr(mex, mex.handle(0xdeadbeef)))
    expect("tci:arg", mex.call, "ss", nlhs=1)              # wrong argument count


def test_create_checks_data_and_construct(mex, cells):
    expect("tci:arg", mex.call, "create")
    expect("tci:data", mex.call, "create", np.zeros(3), "P2P-MS2v5-LacZ-PP7v4")   # not a struct
    d = data_struct(mex, cells, [0, 1])
    try:
        expect("tci:construct", mex.call, "create", d, "P2P-other")              # GetFluorFromPolPos.m:18
        expect("tci:construct", mex.call, "create", d, 5.0)
        bad = MxPtr(mex, mex.struct([{"L0": 6.626, "MS2_start": [0.0, 1.0], "MS2_end": [0.5], "MS2_loopn": [24.0],
                                      "PP7_start": [4.0], "PP7_end": [5.0], "PP7_loopn": [24.0]}],
                                    ["L0", "MS2_start", "MS2_end", "MS2_loopn", "PP7_start", "PP7_end", "PP7_loopn"]))
        expect("tci:construct", mex.call, "create", d, bad)
        bad.free()
    finally:
        d.free()
    t, m, p = cells.cell(0)
    ragged = MxPtr(mex, mex.struct([{"time": t, "MS2": m[:-1], "PP7": p}], DATA_FIELDS))
    expect("tci:data", mex.call, "create", ragged, "P2P-MS2v5-LacZ-PP7v4")      # lengths differ
    ragged.free()
    nofield = MxPtr(mex, mex.struct([{"time": t, "MS2": m}], ["time", "MS2"]))
    expect("tci:data", mex.call, "create", nofield, "P2P-MS2v5-LacZ-PP7v4")     # no PP7
    nofield.free()


def test_device_count_and_create_without_a_gpu(mex, cells):
    n = mex.call("device_count")[0]
    assert n.shape == (1, 1) and n[0, 0] >= 0
    if n[0, 0] == 0:  # this container: the host-side validation passes, the HIP context cannot exist
        d = data_struct(mex, cells, [0])
        e = expect("tci:create", mex.call, "create", d, "P2P-MS2v5-LacZ-PP7v4", 0.0)
        d.free()
        assert "hip" in e.msg.lower()


# ---- GPU: the gateway's results against the Python binding of the same ABI -------------------


@pytest.fixture(scope="module")
def gw(mex, cells):
    d = data_struct(mex, cells, range(cells.n_cells))
    h = mex.call("create", d, "P2P-MS2v5-LacZ-PP7v4", 0.0)[0]
    d.free()
    yield MxPtr(mex, mex.handle(int(h[0, 0])))


@pytest.fixture(scope="module")
def lk(cells):
    from transcriptioncycleinference_amd import Likelihood

    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4", device=0) as L:
        yield L


@pytest.mark.gpu
def test_ss_one_based_cells_equals_the_binding(mex, gw, lk, chain, cells):
    rows = [(int(chain["cell_id"][b]), chain["rows"][b]) for b in range(0, len(chain["rows"]), 37)]
    want = lk.ss_batch(pack([r for _, r in rows], 136), np.array([c for c, _ in rows], np.int32))
    got = np.array([mex.call("ss", gw, float(c + 1), r)[0][0, 0] for c, r in rows])   # MATLAB cell c+1
    np.testing.assert_array_equal(got, want)
    np.testing.assert_allclose(got, chain["ss"][::37], rtol=1e-10, atol=0)             # the oracle goldens (contract 1e-6)
    expect("tci:arg", mex.call, "ss", gw, 0.0, rows[0][1])        # cells are 1-based
    expect("tci:arg", mex.call, "ss", gw, 1.5, rows[0][1])
    expect("tci:call", mex.call, "ss", gw, 300.0, rows[0][1])     # 299 cells: TCI_ERANGE
    expect("tci:call", mex.call, "ss", gw, 1.0, rows[0][1][:50])  # x shorter than 7 + N


@pytest.mark.gpu
def test_ss_batch_column_major_and_active_masks(mex, gw, lk, chain):
    B = 300
    theta = pack(chain["rows"][:B], 136)
    cid = np.asarray(chain["cell_id"][:B], np.int32)
    want = lk.ss_batch(theta, cid)
    X = theta.T                                   # P x B: one theta per COLUMN, as mcmcstat holds them
    got = mex.call("ss_batch", gw, (cid + 1).astype(np.float64), X)[0]
    assert got.shape == (B, 1)
    np.testing.assert_array_equal(got[:, 0], want)
    act = (np.arange(B) % 3) != 0
    lg = MxPtr(mex, mex.logical(act))
    got_l = mex.call("ss_batch", gw, (cid + 1).astype(np.float64), X, lg)[0][:, 0]
    lg.free()
    got_d = mex.call("ss_batch", gw, (cid + 1).astype(np.float64), X, act.astype(np.float64) * 2.5)[0][:, 0]
    for g in (got_l, got_d):
        np.testing.assert_array_equal(g[act], want[act])
        assert np.all(np.isposinf(g[~act]))      # skipped proposals
    expect("tci:arg", mex.call, "ss_batch", gw, (cid[:10] + 1).astype(np.float64), X)   # B mismatch
    expect("tci:arg", mex.call, "ss_batch", gw, (cid + 1).astype(np.float64), X, act[:5].astype(np.float64))
    expect("tci:arg", mex.call, "ss_batch", gw, cid.astype(np.float64) + 0.5, X)        # non-integer cells


@pytest.mark.gpu
def test_forward_raw_and_interp(mex, gw, lk, means, cells):
    for c in (0, 150, 298):
        x = means["rows"][c]
        for mode in ("raw", "interp"):
            ms2, pp7 = mex.call("forward", gw, float(c + 1), x, mode, nlhs=2)
            wm, wp = lk.forward(x[None, :], np.array([c], np.int32), grid=mode)
            n = int(cells.lengths[c])
            assert ms2.shape == (1, n)
            np.testing.assert_array_equal(ms2[0], wm[0, :n])
            np.testing.assert_array_equal(pp7[0], wp[0, :n])
        o, e = cells.offsets[c], cells.offsets[c + 1]
        raw = mex.call("forward", gw, float(c + 1), x, nlhs=1)[0]      # default 'raw': the plot vectors
        np.testing.assert_allclose(raw[0], means["sim_ms2"][o:e], rtol=1e-12, atol=0)


@pytest.mark.gpu
def test_custom_construct_struct_and_destroy(mex, cells):
    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.construct import long_two_loop_construct

    cs = long_two_loop_construct()
    st = MxPtr(mex, mex.struct([{"L0": cs.L0, "MS2_start": cs.ms2_start, "MS2_end": cs.ms2_end,
                                 "MS2_loopn": cs.ms2_loopn, "PP7_start": cs.pp7_start, "PP7_end": cs.pp7_end,
                                 "PP7_loopn": cs.pp7_loopn}],
                               ["L0", "MS2_start", "MS2_end", "MS2_loopn", "PP7_start", "PP7_end", "PP7_loopn"]))
    d = data_struct(mex, cells, range(20))
    h = mex.call("create", d, st, 0.0)[0]
    d.free()
    st.free()
    hp = MxPtr(mex, mex.handle(int(h[0, 0])))
    rng = np.random.default_rng(5)
    from transcriptioncycleinference_amd.data import draw_x0

    rows = [draw_x0(rng, int(cells.lengths[c])) for c in range(20)]
    theta = pack(rows, 136)
    with Likelihood(cells.subset(range(20)), cs, device=0) as L:
        want = L.ss_batch(theta, np.arange(20, dtype=np.int32))
    got = mex.call("ss_batch", hp, np.arange(1, 21, dtype=np.float64), theta.T)[0][:, 0]
    np.testing.assert_array_equal(got, want)
    mex.call("destroy", hp, nlhs=0)
    expect("tci:handle", mex.call, "ss", hp, 1.0, rows[0])   # a destroyed handle is rejected
    hp.free()


# ---- 'dram': the GPU-resident sampler through the gateway (TranscriptionCycleMCMC.m:161-273) ----


def _dram_args(mex, cells, ids, seed=5):
    """The reference's per-cell setup (mcmc.plan_fit, :193-255) as MATLAB holds it: P x n, one chain
    per column, 1-based cells."""
    from transcriptioncycleinference_amd.mcmc import plan_fit

    plan = plan_fit(cells, ids, seed)
    cols = [a.T.copy() for a in (plan.x0, plan.lower, plan.upper, plan.prior_mu, plan.prior_sig, plan.qcov_diag)]
    return plan, [np.asarray(plan.cells, np.float64) + 1] + cols + [1.0]


def _opts(mex, **kv):
    return MxPtr(mex, mex.struct([kv], list(kv)))


def test_dram_arguments_and_options_are_checked(mex, cells):
    """Every argument and option of tci_mex('dram', ...) is checked before the handle is looked at
    (so these run without a GPU); a well-formed call with a dead handle reaches the handle check."""
    fake = MxPtr(mex, mex.handle(12345))
    plan, a = _dram_args(mex, cells, [0, 1, 2])
    P = a[1].shape[0]
    expect("tci:handle", mex.call, "dram", fake, *a)                       # well-formed: only the handle is bad
    expect("tci:arg", mex.call, "dram", fake, *a[:6])                      # too few arguments
    expect("tci:arg", mex.call, "dram", fake, a[0][:2], *a[1:])            # n differs from X0's columns
    expect("tci:arg", mex.call, "dram", fake, a[0] + 0.5, *a[1:])          # non-integer cells
    expect("tci:arg", mex.call, "dram", fake, a[0] - a[0], *a[1:])         # cells are 1-based
    expect("tci:arg", mex.call, "dram", fake, a[0], a[1][:6], *a[2:])      # fewer than 7 rows
    for k in range(2, 7):                                                  # LB .. J0 must match X0's shape
        bad = list(a)
        bad[k] = a[k][:P - 1]
        e = expect("tci:arg", mex.call, "dram", fake, *bad)
        assert ("LB", "UB", "MU", "SIG", "J0")[k - 2] in e.msg
    expect("tci:arg", mex.call, "dram", fake, *a[:-1], np.ones(2))         # sigma2: scalar or one per chain
    expect("tci:handle", mex.call, "dram", fake, *a[:-1], np.ones(3))
    expect("tci:handle", mex.call, "dram", fake, *a, np.zeros((0, 0)))     # [] = default options
    expect("tci:opts", mex.call, "dram", fake, *a, 3.0)                    # options must be a struct
    cases = [({"nsimu": 0.0}, "nsimu"), ({"nsimu": 10.5}, "nsimu"), ({"adaptint": -1.0}, "adaptint"),
             ({"method": "slice"}, "method"), ({"method": 3.0}, "method"), ({"engine": "gpu"}, "engine"),
             ({"qcov": np.eye(P)}, "J0"), ({"nsimul": 100.0}, "nsimul"), ({"thin": [1.0, 2.0]}, "thin"),
             ({"chain_keys": [-1.0, 2.0, 3.0]}, "chain_keys")]
    for kv, word in cases:
        o = _opts(mex, **kv)
        e = expect("tci:opts", mex.call, "dram", fake, *a, o)
        assert word in e.msg, (kv, e.msg)
        o.free()
    o = _opts(mex, chain_keys=[1.0, 2.0])                                  # one key per chain
    expect("tci:arg", mex.call, "dram", fake, *a, o)
    o.free()
    o = _opts(mex, nsimu=50.0, method="AM", verbosity=0.0, updatesigma=True, engine="walk")
    expect("tci:handle", mex.call, "dram", fake, *a, o)                    # mcmcstat's names, case-insensitive
    o.free()


def _dram_gateway_vs_binding(mex, h, lk, cells, ids, opts_kv, nlhs=4):
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    plan, a = _dram_args(mex, cells, ids)
    keys = np.asarray(plan.cells, np.int64) * 3 + 11
    o = _opts(mex, **opts_kv, chain_keys=keys.astype(np.float64))
    res, ch, s2c, R = mex.call("dram", h, *a, o, nlhs=nlhs)
    o.free()
    do = DramOptions(n_steps=int(opts_kv["nsimu"]), burnintime=int(opts_kv["burnintime"]),
                     adaptint=int(opts_kv.get("adaptint", 100)), stats_from=int(opts_kv["burnintime"]),
                     thin=int(opts_kv.get("thin", 1)), seed=int(opts_kv["seed"]),
                     engine=opts_kv.get("engine", "auto"))
    want = dram_run(lk, np.asarray(plan.cells, np.int32), plan.x0, plan.lower, plan.upper, plan.prior_mu,
                    plan.prior_sig, plan.qcov_diag, 1.0, do, want_qcov=True, chain_keys=keys)
    n, P = plan.x0.shape
    for f in ("mean", "std", "final_theta"):
        assert res[f].shape == (P, n)
        np.testing.assert_array_equal(res[f], getattr(want, f).T, err_msg=f)
    for f in ("sigma_mean", "sigma_std", "accept_rate"):
        np.testing.assert_array_equal(res[f][0], getattr(want, f), err_msg=f)
    np.testing.assert_array_equal(res["n_evals"][0], want.n_evals.astype(np.float64))
    assert ch.shape == (P, n, want.chain.shape[0]) and s2c.shape == (n, want.chain.shape[0])
    np.testing.assert_array_equal(np.transpose(ch, (2, 1, 0)), want.chain)     # P x n x rows == [row][chain][P]
    np.testing.assert_array_equal(s2c.T, want.s2chain)
    assert R.shape == (P, P, n)
    np.testing.assert_array_equal(np.transpose(R, (2, 0, 1)), want.qcov_R)     # R(:,:,k) upper, qcov = R'R
    for k in range(n):
        assert np.all(np.tril(R[:, :, k], -1) == 0)
    return plan, res


@pytest.mark.gpu
def test_dram_equals_the_binding_bitwise_on_testdata(mex, gw, lk, cells):
    """tci_mex('dram', ...) on TestData cells (the metric's dataset) equals mcmc.dram_run on the same
    inputs bit for bit: summaries, thinned chain, s2chain and the final proposal factor, for the fused
    and the walk engine; 700 steps with burn-in scaling and four covariance updates."""
    ids = [0, 3, 17, 42, 101, 150, 222, 298]
    for engine in ("fused", "walk"):
        plan, res = _dram_gateway_vs_binding(mex, gw, lk, cells, ids,
                                             dict(nsimu=700.0, burnintime=300.0, adaptint=100.0, thin=7.0,
                                                  seed=91.0, method="dram", engine=engine))
        assert np.all(res["accept_rate"] > 0)
    # nargout = 1: no chain rows are kept (thin 0), the summaries are the same
    plan, a = _dram_args(mex, cells, ids)
    o = _opts(mex, nsimu=700.0, burnintime=300.0, seed=91.0, chain_keys=(np.asarray(plan.cells) * 3 + 11.0))
    only = mex.call("dram", gw, *a, o, nlhs=1)[0]
    o.free()
    np.testing.assert_array_equal(only["mean"], res["mean"])
    expect("tci:call", mex.call, "dram", gw, np.array([300.0]), *[x[:, :1] for x in a[1:7]], 1.0)  # cell 300 of 299


@pytest.mark.gpu
def test_dram_equals_the_binding_bitwise_at_config4_shape(mex):
    """The same at BASELINE config 4's shape: 24 synthetic 200-point cells (P = 207, the matrix-core
    adaptation k_adapt_mfma<8, 13>), through a context the gateway created from a MATLAB data struct."""
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.construct import builtin_construct
    from transcriptioncycleinference_amd.data import synthetic_cells

    cs = builtin_construct("P2P-MS2v5-LacZ-PP7v4")

    def fwd(times, theta):
        nan = [np.full(len(t), np.nan) for t in times]
        with Likelihood(from_lists([(t, a, a) for t, a in zip(times, nan)]), cs, device=0) as L:
            return L.forward(theta, np.arange(len(times), dtype=np.int32), grid="interp")

    syn, _ = synthetic_cells(24, 200, 20201028, fwd)
    d = data_struct(mex, syn, range(syn.n_cells))
    h = mex.call("create", d, "P2P-MS2v5-LacZ-PP7v4", 0.0)[0]
    d.free()
    hp = MxPtr(mex, mex.handle(int(h[0, 0])))
    try:
        with Likelihood(syn, cs, device=0) as L:
            for engine in ("walk", "batched"):
                _dram_gateway_vs_binding(mex, hp, L, syn, list(range(24)),
                                         dict(nsimu=500.0, burnintime=200.0, adaptint=100.0, thin=5.0, seed=7.0,
                                              engine=engine))
    finally:
        mex.call("destroy", hp, nlhs=0)
        hp.free()


@pytest.mark.gpu
def test_dram_methods_map_to_mcmcstat_semantics(mex, gw, lk, cells):
    """options.method as mcmcrun reads it: 'dram' = delayed rejection + adaptation, 'am' = adaptation
    without delayed rejection, 'dr' = delayed rejection without adaptation, 'mh' = neither -- each
    equal bit for bit to mcmc.dram_run with the matching ntry / adaptint; the default chain output
    (two outputs, no 'thin') keeps every row."""
    from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run

    ids = [5, 60, 199]
    plan, a = _dram_args(mex, cells, ids)
    for method, ntry, adaptint in (("am", 1, 100), ("dr", 2, 0), ("mh", 1, 0), ("DRAM", 2, 100)):
        o = _opts(mex, nsimu=400.0, burnintime=150.0, adaptint=100.0, seed=3.0, method=method)
        res, ch = mex.call("dram", gw, *a, o, nlhs=2)
        o.free()
        want = dram_run(lk, np.asarray(plan.cells, np.int32), plan.x0, plan.lower, plan.upper, plan.prior_mu,
                        plan.prior_sig, plan.qcov_diag, 1.0,
                        DramOptions(n_steps=400, burnintime=150, adaptint=adaptint, ntry=ntry, stats_from=150, thin=1,
                                    seed=3))
        np.testing.assert_array_equal(res["mean"], want.mean.T, err_msg=method)
        np.testing.assert_array_equal(res["accept_rate"][0], want.accept_rate, err_msg=method)
        assert ch.shape == (plan.x0.shape[1], len(ids), 400)
        np.testing.assert_array_equal(np.transpose(ch, (2, 1, 0)), want.chain, err_msg=method)
