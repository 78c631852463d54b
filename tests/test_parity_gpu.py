"""HIP path vs the CPU oracle and the reference's golden vectors (needs an MI355X).

Tolerances: the north-star contract is 1e-6 relative on SS; these tests assert 1e-10 (the
kernel reproduces every discontinuous decision bit-exactly and differs only in the order of
continuous sums, ~1e-15 observed). Integer/decision-level properties (exact-scan path, batch
determinism, permutation invariance) are asserted bit-exactly.
"""
import numpy as np
import pytest

from conftest import pack
from oracle import oracle as O

pytestmark = pytest.mark.gpu

REL = 1e-10


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    both_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    ok = both_nan | both_inf
    with np.errstate(invalid="ignore"):
        d = np.where(ok, 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-300))
    d[np.isnan(d)] = np.inf
    return float(np.max(d)) if d.size else 0.0


@pytest.fixture(scope="module")
def lk(cells):
    from transcriptioncycleinference_amd import Likelihood

    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4", device=0) as L:
        yield L


def oracle_ss(c_oracle, cells, construct, theta, cid, active=None):
    ss, st = c_oracle.ss_batch(cells.offsets, cells.t, cells.ms2, cells.pp7, construct, theta, cid, active)
    assert np.all(st == 0), st[st != 0][:5]
    return ss


# --- golden vectors ------------------------------------------------------------------


def test_chain_rows_match_committed_ss_goldens(lk, chain):
    theta = pack(chain["rows"])
    ss = lk.ss_batch(theta, chain["cell_id"])
    e = rel_err(ss, chain["ss"])
    print(f"max rel err over {len(ss)} fixture chain rows: {e:.3e}")
    assert e <= REL


def test_forward_raw_matches_reference_plot_vectors(lk, cells, means):
    """GPU forward model at MCMCresults means == MCMCplot.simMS2/simPP7 written by MATLAB."""
    theta = pack(means["rows"])
    cid = np.arange(cells.n_cells, dtype=np.int32)
    ms2, pp7 = lk.forward(theta, cid, grid="raw")
    worst = 0.0
    for c in range(cells.n_cells):
        o, e = cells.offsets[c], cells.offsets[c + 1]
        n = e - o
        worst = max(worst, rel_err(ms2[c, :n], means["sim_ms2"][o:e]), rel_err(pp7[c, :n], means["sim_pp7"][o:e]))
    print(f"max rel err vs MATLAB MCMCplot vectors: {worst:.3e}")
    assert worst <= 1e-12


def test_forward_interp_matches_oracle(lk, cells, chain, construct, c_oracle):
    pick = np.nonzero(chain["step"] == 5)[0]
    theta = pack([chain["rows"][i] for i in pick])
    cid = chain["cell_id"][pick]
    ms2, pp7 = lk.forward(theta, cid, grid="interp")
    worst = 0.0
    for i, b in enumerate(pick[:60]):
        c = int(cid[i])
        t = cells.cell(c)[0]
        m, p = c_oracle.forward(t, construct, chain["rows"][b], mode=1)
        worst = max(worst, rel_err(ms2[i, :len(t)], m), rel_err(pp7[i, :len(t)], p))
    assert worst <= 1e-12


# --- random parameters over the whole dataset -------------------------------------


def test_x0_distribution_all_cells_vs_oracle(lk, cells, construct, c_oracle):
    from transcriptioncycleinference_amd.data import draw_x0

    rng = np.random.default_rng(1)
    rows, cid = [], []
    for k in range(6):
        for c in range(cells.n_cells):
            rows.append(draw_x0(rng, int(cells.lengths[c])))
            cid.append(c)
    theta = pack(rows)
    cid = np.array(cid, np.int32)
    ss = lk.ss_batch(theta, cid)
    want = oracle_ss(c_oracle, cells, construct, theta, cid)
    e = rel_err(ss, want)
    print(f"max rel err, x0 draws: {e:.3e}")
    assert e <= REL


def test_wide_parameter_box_vs_oracle(lk, cells, construct, c_oracle):
    """Uniform draws over the whole prior box (TranscriptionCycleMCMC.m:242-255)."""
    rng = np.random.default_rng(7)
    B = 2048
    cid = rng.integers(0, cells.n_cells, B).astype(np.int32)
    rows = []
    for c in cid:
        n = int(cells.lengths[c])
        core = rng.uniform([0, 0, 0, 0, 0, 0, 0], [10, 20, 10, 50, 50, 1, 40])
        rows.append(np.concatenate([core, rng.uniform(-30, 30, n)]))
    theta = pack(rows)
    ss = lk.ss_batch(theta, cid)
    want = oracle_ss(c_oracle, cells, construct, theta, cid)
    assert rel_err(ss, want) <= REL


def test_exact_scan_path_is_bitwise_identical(lk, chain):
    """The parallel counter scan + proof and the serial scan give the same cohorts."""
    theta = pack(chain["rows"])
    fast = lk.ss_batch(theta, chain["cell_id"])
    lk.set_force_exact(scan=True)
    try:
        exact = lk.ss_batch(theta, chain["cell_id"])
    finally:
        lk.set_force_exact()
    np.testing.assert_array_equal(fast, exact)


def test_exact_position_sweep_vs_distance_table(lk, cells, chain, construct, c_oracle):
    """The per-(row, cohort) exact sweep and the uniform-grid distance-table convolution agree
    (ulp-level: the fractional occupancy uses P_m instead of the exact position) and both match
    the oracle."""
    from transcriptioncycleinference_amd.data import draw_x0

    rng = np.random.default_rng(5)
    rows = list(chain["rows"]) + [draw_x0(rng, int(cells.lengths[c])) for c in range(cells.n_cells)]
    cid = np.concatenate([chain["cell_id"], np.arange(cells.n_cells, dtype=np.int32)])
    theta = pack(rows)
    fast = lk.ss_batch(theta, cid)
    lk.set_force_exact(scan=True, positions=True)
    try:
        exact = lk.ss_batch(theta, cid)
    finally:
        lk.set_force_exact()
    want = oracle_ss(c_oracle, cells, construct, theta, cid)
    assert rel_err(fast, exact) <= 1e-12
    assert rel_err(exact, want) <= REL and rel_err(fast, want) <= REL


def test_integer_counter_forces_exact_fallback(construct, c_oracle):
    """dt = 0.25 exactly and R = 4: every counter value is an exact integer, so the fast scan
    cannot prove floor() and every wave must take the serial path; results must still match."""
    from transcriptioncycleinference_amd import Likelihood, from_lists

    n = 120
    t = 0.25 * np.arange(n)
    rng = np.random.default_rng(3)
    y1, y2 = rng.normal(4, 1, n), rng.normal(8, 2, n)
    cells = from_lists([(t, y1, y2)])
    rows = []
    for v in (0.5, 1.0, 2.0, 3.0):
        for ton in (0.0, 1.0, 3.3):
            rows.append(np.concatenate([[v, 1.5, ton, 2.0, 1.0, 0.7, 4.0], np.zeros(n)]))
    theta = pack(rows)
    cid = np.zeros(len(rows), np.int32)
    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4") as L:
        ss = L.ss_batch(theta, cid)
    want = oracle_ss(c_oracle, cells, construct, theta, cid)
    assert rel_err(ss, want) <= REL


# --- edge cases the reference defines --------------------------------------------


def test_edge_cases_vs_oracle(lk, cells, construct, c_oracle):
    n0 = int(cells.lengths[0])
    base = np.concatenate([[2.0, 1.0, 1.0, 3.0, 2.0, 0.6, 12.0], np.zeros(n0)])
    cases = {
        "v=0": {0: 0.0},
        "v tiny": {0: 1e-6},
        "v max": {0: 10.0},
        "tau=0": {1: 0.0},
        "tau max": {1: 20.0},
        "ton after last point": {2: 40.0},
        "ton=0": {2: 0.0},
        "A=0": {5: 0.0},
        "basal huge": {3: 50.0, 4: 50.0},
        "R=0": {6: 0.0},
    }
    rows = []
    for upd in cases.values():
        r = base.copy()
        for k, val in upd.items():
            r[k] = val
        rows.append(r)
    r = base.copy()
    r[7:] = -30.0  # every rate clamped to 0: nothing loads
    rows.append(r)
    r = base.copy()
    r[7:] = 30.0
    r[6] = 40.0
    rows.append(r)
    theta = pack(rows)
    cid = np.zeros(len(rows), np.int32)
    ss = lk.ss_batch(theta, cid)
    want = oracle_ss(c_oracle, cells, construct, theta, cid)
    assert rel_err(ss, want) <= REL


def test_positions_on_a_threshold_take_the_exact_sweep(lk, cells, construct, c_oracle):
    """Rates v that put a representative position P_m = m*(v*d) onto a decision threshold (a loop
    start or end, or the gene end L = L0 + tau*v): the lane-parallel distance cut (tci_eval.h,
    distance_cut) must flag the ambiguity, the wave takes the exact sweep, and the SS equals the
    oracle's -- and the forced exact sweep's -- for every such row."""
    rows, cid = [], []
    a_m, e_m, a_p, e_p, L0 = 0.024, 1.299, 4.292, 5.758, 6.626  # P2P-MS2v5-LacZ-PP7v4 (GetFluorFromPolPos.m:18-28)
    for c in (0, 7, 42, 123, 298):
        t = cells.cell(c)[0]
        n = len(t)
        d = float(np.sum(np.diff(t))) / (n - 1)  # the grid increment (SumofSquares...m:29)
        for m in (1, 3, 10, 25):
            if m >= n - 1:
                continue
            tau = 2.0
            for v in (a_m / (m * d), e_m / (m * d), a_p / (m * d), e_p / (m * d), L0 / (m * d - tau)):
                if not (0.0 < v < 20.0):
                    continue
                r = np.concatenate([[v, tau, t[0] + 0.5, 1.0, 2.0, 0.7, 9.0], np.zeros(n)])
                rows.append(r)
                cid.append(c)
    theta = pack(rows)
    cid = np.array(cid, np.int32)
    ss = lk.ss_batch(theta, cid)
    want = oracle_ss(c_oracle, cells, construct, theta, cid)
    assert rel_err(ss, want) <= REL
    lk.set_force_exact(positions=True)
    try:
        ex = lk.ss_batch(theta, cid)
    finally:
        lk.set_force_exact()
    assert rel_err(ss, ex) <= REL
    print(f"{len(ss)} rows with a position on a threshold, max rel err vs oracle {rel_err(ss, want):.2e}")


def test_inactive_rows_and_nonfinite_theta(lk, cells, chain):
    theta = pack(chain["rows"][:8])
    cid = chain["cell_id"][:8]
    active = np.array([1, 0, 1, 0, 1, 1, 1, 1], np.uint8)
    theta[4, 0] = np.nan
    theta[5, 10] = np.inf
    ss = lk.ss_batch(theta, cid, active)
    assert np.isinf(ss[1]) and ss[1] > 0 and np.isinf(ss[3])
    assert np.isnan(ss[4]) and np.isnan(ss[5])
    np.testing.assert_allclose(ss[[0, 2, 6, 7]], chain["ss"][[0, 2, 6, 7]], rtol=REL)


def test_unused_last_rate_and_padding_do_not_matter(lk, chain):
    """dR_N never enters the SS (ConstantElongationSim.m:33); padding past 7+N is ignored."""
    rows = chain["rows"][:16]
    theta = pack(rows, ld=160)
    theta2 = theta.copy()
    for i, r in enumerate(rows):
        theta2[i, len(r) - 1] = 17.0
        theta2[i, len(r):] = np.nan
    np.testing.assert_array_equal(lk.ss_batch(theta, chain["cell_id"][:16]),
                                  lk.ss_batch(theta2, chain["cell_id"][:16]))


def test_all_nan_data_gives_zero(construct):
    from transcriptioncycleinference_amd import Likelihood, from_lists

    n = 50
    t = np.cumsum(np.full(n, 0.3)) - 0.3
    cells = from_lists([(t, np.full(n, np.nan), np.full(n, np.nan))])
    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4") as L:
        th = np.concatenate([[2.0, 1.0, 1.0, 3.0, 2.0, 0.6, 12.0], np.zeros(n)])
        assert L.ssfun(th, 0) == 0.0


def test_argument_errors(lk, chain):
    from transcriptioncycleinference_amd import TciError

    theta = pack(chain["rows"][:2])
    with pytest.raises(TciError):
        lk.ss_batch(theta, np.array([0, 299], np.int32))
    with pytest.raises(TciError):
        lk.ss_batch(theta[:, :100], chain["cell_id"][:2])


# --- kernel variants: rows per lane (1,2,4,8) and segment counts (1..4) ---------------


@pytest.mark.parametrize("n", [2, 3, 64, 65, 66, 129, 130, 200, 257, 258, 400, 513])
def test_rows_per_lane_variants_vs_oracle(n, construct, c_oracle):
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.data import draw_x0, synthetic_times

    rng = np.random.default_rng(100 + n)
    cl = []
    for _ in range(3):
        t = synthetic_times(rng, n)
        y1, y2 = rng.normal(3, 2, n), rng.normal(6, 3, n)
        y1[rng.random(n) < 0.37] = np.nan
        y2[rng.random(n) < 0.37] = np.nan
        cl.append((t, y1, y2))
    cells = from_lists(cl)
    rows, cid = [], []
    for k in range(40):
        c = k % 3
        r = draw_x0(rng, n)
        if k % 5 == 0:
            r[0] = rng.uniform(0.05, 0.5)  # slow elongation: long windows
        rows.append(r)
        cid.append(c)
    theta = pack(rows)
    cid = np.array(cid, np.int32)
    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4") as L:
        ss = L.ss_batch(theta, cid)
        ms2, pp7 = L.forward(theta[:3], cid[:3], grid="raw")
    want = oracle_ss(c_oracle, cells, construct, theta, cid)
    assert rel_err(ss, want) <= REL
    for i in range(3):
        m, p = c_oracle.forward(cells.cell(int(cid[i]))[0], construct, theta[i], mode=0)
        assert rel_err(ms2[i, :n], m) <= 1e-12 and rel_err(pp7[i, :n], p) <= 1e-12


@pytest.mark.parametrize("nseg", [2, 3, 4])
def test_multi_segment_constructs_vs_oracle(nseg, c_oracle):
    from transcriptioncycleinference_amd import Likelihood, from_lists, long_two_loop_construct
    from transcriptioncycleinference_amd.construct import Construct
    from transcriptioncycleinference_amd.data import draw_x0, synthetic_times

    if nseg == 2:
        cs = long_two_loop_construct()
    else:
        a = np.linspace(0.05, 9.0, nseg)
        cs = Construct(11.0, list(a), list(a + 0.8), [24.0, 12.0, 6.0, 24.0][:nseg],
                       list(a + 0.3), list(a + 1.9), [24.0] * nseg, f"seg{nseg}")
    ocs = O.Construct(cs.L0, cs.ms2_start, cs.ms2_end, cs.ms2_loopn, cs.pp7_start, cs.pp7_end, cs.pp7_loopn)
    rng = np.random.default_rng(nseg)
    n = 200
    cl = [(synthetic_times(rng, n), rng.normal(3, 2, n), rng.normal(6, 3, n)) for _ in range(4)]
    cells = from_lists(cl)
    rows = [draw_x0(rng, n) for _ in range(64)]
    cid = np.arange(64, dtype=np.int32) % 4
    theta = pack(rows)
    with Likelihood(cells, cs) as L:
        ss = L.ss_batch(theta, cid)
    want, st = c_oracle.ss_batch(cells.offsets, cells.t, cells.ms2, cells.pp7, ocs, theta, cid)
    assert np.all(st == 0)
    assert rel_err(ss, want) <= REL


# --- full-size batch properties (BASELINE config 2 batch: 299 cells x 256 proposals) -----


def test_full_batch_determinism_and_permutation(lk, cells, chain):
    rng = np.random.default_rng(11)
    K = 256
    base = pack(chain["rows"])
    idx = rng.integers(0, len(base), cells.n_cells * K)
    theta = base[idx] + np.where(np.arange(base.shape[1]) < 7, 0.0, rng.normal(0, 0.5, (len(idx), base.shape[1])))
    theta[:, 7:] = np.clip(theta[:, 7:], -30, 30)
    cid = chain["cell_id"][idx]
    ss = lk.ss_batch(theta, cid)
    assert np.all(np.isfinite(ss))
    again = lk.ss_batch(theta, cid)
    np.testing.assert_array_equal(ss, again)
    perm = rng.permutation(len(idx))
    np.testing.assert_array_equal(lk.ss_batch(theta[perm], cid[perm]), ss[perm])
    # duplicated rows give bitwise-identical results wherever they land in the grid
    dup = np.repeat(theta[:64], 5, axis=0)
    dss = lk.ss_batch(dup, np.repeat(cid[:64], 5))
    np.testing.assert_array_equal(dss.reshape(64, 5), np.repeat(ss[:64, None], 5, axis=1))


def test_full_batch_sample_vs_oracle(lk, cells, construct, chain, c_oracle):
    rng = np.random.default_rng(12)
    base = pack(chain["rows"])
    idx = rng.integers(0, len(base), 4096)
    theta = base[idx].copy()
    theta[:, :7] *= rng.uniform(0.8, 1.2, (len(idx), 7))
    theta[:, 5] = np.clip(theta[:, 5], 0, 1)
    cid = chain["cell_id"][idx]
    ss = lk.ss_batch(theta, cid)
    want = oracle_ss(c_oracle, cells, construct, theta, cid)
    assert rel_err(ss, want) <= REL


# --- device-resident API (torch tensors in HBM) -------------------------------------


def test_device_async_api_matches_host_api(lk, chain):
    import torch

    theta = pack(chain["rows"])
    want = lk.ss_batch(theta, chain["cell_id"])
    dev = torch.device("cuda:0")
    th_d = torch.from_numpy(theta).to(dev)
    cid_d = torch.from_numpy(chain["cell_id"].astype(np.int32)).to(dev)
    out_d = torch.empty(len(theta), dtype=torch.float64, device=dev)
    act_d = torch.ones(len(theta), dtype=torch.uint8, device=dev)
    lk.ss_batch_device(th_d, cid_d, out_d, act_d, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out_d.cpu().numpy(), want)


@pytest.mark.parametrize("offset", [0, 1, 2, 3])
@pytest.mark.parametrize("B", [4093, 4096, 4097, 5])
def test_active_flags_at_every_alignment_and_length(lk, chain, offset, B):
    """The kernel reads the active flags by 4-byte words through the scalar cache where the word lies
    inside the flag array (and the array is 4-byte aligned), byte by byte elsewhere: flag arrays at
    every byte offset of an allocation and batch lengths on and off a multiple of 4 give the host
    API's results row for row (+Inf for every inactive row)."""
    import torch

    rows = pack(chain["rows"])
    rng = np.random.default_rng(B + offset)
    idx = rng.integers(0, len(rows), B)
    theta, cid = rows[idx], chain["cell_id"][idx].astype(np.int32)
    act = (rng.random(B) < 0.7).astype(np.uint8)
    act[-1] = 1
    act[-2:] = [0, 1] if B > 2 else act[-2:]
    want = lk.ss_batch(theta, cid, act)
    dev = torch.device("cuda:0")
    base = torch.zeros(B + 8, dtype=torch.uint8, device=dev)
    act_d = base[offset:offset + B]
    act_d.copy_(torch.from_numpy(act))
    th_d = torch.from_numpy(theta).to(dev)
    cid_d = torch.from_numpy(cid).to(dev)
    out_d = torch.empty(B, dtype=torch.float64, device=dev)
    lk.ss_batch_device(th_d, cid_d, out_d, act_d, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = out_d.cpu().numpy()
    np.testing.assert_array_equal(got, want)
    assert np.all(np.isinf(got[act == 0])) and np.all(np.isfinite(got[act == 1]))


# --- reference-named API -------------------------------------------------------------


def test_reference_named_entry_points(cells, chain, means):
    from transcriptioncycleinference_amd import (SumofSquaresFunction_TranscriptionCycleMCMC, make_ssfun,
                                                 simulate_fluorescence)

    for b in (0, 1234, 2989):
        c = int(chain["cell_id"][b])
        d = cells.data_struct(c)
        ss = SumofSquaresFunction_TranscriptionCycleMCMC("P2P-MS2v5-LacZ-PP7v4", d, chain["rows"][b])
        assert abs(ss - chain["ss"][b]) <= REL * chain["ss"][b]
        assert make_ssfun("P2P-MS2v5-LacZ-PP7v4")(chain["rows"][b], d) == ss
    c = 17
    t = cells.cell(c)[0]
    m, p = simulate_fluorescence("P2P-MS2v5-LacZ-PP7v4", t, means["rows"][c])
    o, e = cells.offsets[c], cells.offsets[c + 1]
    assert rel_err(m, means["sim_ms2"][o:e]) <= 1e-12 and rel_err(p, means["sim_pp7"][o:e]) <= 1e-12
    with pytest.raises(ValueError):
        make_ssfun("not-a-construct")


def test_synthetic_config4_cells(construct, c_oracle):
    """SURVEY config 4 shape (N=200 points, synthetic data from the GPU forward model)."""
    from transcriptioncycleinference_amd import Likelihood, from_lists
    from transcriptioncycleinference_amd.data import synthetic_cells

    def fwd(times, theta):
        nan = [np.full(len(t), np.nan) for t in times]
        cells = from_lists([(t, a, a) for t, a in zip(times, nan)])
        with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4") as L:
            return L.forward(theta, np.arange(len(times), dtype=np.int32), grid="interp")

    cells, truth = synthetic_cells(256, 200, 20201028, fwd)
    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4") as L:
        ss = L.ss_batch(truth, np.arange(256, dtype=np.int32))
    want = oracle_ss(c_oracle, cells, construct, truth, np.arange(256, dtype=np.int32))
    assert rel_err(ss, want) <= REL
    # at the ground truth the residual is pure noise: SS ~ (0.63N)(1 + 4)
    assert 0.5 < np.median(ss) / (0.63 * 200 * 5) < 1.5


# --- long cells (N > 513): the long-cell kernel (rows_per_lane == 0) -------------------


def _long_cells(rng, n, ncell=3):
    from transcriptioncycleinference_amd import from_lists
    from transcriptioncycleinference_amd.data import synthetic_times

    cl = []
    for k in range(ncell):
        nk = n - 7 * k  # ragged lengths in one context
        t = synthetic_times(rng, nk)
        y1, y2 = rng.normal(3, 2, nk), rng.normal(6, 3, nk)
        y1[rng.random(nk) < 0.37] = np.nan
        y2[rng.random(nk) < 0.37] = np.nan
        cl.append((t, y1, y2))
    return from_lists(cl)


@pytest.mark.parametrize("n", [514, 600, 1000, 2048])
def test_long_cells_vs_oracle(n, construct, c_oracle):
    """ConstantElongationSim.m:39-50 has no length cap: cells past the register-resident variants
    (N > 513) run the long-cell kernel, ss_batch and both forward grids against the oracle."""
    from transcriptioncycleinference_amd import Likelihood
    from transcriptioncycleinference_amd.data import draw_x0

    rng = np.random.default_rng(300 + n)
    cells = _long_cells(rng, n)
    rows, cid = [], []
    for k in range(24):
        c = k % 3
        r = draw_x0(rng, int(cells.lengths[c]))
        if k % 4 == 0:
            r[0] = rng.uniform(0.05, 0.5)  # slow elongation: long windows
        rows.append(r)
        cid.append(c)
    theta = pack(rows)
    cid = np.array(cid, np.int32)
    active = np.ones(len(cid), np.uint8)
    active[5] = 0
    with Likelihood(cells, "P2P-MS2v5-LacZ-PP7v4") as L:
        assert L.info["rows_per_lane"] == 0
        ss = L.ss_batch(theta, cid, active)
        fi = L.forward(theta[:3], cid[:3], grid="interp")
        fr = L.forward(theta[:3], cid[:3], grid="raw")
        L.set_force_exact(scan=True, positions=True)
        ss_exact = L.ss_batch(theta, cid, active)
        L.set_force_exact()
    want = oracle_ss(c_oracle, cells, construct, theta, cid, active)
    assert np.isinf(ss[5]) and np.isinf(want[5])
    e, ex = rel_err(ss, want), rel_err(ss_exact, want)
    print(f"N={n}: max rel err {e:.3e} (forced exact paths {ex:.3e})")
    assert e <= REL and ex <= REL
    for i in range(3):
        t = cells.cell(int(cid[i]))[0]
        nk = len(t)
        for mode, (ms2, pp7) in ((1, fi), (0, fr)):
            m, p = c_oracle.forward(t, construct, theta[i], mode=mode)
            assert rel_err(ms2[i, :nk], m) <= 1e-12 and rel_err(pp7[i, :nk], p) <= 1e-12


def test_long_cells_multi_segment_and_edges(c_oracle):
    """Long cells on the 2-segment 3x-length construct (config 5) and the edge rows: non-finite
    theta -> NaN, bad cell id rejected, all-NaN data -> 0."""
    from transcriptioncycleinference_amd import Likelihood, from_lists, long_two_loop_construct
    from transcriptioncycleinference_amd.data import draw_x0, synthetic_times

    rng = np.random.default_rng(77)
    n = 700
    t = synthetic_times(rng, n)
    y1, y2 = rng.normal(3, 2, n), rng.normal(6, 3, n)
    cells = from_lists([(t, y1, y2), (t, np.full(n, np.nan), np.full(n, np.nan))])
    con = long_two_loop_construct()
    rows = [draw_x0(rng, n) for _ in range(10)]
    rows[3][9] = np.inf
    theta = pack(rows)
    cid = np.array([0] * 9 + [1], np.int32)
    ocs = O.Construct(con.L0, con.ms2_start, con.ms2_end, con.ms2_loopn, con.pp7_start, con.pp7_end, con.pp7_loopn)
    with Likelihood(cells, con) as L:
        assert L.info["rows_per_lane"] == 0
        ss = L.ss_batch(theta, cid)
    want, _ = c_oracle.ss_batch(cells.offsets, cells.t, cells.ms2, cells.pp7, ocs, theta, cid)
    assert np.isnan(ss[3])
    ok = np.arange(10) != 3
    assert rel_err(ss[ok], want[ok]) <= REL
    assert ss[9] == 0.0
