import sys, numpy as np, json
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from transcriptioncycleinference_amd import Likelihood, from_lists
from transcriptioncycleinference_amd.data import synthetic_cells
from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run
from test_dram_gpu import setup_rows
def fwd(times, theta):
    nan = [np.full(len(t), np.nan) for t in times]
    with Likelihood(from_lists([(t, a, a) for t, a in zip(times, nan)])) as L:
        return L.forward(theta, np.arange(len(times), dtype=np.int32), grid="interp")
cells, truth = synthetic_cells(64, 120, 99, fwd, nan_fraction=0.0)
truth[:, 7:] = 0.0
ms2, pp7 = fwd([cells.cell(c)[0] for c in range(64)], truth)
rng = np.random.default_rng(1)
cells = from_lists([(cells.cell(c)[0], ms2[c, :120] + rng.normal(0, 0.3, 120), pp7[c, :120] + rng.normal(0, 0.3, 120)) for c in range(64)])
with Likelihood(cells) as L:
    ids = list(range(64))
    x0, lo, hi, mu, sg, J0 = setup_rows(cells, ids, seed=2)
    for steps in (8000,):
        res = dram_run(L, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, DramOptions(n_steps=steps, burnintime=steps//2, stats_from=steps//2, seed=4))
        ev = np.abs(res.mean[:, 0] - truth[:, 0]) / truth[:, 0]
        eR = np.abs(res.mean[:, 6] + res.mean[:, 7:126].mean(axis=1) - truth[:, 6]) / truth[:, 6]
        et = np.abs(res.mean[:, 1] - truth[:, 1])
        eA = np.abs(res.mean[:, 5] - truth[:, 5]) / truth[:, 5]
        print(json.dumps({"steps": steps, "ms": res.elapsed_ms, "med_err_v": float(np.median(ev)), "med_err_R": float(np.median(eR)),
             "med_abs_err_tau": float(np.median(et)), "med_err_A": float(np.median(eA)), "sigma_med": float(np.median(res.sigma_mean)),
             "acc_med": float(np.median(res.accept_rate)), "q90_err_v": float(np.quantile(ev, 0.9))}), flush=True)
    # where do the chains end vs the truth?
    res = dram_run(L, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, DramOptions(n_steps=20000, burnintime=10000, stats_from=10000, seed=4))
    ss_fin = L.ss_batch(res.final_theta, np.array(ids, np.int32))
    ss_true = L.ss_batch(truth[:, :127], np.array(ids, np.int32))
    zv = (res.mean[:, 0] - truth[:, 0]) / res.std[:, 0]
    print(json.dumps({"ss_final_med": float(np.median(ss_fin)), "ss_true_med": float(np.median(ss_true)),
                      "frac_final_below_true": float(np.mean(ss_fin < ss_true)), "z_v_med_abs": float(np.median(np.abs(zv))),
                      "std_v_med": float(np.median(res.std[:, 0]))}), flush=True)
    # start AT the truth
    x0t = x0.copy(); x0t[:, :127] = truth[:, :127]
    res = dram_run(L, np.array(ids, np.int32), x0t, lo, hi, mu, sg, J0, 1.0, DramOptions(n_steps=20000, burnintime=10000, stats_from=10000, seed=5))
    ev = np.abs(res.mean[:, 0] - truth[:, 0]) / truth[:, 0]
    ss_fin = L.ss_batch(res.final_theta, np.array(ids, np.int32))
    print(json.dumps({"from_truth_med_err_v": float(np.median(ev)), "ss_final_med": float(np.median(ss_fin)), "std_v_med": float(np.median(res.std[:, 0]))}), flush=True)
