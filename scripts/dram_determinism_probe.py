import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from transcriptioncycleinference_amd import Likelihood, testdata
from transcriptioncycleinference_amd.mcmc import DramOptions, dram_run
from test_dram_gpu import setup_rows
cells = testdata()
L = Likelihood(cells)
ids = list(range(0, 299, 13))
x0, lo, hi, mu, sg, J0 = setup_rows(cells, ids)
for ai in (100, 0):
    o = DramOptions(n_steps=400, burnintime=200, adaptint=ai, stats_from=100, thin=1, seed=7)
    a = dram_run(L, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o)
    b = dram_run(L, np.array(ids, np.int32), x0, lo, hi, mu, sg, J0, 1.0, o)
    d = np.any(a.chain != b.chain, axis=2)  # rows x chains
    if d.any():
        r, c = np.argwhere(d)[0]
        print("adaptint", ai, "first differing row", r + 1, "chain", c, "n differing chains", d.any(axis=0).sum(),
              "max abs diff", np.nanmax(np.abs(a.chain - b.chain)))
    else:
        print("adaptint", ai, "identical")
