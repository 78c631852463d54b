import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# Load torch (and its HIP runtime) before libtci.so: both carry the soname libamdhip64.so.7, and
# whichever loads first serves the process. bench.py imports torch first too.
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def _ragged(z, key="theta", off="theta_offsets"):
    o = z[off]
    return [z[key][o[i]:o[i + 1]] for i in range(len(o) - 1)]


@pytest.fixture(scope="session")
def cells():
    from transcriptioncycleinference_amd import testdata

    return testdata()


@pytest.fixture(scope="session")
def construct():
    from oracle import oracle as O

    return O.builtin_construct("P2P-MS2v5-LacZ-PP7v4")


@pytest.fixture(scope="session")
def chain():
    z = np.load(os.path.join(GOLDEN, "chain_theta.npz"), allow_pickle=False)
    return {"rows": _ragged(z), "cell_id": z["cell_id"], "step": z["step"], "s2": z["s2"], "ss": z["ss"]}


@pytest.fixture(scope="session")
def means():
    z = np.load(os.path.join(GOLDEN, "forward_means.npz"), allow_pickle=False)
    return {"rows": _ragged(z), "sim_ms2": z["sim_ms2"], "sim_pp7": z["sim_pp7"], "cell_index": z["cell_index"]}


@pytest.fixture(scope="session")
def c_oracle():
    from oracle import c_oracle as CO

    CO.build()
    return CO


def pack(rows, ld=None):
    ld = ld or max(len(r) for r in rows)
    out = np.zeros((len(rows), ld))
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out
