"""MI355X-native likelihood hot path of GarciaLab/TranscriptionCycleInference.

The hot path is mcmcstat's ``ssfun``: SumofSquaresFunction_TranscriptionCycleMCMC ->
ConstantElongationSim -> GetFluorFromPolPos. Compute runs only in the HIP
library ``libtci.so`` (C ABI: ``include/tci.h``); there is no CPU fallback.
"""
from .construct import Construct, builtin_construct, long_two_loop_construct  # noqa: F401
from .data import Cells, from_lists, load_mat, load_npz, testdata  # noqa: F401
from ._lib import TciError, TciLibraryMissing  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # GPU-facing names resolve lazily so that importing the package never needs a GPU.
    if name in ("Likelihood", "version"):
        from . import likelihood

        return getattr(likelihood, name)
    if name in ("SumofSquaresFunction_TranscriptionCycleMCMC", "make_ssfun", "simulate_fluorescence"):
        from . import ssfun

        return getattr(ssfun, name)
    raise AttributeError(name)
