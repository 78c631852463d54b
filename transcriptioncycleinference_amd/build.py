"""In-tree build of ``libtci.so`` for gfx950 (hipcc; no JIT cache, the .so travels with the repo).

``-ffp-contract=off`` is load-bearing: the loading counter (``counter + R(i)*dt(i)``) and the
position updates (``x(i,k) + v*dt(i)``) feed floor() and strict comparisons, and MATLAB never
fuses a multiply into an add. FMA is used only where written explicitly (continuous sums).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
SOURCES = [os.path.join(CSRC, "tci_kernels.hip"), os.path.join(CSRC, "tci_dram.hip"), os.path.join(CSRC, "tci_api.cpp")]
HEADERS = [os.path.join(REPO_ROOT, "include", "tci.h"), os.path.join(CSRC, "tci_internal.h"), os.path.join(CSRC, "tci_diag.h"), os.path.join(CSRC, "tci_tile16.h"), os.path.join(CSRC, "tci_adapt_map.h"),
           os.path.join(CSRC, "tci_dram_internal.h"), os.path.join(CSRC, "tci_eval.h")]
LIB = os.path.join(PKG_DIR, "libtci.so")
ARCH = "gfx950"  # CDNA4 only: the kernels use gfx950 instructions (v_bitop3_b32, permlane16/32 swaps)


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libtci.so)")


def needs_rebuild() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in SOURCES + HEADERS + [__file__])


def build_library(force: bool = False, verbose: bool = False, out: str = LIB, defines=None) -> str:
    """Compile libtci.so (or an A/B variant with extra -D defines into `out`)."""
    if out == LIB and not defines and not force and not needs_rebuild():
        return LIB
    # -amdgpu-mfma-vgpr-form: MFMA accumulators in VGPRs (the AGPR form made the compiler copy every
    # accumulator into AGPRs and back around each f64 MFMA of the draws pass and wait for it)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-mllvm", "-amdgpu-mfma-vgpr-form",
           "-fPIC", "-shared",
           "-Wall", "-Wno-bitwise-instead-of-logical", "-Wno-pass-failed", "-I" + os.path.join(REPO_ROOT, "include"), "-I" + CSRC,
           *[f"-D{d}" for d in (defines or [])], *SOURCES, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


MEX_DIR = os.path.join(REPO_ROOT, "matlab")
MEX_STUB = os.path.join(MEX_DIR, "mexstub", "libtci_mex_stub.so")


def build_mex_stub(verbose: bool = False) -> str:
    """Compile the MATLAB MEX gateway (matlab/tci_mex.cpp) against the builder-written stand-in
    MATLAB API (matlab/mexstub/: MATLAB's own mex.h is absent here) into one shared library linked
    to libtci.so, so tests/test_mex_gateway.py can execute mexFunction. Test infrastructure: a MATLAB
    user builds tci_mex.cpp with `mex`."""
    stub = os.path.join(MEX_DIR, "mexstub")
    cxx = shutil.which("g++") or "g++"
    cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-fPIC", "-shared", "-I" + stub, "-I" + os.path.join(REPO_ROOT, "include"),
           os.path.join(MEX_DIR, "tci_mex.cpp"), os.path.join(stub, "mexstub.cpp"), "-L" + PKG_DIR, "-ltci",
           "-Wl,-rpath,$ORIGIN/../../transcriptioncycleinference_amd", "-o", MEX_STUB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(MEX_STUB + ".tmp", MEX_STUB)
    return MEX_STUB


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
