// tci_diag.h -- the diagnostics switches of the HIP kernels, in one place. Every one defaults to 0
// (the product build); a non-zero value is set only by a measurement build (hipcc -D..., see
// scripts/ab_variants.py) and is never shipped. Ablations produce WRONG results on purpose: they remove work
// to price it; profiles add s_memtime stamps and atomics.
#pragma once

// Likelihood kernel (tci_eval.h, tci_kernels.hip): bit0 row sums, bit2 interp1 + nansum, bit3 the
// counter scan, bit4 loads only, bit5 launch only.
#ifndef TCI_ABLATE
#define TCI_ABLATE 0
#endif
// DRAM draws pass (k_draws): bit0 no normals, bit1 no z*R products, bit2 no scalar draws.
#ifndef TCI_DRAWS_ABLATE
#define TCI_DRAWS_ABLATE 0
#endif
// Adaptation (k_adapt_mfma): bit0 skip the Cholesky, bit1 skip the covupd scatter.
#ifndef TCI_ADAPT_ABLATE
#define TCI_ADAPT_ABLATE 0
#endif
// s_memtime cycles per phase into DramState::prof, printed by tci_dram_run: k_chain (1: wave 0's
// phases, 2: per-wave barrier waits, 3: every wave's phases) / k_adapt_mfma and k_adapt_gt (1:
// thread 0's phases; k_adapt_mfma's slot 6 is the run listing, window_runs).
#ifndef TCI_CHAIN_PROFILE
#define TCI_CHAIN_PROFILE 0
#endif
#ifndef TCI_ADAPT_PROFILE
#define TCI_ADAPT_PROFILE 0
#endif
