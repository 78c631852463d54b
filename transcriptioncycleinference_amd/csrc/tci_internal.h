// tci_internal.h -- shared host/device definitions of the MI355X likelihood path.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "tci.h"

namespace tci {

// Resident cell table. Every cell owns a fixed-stride block of `cell_stride` records in each
// record array, so a wave can address all of its cell's data from the cell id alone and issue
// every load of an evaluation at once (no dependent meta -> data round trip).
struct CellMeta {
  int32_t n;     // acquisition points N (= grid points M, checked at create)
  int32_t pad;
  double d;      // grid increment of t(1):d:t(end) (SumofSquares...m:29)
  double delta;  // max_j |(t_interp(j+1) - t_interp(j)) - d| over the grid (a few ulps)
  double eps_v;  // fast-path position bound per unit v (tci_kernels.hip): eps = v * eps_v
};

// Per grid step g: the step length and the step's start time (ConstantElongationSim.m:43-45,57).
struct StepRec {
  double dt;
  double t;
};

// Per acquisition point j: interp1 interval k and weight w (SumofSquares...m:55-56) and the
// data (NaN = missing). A point outside the grid has w = NaN and k = 0, so its interpolated
// value is NaN exactly as interp1 returns; padding records (j >= N) are all-NaN.
struct PointRec {
  double w;
  double y1;  // MS2
  double y2;  // PP7
  int32_t k;
  int32_t pad;
};

// One stem-loop segment of one dye (GetFluorFromPolPos.m:21-27,48-52,60-64).
struct SegParams {
  double a;    // loop start (kb)
  double e;    // loop end (kb)
  double phi;  // loopn / 24
  double k;    // phi / (e - a): fractional-occupancy slope
  double ka;   // k * a (the ramp's offset term of the fast-path row sums, theta-independent)
};

// Kernel arguments: device pointers of the resident cell table + the construct.
struct KParams {
  const CellMeta* cells;
  const StepRec* steps;      // uniform grid t_interp (SumofSquares...m:30) and its steps
  const StepRec* steps_raw;  // raw times t and raw steps (forward on raw t, TranscriptionCycleMCMC.m:307)
  const PointRec* points;
  const double* thr;         // 64 per-lane thresholds of the distance cuts (tci_eval.h distance_cuts): lane
                             // 1 + 4k .. 4 + 4k = MS2 a, MS2 e, PP7 a, PP7 e of segment k; 0 elsewhere
  int64_t n_cells;
  int64_t cell_stride;       // records per cell in steps/steps_raw/points (64*(rows_per_lane+1); long cells: N_max
                             // rounded up to 64)
  int64_t max_n;             // longest cell (points): sizes the long-cell kernel's LDS
  double L0;            // gene length before tau*v (GetFluorFromPolPos.m:19)
  double emax;          // max loop end over all segments and dyes
  int32_t n_seg;
  int32_t force_exact;  // test hook: bit 0 = always run the exact sequential counter scan,
                        //            bit 1 = always run the exact per-(row, cohort) position sweep
  SegParams ms2[TCI_MAX_SEG];
  SegParams pp7[TCI_MAX_SEG];
};

enum Mode : int { MODE_SS = 0, MODE_FWD_INTERP = 1, MODE_FWD_RAW = 2 };

// Allow `func` up to `bytes` of dynamic LDS (hipFuncAttributeMaxDynamicSharedMemorySize). The
// attribute is set once per kernel and process, raised only when a larger size is asked for: the
// DRAM engines launch the same kernels every chunk, and the host call costs a driver round trip.
// Returns TCI_OK or TCI_EHIP. Thread-safe.
int ensure_dyn_lds(const void* func, size_t bytes);

// Launch the batched kernel (device pointers). rpl = rows per lane (1,2,4,8); 0 = the long-cell
// kernel (tci_tile_kernel, any N up to TCI_MAX_POINTS).
// out0/out1: MODE_SS -> out0 = ss[B]; forward modes -> MS2/PP7 rows of ld_out.
int launch(const KParams& kp, int rpl, int mode, const double* theta, int64_t ld_theta,
           const int32_t* cell_id, const uint8_t* active, int64_t B, double* out0, double* out1,
           int64_t ld_out, void* stream);

}  // namespace tci
