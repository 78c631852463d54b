// tci_internal.h -- shared host/device definitions of the MI355X likelihood path.
#pragma once

#include <stdint.h>

#include "tci.h"

namespace tci {

// Per-cell record of the resident cell table. All per-cell arrays in HBM are packed
// struct-of-arrays at [base, base + n); base is a multiple of 2 (16-byte aligned rows).
struct CellMeta {
  int64_t base;
  int32_t n;     // acquisition points N (= grid points M, checked at create)
  int32_t pad;
  double d;      // grid increment of t(1):d:t(end) (SumofSquares...m:29)
  double delta;  // max_j |(t_interp(j+1) - t_interp(j)) - d| over the grid (a few ulps)
};

// One stem-loop segment of one dye (GetFluorFromPolPos.m:21-27,48-52,60-64).
struct SegParams {
  double a;    // loop start (kb)
  double e;    // loop end (kb)
  double phi;  // loopn / 24
  double k;    // phi / (e - a): fractional-occupancy slope
};

// Kernel arguments: device pointers of the resident cell table + the construct.
struct KParams {
  const CellMeta* cells;
  int64_t n_cells;
  const double* T;      // acquisition times t
  const double* Y1;     // MS2 data (NaN = missing)
  const double* Y2;     // PP7 data
  const double* TI;     // uniform grid t_interp (SumofSquares...m:30)
  const double* DT;     // grid steps t_interp(i+1)-t_interp(i), n-1 used, padded with 0
  const double* DTraw;  // raw steps t(i+1)-t(i) (forward on raw t, TranscriptionCycleMCMC.m:307)
  const double* IW;     // interp1 weight s_j of acquisition time j inside its grid interval
  const int32_t* IK;    // interp1 interval index k_j (-1: outside the grid -> NaN)
  double L0;            // gene length before tau*v (GetFluorFromPolPos.m:19)
  double emax;          // max loop end over all segments and dyes
  int32_t n_seg;
  int32_t force_exact;  // test hook: bit 0 = always run the exact sequential counter scan,
                        //            bit 1 = always run the exact per-(row, cohort) position sweep
  SegParams ms2[TCI_MAX_SEG];
  SegParams pp7[TCI_MAX_SEG];
};

enum Mode : int { MODE_SS = 0, MODE_FWD_INTERP = 1, MODE_FWD_RAW = 2 };

// Launch the batched kernel (device pointers). rpl = rows per lane (1,2,4,8).
// out0/out1: MODE_SS -> out0 = ss[B]; forward modes -> MS2/PP7 rows of ld_out.
int launch(const KParams& kp, int rpl, int mode, const double* theta, int64_t ld_theta,
           const int32_t* cell_id, const uint8_t* active, int64_t B, double* out0, double* out1,
           int64_t ld_out, void* stream);

}  // namespace tci
