// tci_tile16.h -- one wavefront's 16 x 16 FP64 tile helpers in the v_mfma_f64_16x16x4 accumulator
// layout (lane 16 g + j holds rows g, g+4, g+8, g+12 of column j), shared by the adaptation kernels
// (tci_dram.hip) and the calibration kernel scripts/calib/chol16_cycles.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#include "tci_eval.h"

namespace tci {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// Lane l's value of x in every lane (readlane: scalar broadcast, l uniform).
__device__ __forceinline__ double lane_bcast(double x, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}

// This lane's index computed afresh (v_mbcnt). The adaptation kernels run at their register budget,
// where the compiler keeps lane-derived indices alive across whole phases and spills them: a scratch
// reload inside the diagonal factorization or the panel solve puts a memory round trip on a
// latency-bound path (one per pivot pair, r04 asm). Volatile, so it is recomputed where it is used.
__device__ __forceinline__ int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

template <bool F>  // F: lane_now() (a kernel that spills), else threadIdx.x (kept in a register)
__device__ __forceinline__ int lane_idx() {
  if constexpr (F) return lane_now();
  return (int)(threadIdx.x & 63);
}

// Lane (16 g + K)'s x in every lane of 16-lane row g (DPP row_newbcast, no LDS).
template <int K>
__device__ __forceinline__ double row_bcast16(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x150 + K, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x150 + K, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// 16-lane row G's x in every row (lane l gets lane 16 G + (l & 15)): two gfx950 permlane swaps per
// 32-bit half (permlane32_swap pairs rows {0,1} with {2,3}, permlane16_swap row 0 with 1 and 2
// with 3), no LDS round trip (ds_bpermute waits on the LDS pipe).
template <int G>
__device__ __forceinline__ double row_to_all(double x) {
  unsigned h[2] = {(unsigned)__double2loint(x), (unsigned)__double2hiint(x)};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const auto a = __builtin_amdgcn_permlane32_swap(h[q], h[q], false, false);  // [R0 R1 R0 R1], [R2 R3 R2 R3]
    const unsigned y = G < 2 ? a[0] : a[1];
    const auto b = __builtin_amdgcn_permlane16_swap(y, y, false, false);        // [Ra Ra Ra Ra], [Rb Rb Rb Rb]
    h[q] = (G & 1) ? b[1] : b[0];
  }
  return __hiloint2double((int)h[1], (int)h[0]);
}

// Cholesky factorization A = U'U of a symmetric 16 x 16 tile held by ONE wave in registers, in the
// MFMA accumulator layout (lane 16 g + j holds rows g, g+4, g+8, g+12 of column j: slot q = rows
// 4q .. 4q+3), blocked by 4 pivots. Block B is slot B. Its four rows are first replicated into every
// lane group (r_k: row 4B + k, column j in every lane 16 g + j; four independent permlane row
// broadcasts), so the pivots K = 4B + k run on lane-local values and readlane scalars only: d =
// r_k[K], rows k' > k of columns j > K take A -= A[4B+k'][K] A[K][j] / d. A permlane broadcast costs
// ~74 cycles against ~54 for a whole readlane -> v_rcp_f64 -> Newton -> fma pivot step
// (scripts/calib/chol16_cycles.hip), so the pivots no longer wait on one per step. The slot's rows
// are then scaled to U rows (1 / sqrt(d) per row), and the trailing rows and columns >= 4B + 4 take
// the rank-4 update A -= U_B' U_B as ONE v_mfma_f64_16x16x4 -- the slot itself is both operands
// (A[i][k] = U[4B+k][i] sits in lane 16 k + i, the B operand's lane for U[4B+k][j]), zeroed in the
// columns < 4B + 4. rdg[4B + g] = 1 / U[4B+g][4B+g] for the panel solve; bad if a pivot is not
// positive and finite. Every element sees the operations of the one-slot form in the same order.
template <int B, int R, bool F>
__device__ __forceinline__ void chol16_pivot(double (&r)[4], double (&dk)[4], bool& bad) {
  constexpr int K = 4 * B + R;
  const int j = lane_idx<F>() & 15;
  const double d = lane_bcast(r[R], K);  // A[K][K]
  bad = bad || !(d > 0.0) || !isfinite(d);
  dk[R] = d;
  if constexpr (R < 3) {
    double rd = __builtin_amdgcn_rcp(d);
    rd = fma(rd, fma(-d, rd, 1.0), rd);
    const double sj = r[R] * rd;  // A[K][j] / d
#pragma unroll
    for (int k = R + 1; k < 4; ++k) {
      const double aik = lane_bcast(r[k], K);  // A[4B + k][K]
      if (j > K) r[k] = fma(-aik, sj, r[k]);
    }
  }
}

template <int B, bool F>
__device__ __forceinline__ void chol16_block(double (&a)[4], double* rdg, bool& bad) {
  if constexpr (B < 4) {
    const int lane = lane_idx<F>(), g = lane >> 4, j = lane & 15;
    double r[4] = {row_to_all<0>(a[B]), row_to_all<1>(a[B]), row_to_all<2>(a[B]), row_to_all<3>(a[B])};
    double dk[4];
    chol16_pivot<B, 0, F>(r, dk, bad);
    chol16_pivot<B, 1, F>(r, dk, bad);
    chol16_pivot<B, 2, F>(r, dk, bad);
    chol16_pivot<B, 3, F>(r, dk, bad);
    const double x = g == 0 ? r[0] : g == 1 ? r[1] : g == 2 ? r[2] : r[3];
    const double dv = g == 0 ? dk[0] : g == 1 ? dk[1] : g == 2 ? dk[2] : dk[3];
    const double rs = 1.0 / sqrt(dv);
    const double u = x * rs;  // U[4B + g][j] for j >= 4B + g
    if (j == 4 * B + g) rdg[j] = rs;
    if constexpr (B < 3) {
      const double op = j >= 4 * B + 4 ? u : 0.0;
      f64x4 acc = {a[0], a[1], a[2], a[3]};
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-op, op, acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = acc[q];
    }
    a[B] = u;
    chol16_block<B + 1, F>(a, rdg, bad);
  }
}

template <bool F = false>
__device__ __forceinline__ void chol16(double (&a)[4], double* rdg, bool& bad) {
  chol16_block<0, F>(a, rdg, bad);
}

// The panel solve U' X = A of one 16 x 16 row tile, held by one wave in the MFMA layout (x[q]: rows
// g + 4q of column j), U the panel's diagonal tile row-major in LDS (D[k 16 + m] = U[k][m], m >= k)
// and rdg[k] = 1 / U[k][k]. Blocked like chol16: the four rows of slot B are replicated into every
// lane group and solved in turn on lane-local values (row k scaled by rdg, then fma with
// U[4B+k][4B+k'] into the later rows k'), then the rows below take X -= U_B' X_B as one MFMA (A
// operand: U[4B+k][i] for i >= 4B + 4, B operand: the slot). Every coefficient is an LDS load
// independent of the recurrence.
template <int B, bool F>
__device__ __forceinline__ void solve16_block(double (&x)[4], const double* D, const double* rdg) {
  if constexpr (B < 4) {
    const int lane = lane_idx<F>(), g = lane >> 4, j = lane & 15;
    double rg[4], cf[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      rg[k] = rdg[4 * B + k];
#pragma unroll
      for (int m = k + 1; m < 4; ++m) cf[k][m] = D[(4 * B + k) * 16 + 4 * B + m];  // U[4B+k][4B+m]
    }
    const double aop = (B < 3 && j >= 4 * B + 4) ? D[(4 * B + g) * 16 + j] : 0.0;
    double r[4] = {row_to_all<0>(x[B]), row_to_all<1>(x[B]), row_to_all<2>(x[B]), row_to_all<3>(x[B])};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r[k] = r[k] * rg[k];
#pragma unroll
      for (int m = k + 1; m < 4; ++m) r[m] = fma(-cf[k][m], r[k], r[m]);
    }
    const double xb = g == 0 ? r[0] : g == 1 ? r[1] : g == 2 ? r[2] : r[3];
    x[B] = xb;
    if constexpr (B < 3) {
      f64x4 acc = {x[0], x[1], x[2], x[3]};
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-aop, xb, acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = acc[q];
    }
    solve16_block<B + 1, F>(x, D, rdg);
  }
}

template <bool F = false>
__device__ __forceinline__ void solve16(double (&x)[4], const double* D, const double* rdg) {
  solve16_block<0, F>(x, D, rdg);
}

}  // namespace tci
