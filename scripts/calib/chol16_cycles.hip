// Cycles of the adaptation's one-wave 16 x 16 tile routines on gfx950 (s_memtime around a dependent
// loop, one wave on an otherwise idle GPU): chol16 (the shipped 4-pivot blocked factorization),
// solve16 (the blocked panel solve of one row tile), and the floors of the pivot chain they are built
// from. Each iteration's input depends on the previous output, so the loop measures latency.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form \
//     -I include -I transcriptioncycleinference_amd/csrc scripts/calib/chol16_cycles.hip -o scripts/calib/chol16_cycles
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "tci_tile16.h"

using namespace tci;

__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

// SPD test tile in the MFMA layout: A = B B' / 16 + 4 I with B[i][k] = sin(i + 2k + 1)
__device__ void spd_tile(double (&a)[4]) {
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  for (int q = 0; q < 4; ++q) {
    const int i = g + 4 * q;
    double s = 0.0;
    for (int k = 0; k < 16; ++k) s += sin((double)(i + 2 * k + 1)) * sin((double)(j + 2 * k + 1));
    a[q] = s / 16.0 + (i == j ? 4.0 : 0.0);
  }
}

__global__ void k_chol(int iters, double tiny, double* out, long long* cyc) {
  __shared__ double rdg[16];
  double A[4], a[4], prev[4] = {0, 0, 0, 0};
  spd_tile(A);
  bool bad = false;
  const uint64_t t0 = clk();
  for (int it = 0; it < iters; ++it) {
    for (int q = 0; q < 4; ++q) a[q] = A[q] + tiny * prev[q];
    chol16(a, rdg, bad);
    for (int q = 0; q < 4; ++q) prev[q] = a[q];
  }
  const uint64_t t1 = clk();
  if (threadIdx.x == 0) cyc[0] = (long long)(t1 - t0);
  for (int q = 0; q < 4; ++q) out[64 * q + threadIdx.x] = prev[q] + (bad ? 1.0 : 0.0);
}

__global__ void k_solve(int iters, double tiny, double* out, long long* cyc) {
  __shared__ double rdg[16];
  __shared__ double D[256];
  const int lane = threadIdx.x & 63, row = lane & 15, kq = lane >> 4;
  double A[4], x[4], prev[4] = {0, 0, 0, 0};
  spd_tile(A);
  double u[4] = {A[0], A[1], A[2], A[3]};
  bool bad = false;
  chol16(u, rdg, bad);
  for (int q = 0; q < 4; ++q) D[(kq + 4 * q) * 16 + row] = u[q];
  wave_sync();
  const uint64_t t0 = clk();
  for (int it = 0; it < iters; ++it) {
    for (int q = 0; q < 4; ++q) x[q] = A[q] + tiny * prev[q];
    solve16(x, D, rdg);
    for (int q = 0; q < 4; ++q) prev[q] = x[q];
  }
  const uint64_t t1 = clk();
  if (threadIdx.x == 0) cyc[0] = (long long)(t1 - t0);
  for (int q = 0; q < 4; ++q) out[64 * q + threadIdx.x] = prev[q] + (bad ? 1.0 : 0.0);
}

// floors: 16 dependent (readlane -> v_rcp_f64 + one Newton step -> fma) pivots on one register
__global__ void k_pivot_floor(int iters, double tiny, double* out, long long* cyc) {
  double x = 2.0 + 0.001 * threadIdx.x;
  const uint64_t t0 = clk();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const double d = lane_bcast(x, k);
      double rd = __builtin_amdgcn_rcp(d);
      rd = fma(rd, fma(-d, rd, 1.0), rd);
      x = fma(-tiny, rd, x);
    }
  }
  const uint64_t t1 = clk();
  if (threadIdx.x == 0) cyc[0] = (long long)(t1 - t0);
  out[threadIdx.x] = x;
}

// one dependent FP64 FMA chain (latency per v_fma_f64)
__global__ void k_fma_floor(int iters, double tiny, double* out, long long* cyc) {
  double x = 1.0 + 0.001 * threadIdx.x;
  const uint64_t t0 = clk();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) x = fma(x, tiny, x);
  }
  const uint64_t t1 = clk();
  if (threadIdx.x == 0) cyc[0] = (long long)(t1 - t0);
  out[threadIdx.x] = x;
}

// dependent v_mfma_f64_16x16x4 chain (same accumulator)
__global__ void k_mfma_floor(int iters, double tiny, double* out, long long* cyc) {
  f64x4 acc = {1.0, 1.0, 1.0, 1.0};
  const double a = tiny * threadIdx.x;
  const uint64_t t0 = clk();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc, 0, 0, 0);
  }
  const uint64_t t1 = clk();
  if (threadIdx.x == 0) cyc[0] = (long long)(t1 - t0);
  for (int q = 0; q < 4; ++q) out[64 * q + threadIdx.x] = acc[q];
}

// dependent row_to_all (permlane) chain
__global__ void k_perm_floor(int iters, double tiny, double* out, long long* cyc) {
  double x = 1.0 + 0.001 * threadIdx.x;
  const uint64_t t0 = clk();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) x = row_to_all<1>(x) + tiny;
  }
  const uint64_t t1 = clk();
  if (threadIdx.x == 0) cyc[0] = (long long)(t1 - t0);
  out[threadIdx.x] = x;
}

template <class K>
double run(K kern, int iters, int per_iter) {
  double* out;
  long long* cyc;
  hipMalloc(&out, 256 * sizeof(double));
  hipMalloc(&cyc, sizeof(long long));
  kern<<<1, 64>>>(iters, 1e-300, out, cyc);  // warm
  kern<<<1, 64>>>(iters, 1e-300, out, cyc);
  long long c = 0;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  hipFree(out);
  hipFree(cyc);
  return (double)c / ((double)iters * per_iter);
}

int main() {
  const int it = 2000;
  printf("{\"unit\": \"s_memtime cycles, one wave, dependent loop\",\n");
  printf(" \"chol16_per_tile\": %.1f,\n", run(k_chol, it, 1));
  printf(" \"solve16_per_tile\": %.1f,\n", run(k_solve, it, 1));
  printf(" \"pivot_floor_readlane_rcp_newton_fma\": %.1f,\n", run(k_pivot_floor, it, 16));
  printf(" \"fma_f64_latency\": %.1f,\n", run(k_fma_floor, it, 16));
  printf(" \"mfma_f64_16x16x4_dependent\": %.1f,\n", run(k_mfma_floor, it, 16));
  printf(" \"row_to_all_plus_add\": %.1f}\n", run(k_perm_floor, it, 16));
  return 0;
}
