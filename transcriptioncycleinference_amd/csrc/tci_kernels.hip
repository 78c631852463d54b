// tci_kernels.hip -- batched FP64 likelihood kernel for gfx950 (CDNA4): one wavefront per
// ssfun(theta, cell) evaluation (the algorithm and its exactness arguments: tci_eval.h).
#include "tci_eval.h"

// Build-time variants for A/B timing (scripts/ab_variants.py); the shipped defaults are below.
#ifndef TCI_XCD_REMAP
#define TCI_XCD_REMAP 0      // XCD-aware block -> row-range order (A/B: ~1% slower here; the
#endif                       // 3.7 MB cell table fits every XCD's L2 anyway)
#ifndef TCI_WAVES_PER_EU
#define TCI_WAVES_PER_EU 6   // register budget for 6 waves/SIMD (A/B: 50 us vs 58 us at the
#endif                       // compiler's default 5 waves; 7-8 waves no faster)
#if TCI_WAVES_PER_EU > 0
#define TCI_OCCUPANCY __attribute__((amdgpu_waves_per_eu(TCI_WAVES_PER_EU)))
#else
#define TCI_OCCUPANCY
#endif

namespace tci {

namespace {

constexpr int kWavesPerBlock = 4;

template <int RPL, int NSEG, int MODE>
__global__ __launch_bounds__(256) TCI_OCCUPANCY void tci_cohort_kernel(const KParams kp, const double* __restrict__ theta,
                                                         int64_t ld, const int32_t* __restrict__ cell_id,
                                                         const uint8_t* __restrict__ active, int64_t B,
                                                         double* __restrict__ out0, double* __restrict__ out1,
                                                         int64_t ld_out) {
  constexpr int SLOTS = 64 * RPL;      // rows 1..SLOTS (row 0 never holds a polymerase)
  constexpr int NPT = RPL + 1;         // acquisition points per lane (N <= 64*RPL + 1)
  constexpr int WAVE_DOUBLES = eval_lds_doubles<RPL>();  // {K,J} table / the two sim rows
  __shared__ __attribute__((aligned(16))) double s_lds[kWavesPerBlock][WAVE_DOUBLES];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware block order: blocks are dealt round-robin over the 8 XCDs; give each XCD a
  // contiguous range of rows so rows of the same cell share one XCD's L2 (speed only).
#if TCI_XCD_REMAP
  const unsigned nb = gridDim.x, bid = blockIdx.x;
  const unsigned xq = nb / 8, xr = nb % 8, xcd = bid % 8, xk = bid / 8;
  const unsigned vb = xcd < xr ? xcd * (xq + 1) + xk : xr * (xq + 1) + (xcd - xr) * xq + xk;
#else
  const unsigned vb = blockIdx.x;
#endif
  const int64_t b = (int64_t)vb * kWavesPerBlock + wid;
  if (b >= B) return;
  double* lds = s_lds[wid];

  // ---- every load of the evaluation is issued here, in one round trip
  const int c = __builtin_amdgcn_readfirstlane(cell_id[b]);
  const bool act = MODE != MODE_SS || active == nullptr || active[b] != 0;
  if (!act) {
    if (lane == 0) out0[b] = INFINITY;  // skipped proposal (bounds-rejected by the caller)
    return;
  }
  if (c < 0 || c >= kp.n_cells) {
    write_nan<MODE>(lane, 0, b, out0, out1, ld_out);
    return;
  }
  const int64_t cbase = (int64_t)c * kp.cell_stride;
  const StepRec* ST = (MODE == MODE_FWD_RAW ? kp.steps_raw : kp.steps) + cbase;
  const PointRec* PT = kp.points + cbase;
  const double* th = theta + b * ld;
  EvalIn<RPL> e;
  e.cm = kp.cells[c];
  e.v = th[0];
  e.tau = th[1];
  e.ton = th[2];
  e.b1 = th[3];
  e.b2 = th[4];
  e.A = th[5];
  e.R = th[6];
#pragma unroll
  for (int q = 0; q < RPL; ++q) {
    const int g = RPL * lane + q;
    e.dr[q] = 7 + g < ld ? th[7 + g] : 0.0;  // speculative (N unknown yet), kept inside the row
    e.st[q] = ST[g];                          // g < cell_stride
  }
  if (MODE != MODE_FWD_RAW) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int j = lane + 64 * k;
      if (j <= SLOTS) e.pt[k] = PT[j];
      else e.pt[k] = PointRec{NAN, NAN, NAN, 0, 0};  // beyond every cell's points: dropped
    }
  }
  const int N = e.cm.n;
  if (ld < 7 + N) {
    write_nan<MODE>(lane, N, b, out0, out1, ld_out);
    return;
  }
  const double ss = eval_wave<RPL, NSEG, MODE>(kp, e, lane, lds, b, out0, out1, ld_out);
  if (MODE == MODE_SS && lane == 0) out0[b] = ss;
}

template <int RPL, int NSEG, int MODE>
void launch_one(const KParams& kp, const double* theta, int64_t ld, const int32_t* cell_id, const uint8_t* active,
                int64_t B, double* out0, double* out1, int64_t ld_out, hipStream_t stream) {
  const dim3 block(64 * kWavesPerBlock);
  const dim3 grid((unsigned)((B + kWavesPerBlock - 1) / kWavesPerBlock));
  hipLaunchKernelGGL((tci_cohort_kernel<RPL, NSEG, MODE>), grid, block, 0, stream, kp, theta, ld, cell_id, active, B,
                     out0, out1, ld_out);
}

template <int RPL, int NSEG>
int launch_rpl_seg(const KParams& kp, int mode, const double* theta, int64_t ld, const int32_t* cell_id,
                   const uint8_t* active, int64_t B, double* out0, double* out1, int64_t ld_out,
                   hipStream_t stream) {
  switch (mode) {
    case MODE_SS:
      launch_one<RPL, NSEG, MODE_SS>(kp, theta, ld, cell_id, active, B, out0, out1, ld_out, stream);
      break;
    case MODE_FWD_INTERP:
      launch_one<RPL, NSEG, MODE_FWD_INTERP>(kp, theta, ld, cell_id, active, B, out0, out1, ld_out, stream);
      break;
    case MODE_FWD_RAW:
      launch_one<RPL, NSEG, MODE_FWD_RAW>(kp, theta, ld, cell_id, active, B, out0, out1, ld_out, stream);
      break;
    default:
      return TCI_EINVAL;
  }
  return hipGetLastError() == hipSuccess ? TCI_OK : TCI_EHIP;
}

template <int RPL>
int launch_rpl(const KParams& kp, int mode, const double* theta, int64_t ld, const int32_t* cell_id,
               const uint8_t* active, int64_t B, double* out0, double* out1, int64_t ld_out, hipStream_t stream) {
  switch (kp.n_seg) {
    case 1: return launch_rpl_seg<RPL, 1>(kp, mode, theta, ld, cell_id, active, B, out0, out1, ld_out, stream);
    case 2: return launch_rpl_seg<RPL, 2>(kp, mode, theta, ld, cell_id, active, B, out0, out1, ld_out, stream);
    case 3: return launch_rpl_seg<RPL, 3>(kp, mode, theta, ld, cell_id, active, B, out0, out1, ld_out, stream);
    case 4: return launch_rpl_seg<RPL, 4>(kp, mode, theta, ld, cell_id, active, B, out0, out1, ld_out, stream);
    default: return TCI_EINVAL;
  }
}

}  // namespace

int launch(const KParams& kp, int rpl, int mode, const double* theta, int64_t ld_theta, const int32_t* cell_id,
           const uint8_t* active, int64_t B, double* out0, double* out1, int64_t ld_out, void* stream) {
  if (B <= 0) return TCI_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (rpl) {
    case 1: return launch_rpl<1>(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    case 2: return launch_rpl<2>(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    case 4: return launch_rpl<4>(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    case 8: return launch_rpl<8>(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    default: return TCI_EINVAL;
  }
}

}  // namespace tci
