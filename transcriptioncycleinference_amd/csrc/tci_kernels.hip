// tci_kernels.hip -- batched FP64 likelihood kernel for gfx950 (CDNA4): one wavefront per
// ssfun(theta, cell) evaluation (the algorithm and its exactness arguments: tci_eval.h).
#include "tci_eval.h"

namespace tci {

namespace {

// One wave per 64-thread block for RPL <= 2 (round 5): a block's LDS is held until its last wave ends, so with
// 4-wave blocks every bounds-rejected row (a wave that exits at once) kept its 4 KB of LDS allocated
// beside its block's evaluating waves and LDS, not the wave slots, capped the evaluating waves per CU
// (~28 % of the bench's rows are rejected). 1-wave blocks: 33.6 vs 35.4 us per bench launch; with the
// flag read through the scalar cache (below) 32.9 (profiles/r05/r05h_lk.json). Round 2: a register
// budget for 6 waves/SIMD took 50 vs 58 us per launch at the compiler's default 5, and 7-8 were no
// faster then; with round 3's shorter instruction stream 8 pays (below). (An XCD-aware block -> row
// order, SGPR basal operands, cell records shared through LDS by a 4-wave block (45.6 vs 35.2) and
// every load of the evaluation issued with the flag's (40.7 vs 35.2) measured slower or within noise:
// DESIGN.md Appendix A.) RPL >= 4 (cells of 130-513 points) keeps 4-wave blocks: there the 1-wave
// layout let the compiler take 127 instead of 98 VGPRs at the same occupancy and the config-4 kernel
// slowed from 107 to 123 us per launch (profiles/r05/r05i_bench.json).
template <int RPL>
constexpr int waves_per_block() { return RPL <= 2 ? 1 : 4; }

// Waves per SIMD the register budget is set for: 8 while RPL * NSEG <= 2 (58 VGPRs at RPL = 2,
// NSEG = 1, no spill; 34.4 vs 36.0 us per bench launch against 6 in one process,
// profiles/r03_likelihood/r03occ1_ab.json; 7: 35.8), 6 above (RPL = 2 with two segments spills at
// 8; the LDS of a 4-wave block caps RPL = 4 at 4 waves/SIMD anyway).
constexpr int lk_waves_per_eu(int rpl, int nseg) { return rpl * nseg <= 2 ? 8 : 6; }

template <int RPL, int NSEG, int MODE>
__global__ __launch_bounds__(64 * waves_per_block<RPL>()) __attribute__((amdgpu_waves_per_eu(lk_waves_per_eu(RPL, NSEG)))) void tci_cohort_kernel(const KParams kp, const double* __restrict__ theta,
                                                         int64_t ld, const int32_t* __restrict__ cell_id,
                                                         const uint8_t* __restrict__ active, int64_t B,
                                                         double* __restrict__ out0, double* __restrict__ out1,
                                                         int64_t ld_out, int64_t flag_words) {
  constexpr int WAVE_DOUBLES = eval_lds_doubles<RPL>();  // {K,J} table / the two sim rows
  constexpr int kWavesPerBlock = waves_per_block<RPL>();
  __shared__ __attribute__((aligned(16))) double s_lds[kWavesPerBlock][WAVE_DOUBLES];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  if (b >= B) return;
  double* lds = s_lds[wid];
#if TCI_ABLATE & 32
  if (lane == 0) out0[b] = 1.0;  // launch floor (diagnostics only)
  return;
#endif

  // ---- the row's cell id and active flag, then every other load of the evaluation at once. (Also
  //      reading the theta scalars with the cell id, one round trip earlier, measured no faster and
  //      fetched the theta lines of the bounds-rejected rows too: DESIGN.md §3.)
  const int c = __builtin_amdgcn_readfirstlane(cell_id[b]);
  // the flag through the scalar cache (one s_load_dword of its 4-byte word): a rejected row's wave
  // ends without queueing behind the other waves' vector loads (34.2 vs 35.4 us per bench launch,
  // r05h). flag_words: the rows whose whole word lies inside `active` (which is 4-byte aligned);
  // the last partial word and a misaligned array read the byte. (Evaluating only a list of the
  // in-bounds rows, built by a compaction kernel on the stream, measured slower: DESIGN.md
  // Appendix A, r06e/r06f.)
  bool act = true;
  if (MODE == MODE_SS && active != nullptr)
    act = b < flag_words ? ((reinterpret_cast<const uint32_t*>(active)[b >> 2] >> (8 * (b & 3))) & 0xffu) != 0
                         : active[b] != 0;
  if (!act) {
    if (lane == 0) out0[b] = INFINITY;  // skipped proposal (bounds-rejected by the caller)
    return;
  }
  if (c < 0 || ((kp.n_cells >> 31) == 0 && c >= (int)kp.n_cells)) {
    write_nan<MODE>(lane, 0, b, out0, out1, ld_out);
    return;
  }
  const double* th = theta + b * ld;
  // the row length in 32 bits (ld > 0): the lanes' index compares and the row check in 32-bit
  // (scalar) compares instead of 64-bit vector ones
  const int ldi = (ld >> 31) != 0 ? 0x7fffffff : (int)ld;
  EvalIn<RPL> e;
  load_cell<RPL, MODE == MODE_FWD_RAW>(kp, c, lane, e);
  e.v = th[0];
  e.tau = th[1];
  e.ton = th[2];
  e.b1 = th[3];
  e.b2 = th[4];
  e.A = th[5];
  e.R = th[6];
  if (RPL >= 2) {
    // dR pairs (8-B aligned 16-B loads): one load instruction per two entries where the pair is
    // inside the row, entry by entry at the row's end (41.8 vs 42.3 us per bench launch, r03t)
    typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));
#pragma unroll
    for (int q = 0; q < RPL; q += 2) {
      const int g = RPL * lane + q;
      if (8 + g < ldi) {
        const d2u x = *reinterpret_cast<const d2u*>(th + 7 + g);
        e.dr[q] = x.x;
        e.dr[q + 1] = x.y;
      } else {
        e.dr[q] = 7 + g < ldi ? th[7 + g] : 0.0;
        e.dr[q + 1] = 0.0;
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      const int g = RPL * lane + q;
      e.dr[q] = 7 + g < ldi ? th[7 + g] : 0.0;  // speculative (N unknown yet), kept inside the row
    }
  }
  const int N = e.cm.n;
  if (ldi < 7 + N) {  // a row shorter than 7 + N entries
    write_nan<MODE>(lane, N, b, out0, out1, ld_out);
    return;
  }
  const double ss = eval_wave<RPL, NSEG, MODE>(kp, e, lane, lds, b, out0, out1, ld_out);
  if (MODE == MODE_SS && lane == 0) out0[b] = ss;
}

template <int RPL, int NSEG, int MODE>
void launch_one(const KParams& kp, const double* theta, int64_t ld, const int32_t* cell_id, const uint8_t* active,
                int64_t B, double* out0, double* out1, int64_t ld_out, hipStream_t stream) {
  constexpr int kWavesPerBlock = waves_per_block<RPL>();
  const dim3 block(64 * kWavesPerBlock);
  const dim3 grid((unsigned)((B + kWavesPerBlock - 1) / kWavesPerBlock));
  const int64_t flag_words = active != nullptr && (reinterpret_cast<uintptr_t>(active) & 3) == 0 ? (B & ~(int64_t)3) : 0;
  hipLaunchKernelGGL((tci_cohort_kernel<RPL, NSEG, MODE>), grid, block, 0, stream, kp, theta, ld, cell_id, active, B,
                     out0, out1, ld_out, flag_words);
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

// ---- Long cells (N > 64*8 + 1 points): tci_tile_kernel. One wavefront per evaluation walks the
// cell in 64-row tiles with the algorithm of eval_wave; per-tile carries replace the whole-wave
// scans, and the {K,J} tables, the simulated rows and the exact path's per-cohort state live in
// the wave's LDS (dynamic, tile_lds_doubles(N_max) doubles: 64 B per point). One wave per
// workgroup. Same decisions as eval_wave (bit-identical cohorts and region choices); the
// continuous sums may differ from eval_wave's order at the ulp level.
//   LDS (doubles): [KJ: 2 + 2S][simM: N][simP: N][accM: N][accP: N][pc: N][vd: N], S = N - 1;
//   KJ holds (K_i, J_i) for i in [-1, S): entry -1 is the zero the clamped lookups read.
__host__ __device__ inline int64_t tile_lds_doubles(int64_t n) { return 8 * n + 8; }

template <int NSEG, int MODE>
__global__ __launch_bounds__(64) void tci_tile_kernel(const KParams kp, const double* __restrict__ theta, int64_t ld,
                                                      const int32_t* __restrict__ cell_id,
                                                      const uint8_t* __restrict__ active, int64_t B,
                                                      double* __restrict__ out0, double* __restrict__ out1,
                                                      int64_t ld_out) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  if (b >= B) return;
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
  const CellMeta cm = kp.cells[c];
  const int N = cm.n, S = N - 1;
  if (ld < 7 + N) {
    write_nan<MODE>(lane, N, b, out0, out1, ld_out);
    return;
  }
  const int64_t cbase = (int64_t)c * kp.cell_stride;
  const StepRec* ST = (MODE == MODE_FWD_RAW ? kp.steps_raw : kp.steps) + cbase;
  const PointRec* PT = kp.points + cbase;
  const double* th = theta + b * ld;
  const double v = th[0], tau = th[1], ton = th[2], b1 = th[3], b2 = th[4], A = th[5], R = th[6];
  const unsigned ebits = max(max(max(exp_bits(v), exp_bits(tau)), max(exp_bits(ton), exp_bits(b1))),
                            max(max(exp_bits(b2), exp_bits(A)), exp_bits(R)));
  uint64_t nonfinite = 0;
  for (int g0 = 0; g0 < S; g0 += 64) {
    const int g = g0 + lane;
    nonfinite |= wave_ballot(g < S && !isfinite(th[7 + min(g, S - 1)]));
  }
  if (ebits == 0x7ff00000u || nonfinite != 0) {  // outside mcmcstat's finite parameter box
    write_nan<MODE>(lane, N, b, out0, out1, ld_out);
    return;
  }
  double2* KJ = reinterpret_cast<double2*>(dyn) + 1;  // KJ[-1] = (0, 0)
  double* simM = dyn + 2 * N;
  double* simP = simM + N;
  double* accM = simP + N;
  double* accP = accM + N;
  double* pc = accP + N;
  double* vdd = pc + N;
  if (lane == 0) KJ[-1] = make_double2(0.0, 0.0);

  // ---- loading counter (ConstantElongationSim.m:60-61): tile scans with a carry + the exactness
  //      test (margin 2^-38 relative: >> the (S + 64) ulp bound between summation orders, S < 2^11)
  uint64_t amb = 0;
  {
    double carry = 0.0;
    for (int g0 = 0; g0 < S; g0 += 64) {
      const int g = g0 + lane;
      const bool valid = g < S;
      const StepRec sr = ST[min(g, S - 1)];
      const double dr = th[7 + min(g, S - 1)];
      const double rho = fmax(R + dr, 0.0);  // R(R<0) = 0 (ConstantElongationSim.m:36)
      const double prod = (valid && !(sr.t < ton)) ? rho * sr.dt : 0.0;
      if (valid) pc[g] = prod;  // the serial fallback's terms
      const double Sq = carry + wave_incl_scan(prod);
      const double eps = Sq * 0x1p-38;
      const double Kq = floor(Sq);
      amb |= wave_ballot(valid && (Sq - eps < Kq || Sq + eps >= Kq + 1.0));
      if (valid) KJ[g].x = Kq;
      carry = lane63(Sq);
    }
  }
  wave_sync();
  if ((kp.force_exact & 1) || amb != 0) {  // the reference's serial loop, counter = counter + R(i)*dt(i)
    if (lane == 0) {
      double counter = 0.0;
      for (int g = 0; g < S; ++g) {
        counter = counter + pc[g];
        KJ[g].x = floor(counter);
      }
    }
    wave_sync();
  }
  // ---- J_i = sum_{i' <= i} i' c_i' (exact integers), c_i = K_i - K_{i-1}
  {
    double carry = 0.0;
    for (int g0 = 0; g0 < S; g0 += 64) {
      const int g = g0 + lane;
      const bool valid = g < S;
      const double cg = valid ? KJ[g].x - KJ[g - 1].x : 0.0;
      const double Jq = carry + wave_incl_scan((double)g * cg);
      if (valid) KJ[g].y = Jq;
      carry = lane63(Jq);
    }
  }
  wave_sync();

  SegParams sm[NSEG], sp[NSEG];
#pragma unroll
  for (int k = 0; k < NSEG; ++k) {
    sm[k] = kp.ms2[k];
    sp[k] = kp.pp7[k];
  }
  const double L = kp.L0 + tau * v;                 // GetFluorFromPolPos.m:19-20, no FMA
  const double pstop = L > kp.emax ? L : kp.emax;  // f(p) == 0 for every p >= pstop

  bool fast = MODE != MODE_FWD_RAW && !(kp.force_exact & 2);
  const double vd0 = v * cm.d;
  Cuts<NSEG> cu;
  // ---- distance cuts over m = 1..S and their exactness proof (as eval_wave)
  if (v > 0.0 && fast) fast = distance_cuts<NSEG>(kp.thr[lane], L, vd0, v * cm.eps_v, S, lane, cu);
  if (v > 0.0 && fast) {
    // ---- O(1) row sums from the {K, J} tables, floors inside the segment loop, x A
    double kvdM[NSEG], kaM[NSEG], kvdP[NSEG], kaP[NSEG];
#pragma unroll
    for (int k = 0; k < NSEG; ++k) {
      kvdM[k] = sm[k].k * vd0;
      kaM[k] = sm[k].ka;
      kvdP[k] = sp[k].k * vd0;
      kaP[k] = sp[k].ka;
    }
    for (int r0 = 1; r0 <= S; r0 += 64) {
      const int r = r0 + lane;
      if (r > S) break;
      const double rd = (double)r;
      const double kL = kj_at<true>(KJ, r - cu.nL - 1).x;
      double m = 0.0, pp = 0.0;
#pragma unroll
      for (int k = 0; k < NSEG; ++k) {
        const double aM = row_sum<true>(KJ, r, rd, cu.nMa[k], cu.nMe[k], kL, sm[k], kvdM[k], kaM[k]);
        const double aP = row_sum<true>(KJ, r, rd, cu.nPa[k], cu.nPe[k], kL, sp[k], kvdP[k], kaP[k]);
        m = k == 0 ? fmax(aM, b1) : fmax(m + aM, b1);
        pp = k == 0 ? fmax(aP, b2) : fmax(pp + aP, b2);
      }
      simM[r] = A * m;
      simP[r] = pp;
    }
  } else {
    // ---- exact path (or v <= 0: nothing lit): per segment, the diagonal sweep -- at distance s
    //      cohort i (loaded at step i) sits at row i + s with its forward-summed position
    //      p = p + v*dt(i+s-1) (ConstantElongationSim.m:64), so every branch is decided on
    //      bit-identical positions; row r receives cohorts r-1, r-2, .. in eval_wave's order.
    for (int i0 = 0; i0 < S; i0 += 64) {
      const int i = i0 + lane;
      if (i < S) vdd[i] = v * ST[i].dt;  // v*dt(i), rounded once
    }
    for (int k = 0; k < NSEG; ++k) {
      for (int i0 = 0; i0 < N; i0 += 64) {
        const int i = i0 + lane;
        if (i < N) {
          accM[i] = 0.0;
          accP[i] = 0.0;
          pc[i] = 0.0;
        }
      }
      wave_sync();
      if (v > 0.0) {
        for (int s = 1; s <= S; ++s) {
          uint64_t alive = 0;
          for (int i0 = 0; i0 + s <= S; i0 += 64) {
            const int i = i0 + lane, r = i + s;
            const bool valid = r <= S;
            if (valid) {
              const double p = pc[i] + vdd[r - 1];
              pc[i] = p;
              const double ci = KJ[i].x - KJ[i - 1].x;
              accM[r] = fma(ci, occupancy(p, sm[k], L), accM[r]);
              accP[r] = fma(ci, occupancy(p, sp[k], L), accP[r]);
              alive |= wave_ballot(ci > 0.0 && p < pstop);
            }
          }
          wave_sync();
          if (alive == 0) break;
        }
      }
      for (int r0 = 1; r0 <= S; r0 += 64) {  // basal floor inside the segment loop (GetFluorFromPolPos.m:54-57,66-69)
        const int r = r0 + lane;
        if (r <= S) {
          simM[r] = k == 0 ? fmax(accM[r], b1) : fmax(simM[r] + accM[r], b1);
          simP[r] = k == 0 ? fmax(accP[r], b2) : fmax(simP[r] + accP[r], b2);
        }
      }
      wave_sync();
    }
    for (int r0 = 1; r0 <= S; r0 += 64) {
      const int r = r0 + lane;
      if (r <= S) simM[r] = A * simM[r];  // x A (SumofSquares...m:51)
    }
  }
  if (lane == 0) {  // first row of the reference: no polymerase yet
    double m = 0.0, pp = 0.0;
#pragma unroll
    for (int k = 0; k < NSEG; ++k) {
      m = m < b1 ? b1 : m;
      pp = pp < b2 ? b2 : pp;
    }
    simM[0] = A * m;
    simP[0] = pp;
  }
  wave_sync();
  if (MODE == MODE_FWD_RAW) {
    for (int j = lane; j < N; j += 64) {
      out0[b * ld_out + j] = simM[j];
      out1[b * ld_out + j] = simP[j];
    }
    return;
  }
  // ---- interp1 to the acquisition times (SumofSquares...m:55-56) and nansum of the squared residuals
  double ss = 0.0;
  for (int j = lane; j < N; j += 64) {
    const PointRec pt = PT[j];
    const int k = pt.k;
    const double m = fma(pt.w, simM[k + 1] - simM[k], simM[k]);
    const double pp = fma(pt.w, simP[k + 1] - simP[k], simP[k]);
    if (MODE == MODE_FWD_INTERP) {
      out0[b * ld_out + j] = m;
      out1[b * ld_out + j] = pp;
    } else {
      const double r1 = pt.y1 - m;
      ss = fmax(fma(r1, r1, ss), ss);
      const double r2 = pt.y2 - pp;
      ss = fmax(fma(r2, r2, ss), ss);
    }
  }
  if (MODE == MODE_SS) {
    ss = lane63(wave_incl_scan(ss));
    if (lane == 0) out0[b] = ss;
  }
}

template <int NSEG, int MODE>
int launch_tile(const KParams& kp, const double* theta, int64_t ld, const int32_t* cell_id, const uint8_t* active,
                int64_t B, double* out0, double* out1, int64_t ld_out, hipStream_t stream) {
  // LDS sized by the context's longest cell (64 B per point: 131 KB at 2,048 points, one wave per
  // CU); the limit is raised once, to the largest cell any context allows (ensure_dyn_lds)
  const size_t lds = (size_t)tile_lds_doubles(kp.max_n) * sizeof(double);
  auto k = tci_tile_kernel<NSEG, MODE>;
  if (ensure_dyn_lds((const void*)k, (size_t)tile_lds_doubles(TCI_MAX_POINTS) * sizeof(double)) != TCI_OK)
    return TCI_EHIP;
  hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(64), lds, stream, kp, theta, ld, cell_id, active, B, out0, out1, ld_out);
  return hipGetLastError() == hipSuccess ? TCI_OK : TCI_EHIP;
}

template <int NSEG>
int launch_tile_mode(const KParams& kp, int mode, const double* theta, int64_t ld, const int32_t* cell_id,
                     const uint8_t* active, int64_t B, double* out0, double* out1, int64_t ld_out, hipStream_t st) {
  switch (mode) {
    case MODE_SS: return launch_tile<NSEG, MODE_SS>(kp, theta, ld, cell_id, active, B, out0, out1, ld_out, st);
    case MODE_FWD_INTERP:
      return launch_tile<NSEG, MODE_FWD_INTERP>(kp, theta, ld, cell_id, active, B, out0, out1, ld_out, st);
    case MODE_FWD_RAW: return launch_tile<NSEG, MODE_FWD_RAW>(kp, theta, ld, cell_id, active, B, out0, out1, ld_out, st);
    default: return TCI_EINVAL;
  }
}

int launch_tiled(const KParams& kp, int mode, const double* theta, int64_t ld, const int32_t* cell_id,
                 const uint8_t* active, int64_t B, double* out0, double* out1, int64_t ld_out, hipStream_t st) {
  switch (kp.n_seg) {
    case 1: return launch_tile_mode<1>(kp, mode, theta, ld, cell_id, active, B, out0, out1, ld_out, st);
    case 2: return launch_tile_mode<2>(kp, mode, theta, ld, cell_id, active, B, out0, out1, ld_out, st);
    case 3: return launch_tile_mode<3>(kp, mode, theta, ld, cell_id, active, B, out0, out1, ld_out, st);
    case 4: return launch_tile_mode<4>(kp, mode, theta, ld, cell_id, active, B, out0, out1, ld_out, st);
    default: return TCI_EINVAL;
  }
}

}  // namespace

int launch(const KParams& kp, int rpl, int mode, const double* theta, int64_t ld_theta, const int32_t* cell_id,
           const uint8_t* active, int64_t B, double* out0, double* out1, int64_t ld_out, void* stream) {
  if (B <= 0) return TCI_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (rpl) {
    case 0: return launch_tiled(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    case 1: return launch_rpl<1>(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    case 2: return launch_rpl<2>(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    case 4: return launch_rpl<4>(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    case 8: return launch_rpl<8>(kp, mode, theta, ld_theta, cell_id, active, B, out0, out1, ld_out, st);
    default: return TCI_EINVAL;
  }
}

}  // namespace tci
