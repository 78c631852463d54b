// tci_eval.h -- one FP64 ssfun evaluation per wavefront on gfx950 (CDNA4), device code shared by
// the batched likelihood kernel (tci_kernels.hip) and the fused DRAM chain kernel (tci_dram.hip).
//
// One wavefront (64 lanes) evaluates one ssfun(theta, cell):
//   SumofSquaresFunction_TranscriptionCycleMCMC.m:1-64
//     -> ConstantElongationSim.m:1-67 -> GetFluorFromPolPos.m:1-71
// without ever materialising the reference's time x polymerase matrix.
//
// Cohort form. Every polymerase loaded at grid step i (ConstantElongationSim.m:60-64) has the
// same position at every later row r:  p(r,i) = (..((v*dt_i) + v*dt_{i+1}) + ..) + v*dt_{r-1},
// accumulated FORWARD exactly as x(i+1,k) = x(i,k) + v*dt(i) does. The
// c_i = floor(counter_i) - floor(counter_{i-1}) polymerases of step i form one cohort, so a
// row's stem-loop sum over polymerases is  sum_i c_i * f(p(r,i))  (GetFluorFromPolPos.m:47-66).
//
// Lane layout. Lane l owns RPL consecutive rows (slots g = RPL*l + q hold row g+1). Cohort
// values travel between slots by register rename inside a lane and one DPP wave_shr:1 across
// lanes, so row accumulators never leave registers.
//
// Loading counter. counter = counter + R(i)*dt(i) (multiply, then add; no FMA) feeds floor().
// A wave-parallel prefix sum gives every step's counter within a proven bound (<= ~530 ulp of
// the sum); floor() is taken from it unless a step lands within 2^-42 (relative) of an integer,
// in which case the wave runs the reference's serial loop (LDS, lane 0). Bit-identical to the
// serial MATLAB loop either way.
//
// Positions, fast path (uniform grid). The SS grid is t(1):d:t(end), so every step's v*dt is
// v*d up to a few ulps (delta = max |dt_j - d| is precomputed per cell). A cohort's position
// after m steps is then m*v*d within a proven bound eps_m, for EVERY cohort. If no
// representative position P_m = m*(v*d) lies within eps_m of a decision threshold (loop
// starts/ends, gene end L: the strict < / > of GetFluorFromPolPos.m:50-51,62-63), every
// (row, cohort) pair at distance m takes the branch the reference takes, so the occupancy is a
// function of the distance alone: 0 while P_m <= a, a ramp (P_m - a)*phi/(e - a) while
// a < P_m < e, phi while e < P_m < L, 0 after. With K_i = floor(counter_i) the exact cumulative
// number of polymerases loaded through step i, a row's sum over all polymerases is then
//   phi * (K[r - f_lo] - K[r - f_hi - 1])  +  sum_{m in ramp} (K[r-m] - K[r-m-1]) * F(m)
// -- O(1 + ramp length) per row instead of one term per polymerase (the reference) or per
// cohort. The ramp values use P_m instead of each cohort's exact position: ulp-level only.
//
// Positions, exact path. Otherwise (an ambiguous distance, the raw non-uniform grid of the
// plot/summary forward model, or the test hook) the wave runs the systolic sweep: each cohort
// carries its exactly-accumulated forward position, one add per (row, cohort) pair in the
// reference's order, and every branch is decided on bit-identical positions.
//
// This file is compiled with -ffp-contract=off (see build.py) so hipcc never fuses the
// multiply-then-add statements that feed floor() and the strict comparisons. Continuous parts
// (row sums, interp1, the residual sum) use explicit FMA and wave reductions; they differ from
// MATLAB only at the ulp level.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#include "tci_diag.h"
#include "tci_internal.h"

namespace tci {

namespace {


template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, ROW_MASK, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, ROW_MASK, 0xF, true);
  return __hiloint2double(hi, lo);
}

// DPP wave_shr:1 (GFX9 family; dpp_ctrl 0x138): lane l receives lane l-1, lane 0 gets 0.
__device__ __forceinline__ double wave_shr1(double x) { return dpp_f64<0x138, 0xF>(x); }

// Inclusive wave64 prefix sum in registers (DPP row_shr 1/2/4/8 inside 16-lane rows, then
// row_bcast:15 and row_bcast:31 across rows): no LDS round trips.
__device__ __forceinline__ double wave_incl_scan(double x) {
  x = x + dpp_f64<0x111, 0xF>(x);
  x = x + dpp_f64<0x112, 0xF>(x);
  x = x + dpp_f64<0x114, 0xF>(x);
  x = x + dpp_f64<0x118, 0xF>(x);
  x = x + dpp_f64<0x142, 0xA>(x);
  x = x + dpp_f64<0x143, 0xC>(x);
  return x;
}

__device__ __forceinline__ double lane63(double x);

// DPP move that writes every lane (row_mask 0xF, bound_ctrl: invalid sources read 0), so the old
// value is dead and no zero-initialised destination is needed.
template <int CTRL>
__device__ __forceinline__ double dpp_f64_all(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// The scan's value at lane 63 only (a wave sum), with the same adds in the same order there as
// wave_incl_scan: the two cross-row stages update every row (rows 0-2 end up with other partial sums,
// which no stage feeds into lane 63: lane 63 takes lane 47's row-2 total, then lane 31's rows-0..1
// total), so their moves need no zeroed destination -- 4 fewer VALU per sum.
__device__ __forceinline__ double wave_sum(double x) {
  x = x + dpp_f64<0x111, 0xF>(x);
  x = x + dpp_f64<0x112, 0xF>(x);
  x = x + dpp_f64<0x114, 0xF>(x);
  x = x + dpp_f64<0x118, 0xF>(x);
  x = x + dpp_f64_all<0x142>(x);
  x = x + dpp_f64_all<0x143>(x);
  return lane63(x);
}

// Two independent scans stage by stage (each value's adds in wave_incl_scan's order, so the same
// bits): the second one's DPP moves fill the first one's wait states.
__device__ __forceinline__ void wave_sum2(double& x, double& y) {  // wave_sum of both, interleaved
  x = x + dpp_f64<0x111, 0xF>(x);
  y = y + dpp_f64<0x111, 0xF>(y);
  x = x + dpp_f64<0x112, 0xF>(x);
  y = y + dpp_f64<0x112, 0xF>(y);
  x = x + dpp_f64<0x114, 0xF>(x);
  y = y + dpp_f64<0x114, 0xF>(y);
  x = x + dpp_f64<0x118, 0xF>(x);
  y = y + dpp_f64<0x118, 0xF>(y);
  x = x + dpp_f64_all<0x142>(x);
  y = y + dpp_f64_all<0x142>(y);
  x = x + dpp_f64_all<0x143>(x);
  y = y + dpp_f64_all<0x143>(y);
  x = lane63(x);
  y = lane63(y);
}

__device__ __forceinline__ double lane63(double x) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), 63);
  return __hiloint2double(hi, lo);
}

// Order LDS traffic between lanes of ONE wavefront (a wave's LDS ops execute in order; this
// only stops the compiler from moving accesses across the point).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave votes straight on the compare mask (the int-predicate __ballot/__any/__all round-trip
// every bool through a VGPR select and a compare: two extra VALU per vote).
// Votes are OR-ed / AND-ed as 64-bit masks on the scalar unit; the ballot operand is kept a
// single compare.
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Mask of the lanes l whose slot RPL*l + q is a loading step (g < nsteps), built on the scalar
// unit: lanes 0 .. ceil((nsteps - q) / RPL) - 1.
template <int RPL>
__device__ __forceinline__ uint64_t step_lanes(int nsteps, int q) {
  const int n = nsteps > q ? (nsteps - q + RPL - 1) / RPL : 0;
  return n >= 64 ? ~0ull : (1ull << n) - 1;
}

// max of two non-NaN doubles as one v_max_f64: fmax() makes the compiler canonicalise operands it
// cannot prove canonical (values merged from several paths), one more VALU each.
__device__ __forceinline__ double max_f64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Exponent field of a double: all ones iff the value is +-Inf or NaN. The max over the
// wave-uniform theta entries stays on the scalar unit (isfinite() would be a vector compare each).
__device__ __forceinline__ unsigned exp_bits(double x) { return (unsigned)__double2hiint(x) & 0x7ff00000u; }

// Stem-loop occupancy of one polymerase at position p (GetFluorFromPolPos.m:50-52):
//   phi                 if e < p < L
//   (p - a)*phi/(e-a)   if a < p < e      (slope precomputed: ulp-level difference only)
//   0                   otherwise (strict inequalities: p == e gives 0).
// p <= a makes (p-a)*k <= 0, so max(.,0) realises the p > a test exactly.
__device__ __forceinline__ double occupancy(double p, const SegParams& s, double L) {
  double fr = (p - s.a) * s.k;
  fr = fr > 0.0 ? fr : 0.0;
  const double full = (p > s.e && p < L) ? s.phi : 0.0;
  return p < s.e ? fr : full;
}

// Distance cut of one threshold x on the fast path: n(x) = #{m in [1, nsteps] : P_m < x}, where
// P_m = m * vd0 is the representative position m steps after loading (P_m is monotone in m).
// The cuts of all thresholds are computed at once, one threshold per lane, from an estimate of
// x / vd0 and the two exact products that should bracket x:
//   m0 = clamp(ceil(x * rcp(vd0)) - 1, 0, nsteps),  n(x) = m0  when  P_{m0} < x <= P_{m0+1}
// (m0 = 0 needs no lower product, m0 = nsteps no upper one). rcp(vd0) is v_rcp_f64, which is not
// correctly rounded: its relative error reaches 4.6e-8 on gfx950 (4.2 M samples, never exact:
// scripts/calib/rcp_f64.hip, profiles/r04_likelihood/r04d_rcp_f64_accuracy.json), so the estimate
// is off by one when x / vd0 lies within ~N * 5e-8 of an integer (N <= 2,048 steps). Such a pair does
// not bracket x and is flagged instead of trusted (a few waves in 10^5 take the exact sweep). `bad`
// also flags a bracketing product within eps of x: the same exactness test as one vote per m,
// because every other P_m is at least ~vd0 > 4 eps away from x (eps >= vd0/4 is flagged too). A
// flagged wave takes the exact sweep.
__device__ __forceinline__ int distance_cut(double x, double vd0, double rvd0, double eps, int nsteps, bool& bad) {
  // x <= 0 (no P_m with m >= 1 below it): x * rvd0 <= 0, or NaN for 0 * Inf, and the clamp gives 0
  double mc = ceil(x * rvd0) - 1.0;
  mc = fmax(mc, 0.0);                    // also NaN (v_max_f64 returns the other operand)
  mc = fmin(mc, (double)nsteps);         // also +Inf (rcp of a denormal)
  const int m0 = (int)mc;
  const double P0 = mc * vd0, P1 = (mc + 1.0) * vd0;         // the products P_m = (g + 1) * vd0 of the slots
  // bitwise, not short-circuit: straight-line lane masks (no branch, no mask rebuilt for the vote)
  const bool lo_ok = (m0 == 0) | (P0 < x);
  const bool hi_ok = (m0 == nsteps) | !(P1 < x);
  const bool near = !(eps < 0.25 * vd0) | ((m0 >= 1) & (fabs(P0 - x) <= eps)) | ((m0 < nsteps) & (fabs(P1 - x) <= eps));
  bad = near | !lo_ok | !hi_ok;
  return m0;
}

// Cuts of one evaluation (wave-uniform, SGPRs): nL = n(L); per segment and dye na = n(a), ne = n(e).
// The row sums need only three table entries per (segment, dye) and one shared one (row_sum).
template <int NSEG>
struct Cuts {
  int nL;
  int nMa[NSEG], nMe[NSEG], nPa[NSEG], nPe[NSEG];
};

// Lane j holds threshold j: 0 -> L, 1 + 4k .. 4 + 4k -> MS2 a, MS2 e, PP7 a, PP7 e of segment k.
// Returns false (take the exact sweep) when any cut is flagged.
// xt: this lane's construct threshold from the context's table (KParams::thr, loaded by the caller
// ahead of time; one load instead of 4 NSEG lane selects); lane 0 takes L, which depends on theta.
template <int NSEG>
__device__ __forceinline__ bool distance_cuts(double xt, double L, double vd0, double eps, int nsteps, int lane,
                                              Cuts<NSEG>& cu) {
  const double x = lane == 0 ? L : xt;
  bool bad;
  const int cnt = distance_cut(x, vd0, __builtin_amdgcn_rcp(vd0), eps, nsteps, bad);
  constexpr uint64_t used = (1ull << (1 + 4 * NSEG)) - 1;
  cu.nL = __builtin_amdgcn_readlane(cnt, 0);
#pragma unroll
  for (int k = 0; k < NSEG; ++k) {
    cu.nMa[k] = __builtin_amdgcn_readlane(cnt, 1 + 4 * k);
    cu.nMe[k] = __builtin_amdgcn_readlane(cnt, 2 + 4 * k);
    cu.nPa[k] = __builtin_amdgcn_readlane(cnt, 3 + 4 * k);
    cu.nPe[k] = __builtin_amdgcn_readlane(cnt, 4 + 4 * k);
  }
  return (wave_ballot(bad) & used) == 0;
}

// Exact prefix tables of the fast path, interleaved per cohort index i (LDS, 16 B per entry):
//   K_i = sum_{i' <= i} c_i'        (= floor(counter_i): polymerases loaded through step i)
//   J_i = sum_{i' <= i} i' * c_i'
// Both are integers < 2^53, exact in any summation order. KJ points at i = 0 of a table whose
// SLOTS entries below i = 0 are zeros (of SLOTS+RPL reserved), so every index r - m - 1 >= -SLOTS
// needs no clamp.
// CLAMP (the long-cell kernel): the table has ONE zero entry below i = 0 and lower indices read it.
template <bool CLAMP = false>
__device__ __forceinline__ double2 kj_at(const double2* KJ, int i) { return KJ[CLAMP ? max(i, -1) : i]; }

// Row sum of one segment of one dye on the fast path (see the header), O(1) per row, from the
// cuts na = n(a), ne = n(e), nL = n(L):
//   full  (e < P_m < L, m in [ne + 1, nL]):  phi * (K[r - ne - 1] - K[r - nL - 1])   (kL = K[r - nL - 1])
//   ramp  (a < P_m < e, m in [na + 1, ne]):  sum_m c_{r-m} * (m*vd0 - a) * k
//        = (k*vd0) * sum_m m*c_{r-m}  -  (k*a) * sum_m c_{r-m},   sum_m m*c_{r-m} = r*C - (J_A - J_E)
// with A = KJ[r - na - 1], E = KJ[r - ne - 1]. kvd = k*vd0 and ka = k*a are wave constants; C, the
// J difference and r*C - dJ are exact integers. Branch-free, so every table read of a row issues
// at once: an empty ramp (na == ne) reads A == E and adds exactly 0; an empty full region
// (ne >= nL) has K[r - ne - 1] <= kL and max(., 0) makes it exactly 0, as skipping it would.
template <bool CLAMP = false>
__device__ __forceinline__ double row_sum(const double2* KJ, int r, double rd, int na, int ne, double kL,
                                          const SegParams& s, double kvd, double ka) {
  const double2 A = kj_at<CLAMP>(KJ, r - na - 1), E = kj_at<CLAMP>(KJ, r - ne - 1);
  const double full = s.phi * fmax(E.x - kL, 0.0);
  const double C = A.x - E.x;
  const double Mc = fma(rd, C, -(A.y - E.y));  // sum of m * c_{r-m}, exact
  return fma(kvd, Mc, fma(-ka, C, full));
}

// The {K, J} table of eval_wave. RPL >= 4: stored TRANSPOSED by residue -- entry e = RPL * lane + t
// (t wave-uniform, >= -64 RPL) at slot (u mod RPL) * kKJS + u / RPL, u = e + 65 RPL -- so a wave's
// accesses to entries RPL * lane + t are 64 consecutive 16-B slots, conflict-free for ds_read_b128
// and ds_write_b128, where the plain layout puts them RPL slots apart (4-way bank conflicts at
// RPL = 4, 8-way at 8: the MI355X_MICROARCH.md §LDS lane groups). Config 4's walk (RPL = 4):
// 4,166 -> 3,894 us per launch, bitwise equal (r06g). RPL <= 2 keeps the plain layout: its 2-way
// conflicts cost less than the slot arithmetic (TestData bench launch 35.8 plain vs 36.6 us
// transposed, k_chain 218.6 vs 222.5 us per chunk, r06g). Pure addressing: the same entries, the
// same bits. Needs (2 * 64 + 1) RPL slots: eval_lds_doubles. TCI_KJ_LINEAR=1: plain at every RPL
// (the A/B).
#ifndef TCI_KJ_LINEAR
#define TCI_KJ_LINEAR 0
#endif
template <int RPL>
struct KJTable {
  static constexpr bool kPlain = TCI_KJ_LINEAR || RPL <= 2;
  static constexpr int kOff = 65 * RPL;  // u = e + kOff >= RPL for every entry a row reads
  static constexpr int kKJS = 129;       // slots per residue (u / RPL <= 128)
  static constexpr int kLg = RPL == 1 ? 0 : RPL == 2 ? 1 : RPL == 4 ? 2 : 3;
  double2* base;                         // this lane's slot 0 of residue 0 (transposed) / entry RPL * lane (plain)
  __device__ __forceinline__ KJTable(double* lds, int lane)
      : base(reinterpret_cast<double2*>(lds) + (kPlain ? RPL * lane + kOff : lane)) {}
  // slot of this lane's entry RPL * lane + t, relative to base (t uniform: scalar arithmetic)
  __device__ __forceinline__ int slot(int t) const {
    if (kPlain) return t;
    const int T = t + kOff;
    return (T & (RPL - 1)) * kKJS + (T >> kLg);
  }
  __device__ __forceinline__ double2 at(int t) const { return base[slot(t)]; }
  __device__ __forceinline__ void put(int t, double2 v) { base[slot(t)] = v; }
};

// row_sum on this lane's row RPL * lane + q + 1 of a KJTable (entries RPL * lane + q - n)
template <int RPL>
__device__ __forceinline__ double row_sum_t(const KJTable<RPL>& T, int q, double rd, int na, int ne, double kL,
                                            const SegParams& s, double kvd, double ka) {
  const double2 A = T.at(q - na), E = T.at(q - ne);
  const double full = s.phi * fmax(E.x - kL, 0.0);
  const double C = A.x - E.x;
  const double Mc = fma(rd, C, -(A.y - E.y));  // sum of m * c_{r-m}, exact
  return fma(kvd, Mc, fma(-ka, C, full));
}

template <int MODE>
__device__ __forceinline__ void write_nan(int lane, int N, int64_t b, double* out0, double* out1, int64_t ld_out) {
  if (MODE == MODE_SS) {
    if (lane == 0) out0[b] = NAN;
  } else {
    for (int j = lane; j < N; j += 64) out0[b * ld_out + j] = out1[b * ld_out + j] = NAN;
  }
}

// LDS doubles one evaluating wavefront needs: the {K,J} table (2*64*RPL + RPL entries of 16 B),
// aliased by the two simulated rows.
template <int RPL>
constexpr int eval_lds_doubles() {
  return 4 * 64 * RPL + 4 * RPL;
}

// Register-resident inputs of one evaluation: the parameter row theta (SumofSquares...m:7-13)
// and the cell's step / acquisition-point records for this lane.
template <int RPL>
struct EvalIn {
  double v, tau, ton, b1, b2, A, R;  // wave-uniform
  double dr[RPL];                     // dR of the lane's steps RPL*lane + q (any value past N-1)
  CellMeta cm;
  double thr;                         // this lane's distance-cut threshold (KParams::thr)
  StepRec st[RPL];
  PointRec pt[RPL + 1];               // points lane + 64*k, k < RPL; pt[RPL]: point 64*RPL in every lane
                                      // (wave-uniform; only N = 64*RPL + 1 has it, and lane 0 uses it)
};

// The cell's records into registers: lane l holds steps RPL*l .. RPL*l + RPL - 1 and points
// l + 64*k. RAW: the raw-time steps (forward model on raw t). A point past 64*RPL (only
// N = 64*RPL + 1 has one, on lane 0) is read only where it exists in the table.
template <int RPL, bool RAW>
__device__ __forceinline__ void load_cell(const KParams& kp, int c, int lane, EvalIn<RPL>& e) {
  const int64_t cbase = (int64_t)c * kp.cell_stride;
  const StepRec* ST = (RAW ? kp.steps_raw : kp.steps) + cbase;
  const PointRec* PT = kp.points + cbase;
  e.cm = kp.cells[c];
  e.thr = kp.thr[lane];  // with the cell's loads (a load at its use would wait there)
#pragma unroll
  for (int q = 0; q < RPL; ++q) e.st[q] = ST[RPL * lane + q];  // < cell_stride
  if (!RAW) {
#pragma unroll
    for (int k = 0; k <= RPL; ++k) {
      const int j = lane + 64 * k;
      // the tail point at a uniform address: scalar loads, no per-lane defaults to materialise
      e.pt[k] = PT[k < RPL ? j : 64 * RPL];
    }
  }
}

// One ssfun evaluation (MODE_SS: returns the SS, wave-uniform) or forward model (rows written
// to out0/out1 row b) by one wavefront, on its LDS (2 * (2*64*RPL + 2*RPL) doubles). Needs
// 2 <= N = e.cm.n <= 64*RPL + 1. aux (MODE_SS, optional): a per-lane partial on entry, its wave sum
// (lane63(wave_incl_scan), the same bits) on return -- reduced together with the SS (the DRAM chain
// kernel's prior).
template <int RPL, int NSEG, int MODE>
__device__ __forceinline__ double eval_wave(const KParams& kp, const EvalIn<RPL>& e, int lane, double* lds,
                                            int64_t b, double* __restrict__ out0, double* __restrict__ out1,
                                            int64_t ld_out, double* aux = nullptr) {
  constexpr int SLOTS = 64 * RPL;      // rows 1..SLOTS (row 0 never holds a polymerase)
  // Simulated rows j = 0..SLOTS of each dye: simM[j] = lds[1 + j], simP[j] = lds[SLOTS + 3 + j],
  // so a lane's first row RPL*lane + 1 starts 16-B aligned (paired 16-B row stores).
  constexpr int SIMM = 1, SIMP = SLOTS + 3;
  constexpr int NPT = RPL + 1;         // acquisition points per lane (N <= 64*RPL + 1)
  static_assert(SIMP + SLOTS + 1 <= 4 * SLOTS + 4 * RPL, "sim rows exceed the wave's LDS");
  double* simM = lds + SIMM;
  double* simP = lds + SIMP;
  const CellMeta& cm = e.cm;
  const double v = e.v, tau = e.tau, ton = e.ton, b1 = e.b1, b2 = e.b2, A = e.A, R = e.R;
  const double* dr = e.dr;
  const StepRec* st = e.st;
  const PointRec* pt = e.pt;
  const int N = cm.n;
  const int nsteps = N - 1;  // loading steps = rows that can hold polymerases
#if TCI_ABLATE & 16
  if (MODE == MODE_SS) {  // memory floor: every load, no compute
    double x = v + tau + ton + b1 + b2 + A + R + cm.d;
#pragma unroll
    for (int q = 0; q < RPL; ++q) x += dr[q] + st[q].dt + st[q].t;
#pragma unroll
    for (int k = 0; k < NPT; ++k) x += pt[k].w + pt[k].y1 + pt[k].y2 + (double)pt[k].k;
    return lane63(wave_incl_scan(x));
  }
#endif

  // ---- per-step setup: R_full = R + dR (SumofSquares...m:45); R<0 -> 0 (ConstantElongationSim.m:36)
  double prod[RPL];
  const unsigned ebits = max(max(max(exp_bits(v), exp_bits(tau)), max(exp_bits(ton), exp_bits(b1))),
                            max(max(exp_bits(b2), exp_bits(A)), exp_bits(R)));
  const bool fin = ebits != 0x7ff00000u;
  uint64_t nonfinite = 0;
#pragma unroll
  for (int q = 0; q < RPL; ++q) {
    nonfinite |= step_lanes<RPL>(nsteps, q) & wave_ballot(!isfinite(dr[q]));
    const double rho = fmax(R + dr[q], 0.0);  // R(R<0) = 0 (the sign of a zero cannot reach floor())
    // skipped steps add nothing (:57-60); slots past the last step have t = -Inf (tci_create), so
    // they are skipped too, whatever dR holds there
    prod[q] = !(st[q].t < ton) ? rho * st[q].dt : 0.0;
  }
  if (!fin || nonfinite != 0) {  // outside mcmcstat's finite parameter box: reported as NaN
    if (MODE != MODE_SS) write_nan<MODE>(lane, N, b, out0, out1, ld_out);
    if (aux) *aux = wave_sum(*aux);
    return NAN;
  }

  // ---- loading counter (ConstantElongationSim.m:60-61): DPP prefix sum + exactness proof
  double K[RPL];
  {
    double loc[RPL];
    double s = prod[0];  // (0.0 + prod[0] only turns a -0 into +0, which no count can see)
    loc[0] = s;
#pragma unroll
    for (int q = 1; q < RPL; ++q) {
      s = s + prod[q];
      loc[q] = s;
    }
#if TCI_ABLATE & 8
    const double excl = 0.0;
#else
    const double excl = wave_shr1(wave_incl_scan(s));
#endif
    uint64_t amb = 0;
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      const double Sq = excl + loc[q];
      const double eps = Sq * 0x1p-42;  // >> the (g + 16) ulp bound between any two summation orders
      const double Kq = floor(Sq);
      const double f = Sq - Kq;         // exact (Sterbenz): the fraction
      amb |= wave_ballot(f < eps) | wave_ballot(f + eps >= 1.0);  // an integer within eps of Sq
      K[q] = Kq;
    }
    if ((kp.force_exact & 1) || amb != 0) {
      // Exact path: the reference's serial loop, counter = counter + R(i)*dt(i).
#pragma unroll
      for (int q = 0; q < RPL; ++q) simM[RPL * lane + q] = prod[q];
      wave_sync();
      if (lane == 0) {
        double counter = 0.0;
        for (int g = 0; g < nsteps; ++g) {
          counter = counter + simM[g];
          simP[g] = floor(counter);
        }
      }
      wave_sync();
#pragma unroll
      for (int q = 0; q < RPL; ++q) {
        const int g = RPL * lane + q;
        K[q] = simP[min(g, nsteps - 1)];  // constant past the last step, as the scan gives
      }
      wave_sync();
    }
  }

  SegParams sm[NSEG], sp[NSEG];
#pragma unroll
  for (int k = 0; k < NSEG; ++k) {
    sm[k] = kp.ms2[k];
    sp[k] = kp.pp7[k];
  }
  const double L = kp.L0 + tau * v;                 // L_MS2 = L_PP7 (GetFluorFromPolPos.m:19-20), no FMA
  const double pstop = L > kp.emax ? L : kp.emax;  // f(p) == 0 for every p >= pstop
  // Row sums per segment: assigned by the fast path, accumulated from 0 by the exact sweep, 0 for
  // v <= 0 (zeroed in those branches only: no zero moves on the fast path).
  double accM[NSEG][RPL], accP[NSEG][RPL];
  auto zero_acc = [&]() {
#pragma unroll
    for (int q = 0; q < RPL; ++q)
#pragma unroll
      for (int k = 0; k < NSEG; ++k) accM[k][q] = accP[k][q] = 0.0;
  };

  // v <= 0: every position stays <= 0 <= loop start, so no polymerase is ever lit (the exact
  // branch's zeros, without the sweep).
  {
    bool fast = v > 0.0 && MODE != MODE_FWD_RAW && !(kp.force_exact & 2);
    const double vd0 = v * cm.d;
    Cuts<NSEG> cu;
    // ---- distance cuts and their exactness proof (distance_cut)
    // |p(r, r-m) - P_m| <= v * (m*delta + (m+4)*u*m*(d+delta)) for every m <= nsteps; eps is
    // twice that at m = nsteps, precomputed per cell up to the factor v (CellMeta::eps_v).
    // No P_m equals a threshold unless it is within eps > 0 of it (then the wave goes exact),
    // so on the fast path #(P_m <= x) == #(P_m < x) and one count per threshold suffices.
    if (fast) fast = distance_cuts<NSEG>(e.thr, L, vd0, v * cm.eps_v, nsteps, lane, cu);
    if (fast) {
      // ---- {K, J} prefix tables (exact) and O(1) row sums
      double jloc[RPL], js = 0.0;
      {
        const double kprev = wave_shr1(K[RPL - 1]);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
          const int g = RPL * lane + q;
          const double cg = K[q] - (q == 0 ? kprev : K[q - 1]);  // 0 past the last step (K constant)
          js = fma((double)g, cg, js);                           // integers < 2^53: exact
          jloc[q] = js;
        }
      }
      const double jexcl = wave_incl_scan(js) - js;  // integers < 2^53: exact, as a shifted scan
      // KJ[i], i in [-SLOTS, SLOTS): the SLOTS entries below i = 0 are zeros (KJTable: transposed)
      KJTable<RPL> KJ(lds, lane);
#pragma unroll
      for (int q = 0; q < RPL; ++q) {
        KJ.put(q, make_double2(K[q], jexcl + jloc[q]));
        KJ.put(q - SLOTS, make_double2(0.0, 0.0));  // [-SLOTS, 0): every index a row reads
      }
      wave_sync();
      double kvdM[NSEG], kaM[NSEG], kvdP[NSEG], kaP[NSEG];
#pragma unroll
      for (int k = 0; k < NSEG; ++k) {
        kvdM[k] = sm[k].k * vd0;
        kaM[k] = sm[k].ka;
        kvdP[k] = sp[k].k * vd0;
        kaP[k] = sp[k].ka;
      }
#pragma unroll
      for (int q = 0; q < RPL; ++q) {
        const int r = RPL * lane + q + 1;
        const double rd = (double)r;
        // entries r - n - 1 of this lane's rows: entry RPL * lane + q - n, one scalar slot per cut
        const double kL = KJ.at(q - cu.nL).x;  // shared by every segment and dye (L_MS2 = L_PP7)
#pragma unroll
        for (int k = 0; k < NSEG; ++k) {
#if TCI_ABLATE & 1
          accM[k][q] = KJ.at(q).x + (double)cu.nMa[k];
          accP[k][q] = KJ.at(q).y + (double)cu.nL;
#else
          accM[k][q] = row_sum_t(KJ, q, rd, cu.nMa[k], cu.nMe[k], kL, sm[k], kvdM[k], kaM[k]);
          accP[k][q] = row_sum_t(KJ, q, rd, cu.nPa[k], cu.nPe[k], kL, sp[k], kvdP[k], kaP[k]);
#endif
        }
        // one row's table reads in flight at a time: issued all at once, the 4*NSEG + 1 reads of
        // every row would hold 16 VGPRs per (row, segment) and push the register-bound chain
        // kernels (tci_dram.hip) into spills
        if (RPL * NSEG > 2) __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      // ---- exact systolic sweep: at iteration s slot g holds cohort g-s+1 with its forward position
      zero_acc();
      double cc[RPL], p[RPL], vd[RPL];
      if (v > 0.0) {
      {
        const double kprev = wave_shr1(K[RPL - 1]);
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
          const int g = RPL * lane + q;
          const double km1 = q == 0 ? kprev : K[q - 1];
          cc[q] = g < nsteps ? K[q] - km1 : 0.0;
          p[q] = 0.0;
          vd[q] = g < nsteps ? v * st[q].dt : 0.0;  // v*dt(i), rounded once (:64)
        }
      }
      for (int s = 1; s <= nsteps; ++s) {
        if (s > 1) {
          const double pin = wave_shr1(p[RPL - 1]);
          const double cin = wave_shr1(cc[RPL - 1]);
#pragma unroll
          for (int q = RPL - 1; q >= 1; --q) {
            p[q] = p[q - 1];
            cc[q] = cc[q - 1];
          }
          p[0] = pin;
          cc[0] = cin;
        }
        uint64_t alive = 0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
          p[q] = p[q] + vd[q];  // x(i+1,k) = x(i,k) + v*dt(i)
#pragma unroll
          for (int k = 0; k < NSEG; ++k) {
            accM[k][q] = fma(cc[q], occupancy(p[q], sm[k], L), accM[k][q]);
            accP[k][q] = fma(cc[q], occupancy(p[q], sp[k], L), accP[k][q]);
          }
          alive |= step_lanes<RPL>(nsteps, q) & wave_ballot(cc[q] > 0.0) & wave_ballot(p[q] < pstop);
        }
        if (alive == 0) break;
      }
      }  // v > 0
    }
  }
  wave_sync();  // every {K,J}-table read is done before the rows overwrite the LDS

  // ---- basal floor inside the segment loop (GetFluorFromPolPos.m:54-57,66-69), x A (SumofSquares...m:51)
  //      Rows past the last step are stored too (never read): stores stay whole 16-B pairs.
  double rowM[RPL], rowP[RPL];
#pragma unroll
  for (int q = 0; q < RPL; ++q) {
    // MS2(MS2 < basal) = basal == max(MS2, basal): the sums are finite and >= 0 here
    double m = max_f64(accM[0][q], b1), pp = max_f64(accP[0][q], b2);
#pragma unroll
    for (int k = 1; k < NSEG; ++k) {
      m = max_f64(m + accM[k][q], b1);
      pp = max_f64(pp + accP[k][q], b2);
    }
    rowM[q] = A * m;
    rowP[q] = pp;
  }
  if (RPL == 1) {
    simM[lane + 1] = rowM[0];
    simP[lane + 1] = rowP[0];
  } else {
#pragma unroll
    for (int q = 0; q < RPL; q += 2) {
      *reinterpret_cast<double2*>(simM + RPL * lane + q + 1) = make_double2(rowM[q], rowM[q + 1]);
      *reinterpret_cast<double2*>(simP + RPL * lane + q + 1) = make_double2(rowP[q], rowP[q + 1]);
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
    return 0.0;
  }

  // ---- interp1 back to the acquisition times (SumofSquares...m:55-56) and nansum of the
  //      squared residuals over [MS2, PP7] (:57-64).
  double ss = 0.0;
#if TCI_ABLATE & 4
  if (MODE == MODE_SS) return lane63(wave_incl_scan(simM[lane] + simP[lane] + pt[0].y1 + pt[1].y2));
#endif
#pragma unroll
  for (int kk = 0; kk < NPT; ++kk) {
    if (kk == RPL && N <= 64 * RPL) break;  // uniform: only N = 64*RPL + 1 has a tail point
    const int j = lane + 64 * kk;
    // interp1: NaN outside the grid comes in through w = NaN (PointRec)
    const int k = pt[kk].k;
    const double w = pt[kk].w;
    const double m = fma(w, simM[k + 1] - simM[k], simM[k]);
    const double pp = fma(w, simP[k + 1] - simP[k], simP[k]);
    if (MODE == MODE_FWD_INTERP) {
      if (j < N) {  // the tail (kk == RPL): lane 0 only
        out0[b * ld_out + j] = m;
        out1[b * ld_out + j] = pp;
      }
    } else if (kk < RPL || lane == 0) {  // the tail point is every lane's pt[RPL]: lane 0 adds it
      // nansum drops NaN data, NaN simulation and the all-NaN padding points (j >= N) alike:
      // fma(r, r, ss) >= ss unless it is NaN, and max() returns the non-NaN operand.
      const double r1 = pt[kk].y1 - m;
      ss = fmax(fma(r1, r1, ss), ss);
      const double r2 = pt[kk].y2 - pp;
      ss = fmax(fma(r2, r2, ss), ss);
    }
  }
  if (MODE == MODE_SS && aux) {
    double x = *aux;
    wave_sum2(ss, x);
    *aux = x;
    return ss;
  }
  return MODE == MODE_SS ? wave_sum(ss) : 0.0;
}

}  // namespace

}  // namespace tci
