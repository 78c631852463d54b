// tci_dram.hip -- GPU-resident batched DRAM (delayed-rejection adaptive Metropolis) for the
// TranscriptionCycleInference fit: the caller of the likelihood hot path.
//
// The reference runs one mcmcstat chain per cell inside a parfor (TranscriptionCycleMCMC.m:161)
// with options nsimu, updatesigma=1, qcov=J0, burnintime, adaptint=100, method 'dram' (:263-270).
// mcmcstat (github.com/mjlaine/mcmcstat, mcmcrun.m) is not vendored and has no pinned version;
// the algorithm below restates its published DRAM (Haario, Laine, Mira & Saksman 2006) as
// mcmcrun implements it:
//   stage 1   newpar = oldpar + randn(1,npar)*R;  out of bounds -> rejected, ssfun not called;
//             alpha12 = min(1, exp(-0.5*(newss-oldss)/sigma2 - 0.5*(newprior-oldprior)))
//   stage 2   (stage 1 rejected) newpar2 = oldpar + randn(1,npar)*R/drscale
//             alpha32 = min(1, exp(-0.5*(newss-newss2)/sigma2 - 0.5*(newprior-newprior2)))
//             l2 = exp(-0.5*(newss2-oldss)/sigma2 - 0.5*(newprior2-oldprior))
//             q1 = exp(-0.5*(|(newpar2-newpar)*iR|^2 - |(oldpar-newpar)*iR|^2)), iR = inv(R)
//             -- with newpar = oldpar + z1*R and newpar2 = oldpar + z2*R/drscale this is
//             exp(-0.5*(|z2/drscale - z1|^2 - |z1|^2)) exactly, which is what is evaluated (no iR)
//             alpha13 = l2*q1*(1-alpha32)/(1-alpha12)
//   sigma2    1/sigma2 ~ Gamma((N0+N)/2, scale 2/(N0*S20 + oldss)), N0 = 0, N = length(ydata)
//   adapt     every adaptint steps: burn-in (step < burnintime): R scaled by 1/burnin_scale or
//             burnin_scale when the window's rejection rate is > 0.95 or < 0.05; afterwards
//             covupd over all chain rows so far, R = chol(cov + qcovadj*I) * adascale
//   prior     sum(((theta - mu)./sig).^2) over parameters with finite sig (dR: N(0, 50), :254)
// The proposal factor R is FP64, as mcmcstat's double chol: a chain's R is a packed upper triangle
// (P(P+1)/2 doubles: DramState::Rd, the only device copy), staged into LDS for the proposal
// products while it fits beside a pass of normals (every TestData cell), read from global memory
// beyond (configs 4/5) in the same MFMA order.
// Randomness: Philox4x32-10 keyed by (seed), counter (chain, step, purpose, index) -- the
// stream is reproducible and independent of launch geometry (MATLAB's MT19937 is not
// reproducible here, so chain parity with the reference is statistical only).
//
// Kernels: one wavefront per chain for propose/accept (4 chains per 256-thread block), one
// 256-thread workgroup per chain for adaptation. The SS of the proposals is the batched
// likelihood kernel (tci_kernels.hip), launched between these kernels on device buffers.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <type_traits>

#include "tci_diag.h"
#include "tci_dram_internal.h"
#include "tci_eval.h"
#include "tci_tile16.h"
#include "tci_adapt_map.h"

namespace tci {

namespace {

constexpr int kThreads = 256;  // one workgroup (4 waves) per chain

enum Purpose : uint32_t { P_NORM1 = 1, P_U1 = 2, P_NORM2 = 3, P_U2 = 4, P_GAMMA = 5 };


// The 32 x 32 -> 64-bit product of a Philox round in one v_mad_u64_u32: the compiler's
// v_mul_lo_u32 + v_mul_hi_u32 pair is two quarter-rate instructions (draws pass: TestData 105.0 ->
// 97.5 us per chunk, config 4 62.1 -> 52.7 ms per 1,000 steps, r03v; the same exact product).
__device__ __forceinline__ uint64_t mul64(uint32_t a, uint32_t b) {
  uint64_t r, carry;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(carry) : "v"(a), "v"(b));
  return r;
}

// Philox4x32-10 (Salmon et al. 2011).
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = mul64(0xD2511F53u, c.x), p1 = mul64(0xCD9E8D57u, c.z);
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = make_uint4(__builtin_amdgcn_bitop3_b32(hi1, c.y, k.x, 0x96), lo1, __builtin_amdgcn_bitop3_b32(hi0, c.w, k.y, 0x96),
                   lo0);  // 0x96: three-input xor
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ uint4 rng(uint64_t seed, int64_t chain, int64_t step, uint32_t purpose, uint32_t idx) {
  const uint4 ctr = make_uint4((uint32_t)chain, (uint32_t)step, ((uint32_t)(step >> 32) & 0x00FFFFFFu) | (purpose << 24),
                               idx);
  return philox(ctr, make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
}

// Uniform in (0,1) from 64 random bits (53-bit mantissa, never 0 or 1).
__device__ __forceinline__ double u01(uint32_t a, uint32_t b) {
  const uint64_t x = (((uint64_t)a << 32) | b) >> 11;
  return ((double)x + 0.5) * 0x1p-53;
}

// Standard normals of the stream (chain, step, purpose), kNPer per Philox call (item), Box-Muller:
// two 53-bit uniforms per pair, log / sincospi in FP64, 2 normals per call -- the double-precision
// N(0,1) of mcmcstat's randn (no 2^-24 discretisation, no tail cut). (An fp32 Box-Muller measured
// 5-7 % faster fits, profiles/r02_likelihood/r02k_dram_libs.jsonl; not worth the narrower proposals.)
constexpr int kNPer = 2;

// The transcendental pair in plain FP64 arithmetic -- correctly rounded +, *, /, sqrt and fma
// only, so the CPU restatement (oracle/tci_dram_oracle.c: bm_neg2log, bm_sincospi) repeats them
// bit for bit -- at about half the instructions of the libm log and sincospi (each within ~2 ulp).
//   -2 log(u), u in (0, 1): u = m 2^e, m in [sqrt(1/2), sqrt(2)); log m = 2 atanh(s) with
//   s = (m - 1)/(m + 1), |s| < 0.1716: s (1 + z/3 + .. + z^9/19), z = s^2 (truncation < 1e-19);
//   e ln 2 as fdlibm's ln2_hi (32 bits: e ln2_hi is exact) + ln2_lo.
__device__ __forceinline__ double bm_neg2log(double u) {
  double m = __builtin_amdgcn_frexp_mant(u);  // [1/2, 1)
  int e = __builtin_amdgcn_frexp_exp(u);
  if (m < 0.70710678118654752440) {
    m = m * 2.0;
    e = e - 1;
  }
  const double sv = (m - 1.0) / (m + 1.0);
  const double z = sv * sv;
  double q = 1.0 / 19;
  q = fma(q, z, 1.0 / 17);
  q = fma(q, z, 1.0 / 15);
  q = fma(q, z, 1.0 / 13);
  q = fma(q, z, 1.0 / 11);
  q = fma(q, z, 1.0 / 9);
  q = fma(q, z, 1.0 / 7);
  q = fma(q, z, 1.0 / 5);
  q = fma(q, z, 1.0 / 3);
  const double lm = fma(sv * z, q, sv);  // log(m) / 2
  const double de = (double)e;
  return -2.0 * (de * 6.93147180369123816490e-01 + (2.0 * lm + de * 1.90821492927058770002e-10));
}
//   sin(pi x), cos(pi x) for x in (0, 2): t = 2x quarter turns, n = rint(t), r = t - n in
//   [-1/2, 1/2] (exact); phi = (pi/2) r by its Taylor series to r^17 / r^16 (truncation < 1e-17),
//   then the quadrant n mod 4.
__device__ __forceinline__ void bm_sincospi(double x, double& sn, double& cs) {
  const double t = 2.0 * x;
  const double n = __builtin_rint(t);
  const double r = t - n, r2 = r * r;
  double ps = 6.0669357311061955e-12;
  ps = fma(ps, r2, -6.688035109811468e-10);
  ps = fma(ps, r2, 5.692172921967927e-08);
  ps = fma(ps, r2, -3.598843235212085e-06);
  ps = fma(ps, r2, 0.00016044118478735983);
  ps = fma(ps, r2, -0.004681754135318688);
  ps = fma(ps, r2, 0.07969262624616705);
  ps = fma(ps, r2, -0.6459640975062463);
  ps = fma(ps, r2, 1.5707963267948966);
  const double sp = ps * r;
  double pc = 6.565963114979473e-11;
  pc = fma(pc, r2, -6.386603083791852e-09);
  pc = fma(pc, r2, 4.710874778818172e-07);
  pc = fma(pc, r2, -2.5202042373060607e-05);
  pc = fma(pc, r2, 0.0009192602748394266);
  pc = fma(pc, r2, -0.02086348076335296);
  pc = fma(pc, r2, 0.25366950790104803);
  pc = fma(pc, r2, -1.2337005501361697);
  const double cp = fma(pc, r2, 1.0);
  const int k = (int)n & 3;
  const double a = (k & 1) ? cp : sp, b = (k & 1) ? sp : cp;  // sin, cos of (pi/2)(k & 1) + phi, up to sign
  sn = (k & 2) ? -a : a;
  cs = ((k + 1) & 2) ? -b : b;
}

__device__ __forceinline__ void normals_at(uint64_t seed, int64_t c, int64_t step, uint32_t purpose, int item,
                                           double (&z)[kNPer]) {
  const uint4 r = rng(seed, c, step, purpose, (uint32_t)item);
  const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
  const double rad = sqrt(bm_neg2log(u1));
  double sn, cs;
  bm_sincospi(2.0 * u2, sn, cs);
  z[0] = rad * cs;
  z[1] = rad * sn;
}

// z[0..P) of stream `purpose` into LDS, one Philox call per thread and round.
__device__ __forceinline__ void draw_normals(uint64_t seed, int64_t c, int64_t step, uint32_t purpose, int P,
                                             double* z, int t) {
  for (int q = t; kNPer * q < P; q += kThreads) {
    double n[kNPer];
    normals_at(seed, c, step, purpose, q, n);
#pragma unroll
    for (int h = 0; h < kNPer; ++h)
      if (kNPer * q + h < P) z[kNPer * q + h] = n[h];
  }
}

__device__ __forceinline__ double uniform_at(uint64_t seed, int64_t c, int64_t step, uint32_t purpose) {
  const uint4 r = rng(seed, c, step, purpose, 0);
  return u01(r.x, r.y);
}

// Gamma(a, 1) by Marsaglia & Tsang (a >= 1 here: a = N/2 >= 2) as the product d*v; a Gamma(a, scale)
// variate is (d*v)*scale. The unit variate depends only on the stream and a, so the fused engine
// draws it ahead of the chain (k_draws) and the scale (2/SS of the current state) is applied when
// it is used: the same bits as gamma_at.
template <int = 0>  // the body, inlined where the caller's register budget needs it (k_draws)
__device__ __forceinline__ double gamma_unit_t(uint64_t seed, int64_t c, int64_t step, double a) {
  const double d = a - 1.0 / 3.0, cc = 1.0 / sqrt(9.0 * d);
  for (uint32_t it = 0; it < 1024; ++it) {
    const uint4 r = rng(seed, c, step, P_GAMMA, it);
    const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
    const double x = sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
    const uint4 r2 = rng(seed, c, step, P_GAMMA, it | 0x80000000u);
    const double u = u01(r2.x, r2.y);
    double v = 1.0 + cc * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double x2 = x * x;
    if (u < 1.0 - 0.0331 * x2 * x2) return d * v;  // squeeze (implies the log test)
    if (log(u) < 0.5 * x2 + d - d * v + d * log(v)) return d * v;
  }
  return a;  // unreachable in practice (acceptance > 0.95 per try)
}
__device__ double gamma_unit(uint64_t seed, int64_t c, int64_t step, double a) { return gamma_unit_t(seed, c, step, a); }
__device__ __forceinline__ double gamma_at(uint64_t seed, int64_t c, int64_t step, double a, double scale) {
  return gamma_unit(seed, c, step, a) * scale;
}

// Wave sum, result in every lane: DPP inclusive scan + lane 63 (tci_eval.h), no LDS round trips.
// Every engine reduces through this one function, so their bits agree.
__device__ __forceinline__ double wsum64(double x) { return wave_sum(x); }

// Acceptance terms shared by every engine (the same expressions, so the same bits):
//   log of a Metropolis ratio  -0.5*(ss_new - ss_old)/s2 - 0.5*(prior_new - prior_old), with the
//   division by s2 taken as a product with the precision ip = 1/s2 (computed once per state);
//   the delayed-rejection test  u2 < alpha13 = l2*q1*(1-alpha32)/(1-alpha12)  as the product form
//   u2*(1-alpha12) < l2*q1*(1-alpha32)  (stage 2 runs only after a stage-1 rejection, so
//   alpha12 < 1 there and the two tests agree in exact arithmetic).
__device__ __forceinline__ double dram_log_ratio(double ss_new, double ss_old, double pr_new, double pr_old, double ip) {
  return -0.5 * (ss_new - ss_old) * ip - 0.5 * (pr_new - pr_old);
}
__device__ __forceinline__ bool dram_dr_accept(double u2, double a12, double a32, double l2, double q1) {
  return u2 * (1.0 - a12) < l2 * q1 * (1.0 - a32);
}

// Prior precision of one entry: 1/sig for a finite sig, 0 for sig = +Inf (no prior: the entry adds
// exactly 0). Every engine forms ((th - mu) * (1/sig))^2 from it -- one rounding more than MATLAB's
// ((th - mu)./sig).^2 per entry, the same bits in every engine; the chain kernels take the
// reciprocal once per chunk instead of dividing at every evaluation.
__device__ __forceinline__ double prior_prec(double sg) { return isfinite(sg) ? 1.0 / sg : 0.0; }

// Prior SS sum(((th - mu)./sig).^2) over finite sig (mcmcstat's default priorfun) by ONE wave:
// lane l sums j = l, l + 64, .. in order, then a fixed xor-shuffle tree. Both engines call this,
// so the bits agree.
__device__ double wave_prior(const double* th, const double* mu, const double* sig, int P, int lane) {
  double s = 0.0;
  for (int j = lane; j < P; j += 64) {
    const double z = (th[j] - mu[j]) * prior_prec(sig[j]);
    s += z * z;
  }
  return wsum64(s);
}

// |z2/drscale - z1|^2 and |z1|^2 (the delayed-rejection ratio, header) by ONE wave.
__device__ double2 wave_q(const double* z1, const double* z2, double inv_ds, int P, int lane) {
  double q21 = 0.0, q01 = 0.0;
  for (int j = lane; j < P; j += 64) {
    const double d = z2[j] * inv_ds - z1[j];
    q21 += d * d;
    q01 += z1[j] * z1[j];
  }
  return make_double2(wsum64(q21), wsum64(q01));
}

// Workgroup sum (all threads get the result). red: LDS scratch of >= 4 doubles.
__device__ double block_sum(double x, double* red) {
  x = wsum64(x);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = x;
  __syncthreads();
  const double s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

// prior SS: sum(((th - mu) ./ sig).^2) (mcmcstat default priorfun)
__device__ double prior_ss(const double* th, const double* mu, const double* sig, int P, double* red) {
  double s = 0.0;
  for (int j = threadIdx.x; j < P; j += kThreads) {
    const double z = (th[j] - mu[j]) * prior_prec(sig[j]);
    s += z * z;
  }
  return block_sum(s, red);
}

// Packed upper triangle (row i at i*P - i*(i-1)/2) of a chain's R in FP64 -- mcmcstat's double
// chol -- (st.Rd, chain c at c * tri_stride(ld), the only device copy), so a workgroup stages it
// into LDS with one coalesced copy.
__device__ __forceinline__ int tri_off(int i, int P) { return i * P - (i * (i - 1)) / 2; }
__host__ __device__ inline int64_t tri_stride(int64_t ld) { return dram_tri_stride(ld); }
__device__ __forceinline__ void store_R(const DramState& st, int64_t c, int P, int i, int j, double v) {
  if (j >= i) st.Rd[c * tri_stride(st.ld) + tri_off(i, P) + j - i] = v;
}
// Burn-in scaling R <- R * s, on the packed triangle (the lower triangle is zero).
__device__ __forceinline__ void scale_R(const DramState& st, int64_t c, int P, double s, int t, int nth) {
  double* Rd = st.Rd + c * tri_stride(st.ld);
  for (int e = t; e < P * (P + 1) / 2; e += nth) Rd[e] = Rd[e] * s;
}
// The copy by LDS-DMA (global_load_lds_dwordx4: 1 KiB = 128 doubles per wave-instruction, no
// registers): every piece is in flight at once, and the caller's next work (the draws pass's
// normals) runs while they land; the caller waits for vmcnt and then barriers. Rl: 16-byte aligned,
// room for the triangle rounded up to 128 doubles (the source stride is, dram_tri_stride).
template <int NTH>
__device__ __forceinline__ void load_R_glds(double* Rl, const DramState& st, int64_t c, int P) {
  const double* src = st.Rd + c * tri_stride(st.ld);
  const int pieces = (P * (P + 1) / 2 + 127) >> 7;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  for (int k = w; k < pieces; k += NTH / 64)
    __builtin_amdgcn_global_load_lds((const void*)(src + 128 * k + 2 * lane),
                                     (__attribute__((address_space(3))) void*)(Rl + 128 * k), 16, 0, 0);
}
template <int NTH = kThreads>
__device__ void load_R(double* Rl, const DramState& st, int64_t c, int P) {
  const double* src = st.Rd + c * tri_stride(st.ld);
  const int tri = P * (P + 1) / 2;
#pragma unroll 4
  for (int e = threadIdx.x; e < tri; e += NTH) Rl[e] = src[e];
}

// Proposal products U[r][j] = sum_{i<=j} Z[r][i] R[i][j] for r < M <= 16*MT rows of normals (LDS,
// row stride zs) and the chain's packed FP64 R (LDS or global); store(r, j, value) receives every product.
// One v_mfma_f64_16x16x4_f64 per 4-row k-step of a 16 x 16 (row tile, column tile) block:
// A = Z[row = lane&15][k = lane>>4], B = R[k = lane>>4][col = lane&15], D row = (lane>>4) + 4 q,
// col = lane&15 (cdna_hip_programming.md f64 MFMA map). Column tiles go to the 4 waves in snake order
// from the last (costliest) tile down (balanced triangle costs: 12/11/11/11 k-step units for 9 tiles,
// where ascending order gave one wave 18); a wave runs its (up to CT) column tiles x MT row tiles together, so one
// A and one B fragment load feed CT*MT independent MFMA chains. Each tile skips the k-steps below
// the triangle. A product depends only on its row of Z and the fixed k order, so every MT/CT
// instance (the batched engine's 1-row proposals, the fused engine's 32-row draws) gives the same
// bits.
// top: the highest column tile of this call (tiles top, top-1, .. top+1-NWV*CT are computed):
// (P + 15)/16 - 1 for one call; wider rows loop over tops (propose_block).
// PF > 0 (R in global memory): every k-step also loads the R values of all CT tiles PF k-steps
// ahead, so an L2/HBM round trip overlaps PF k-steps' MFMAs instead of preceding them.
template <int MT, int CT, int NWV, class Store, int PF = 0>  // NWV: waves sharing the column tiles; PF: prefetch depth
__device__ __forceinline__ void mfma_zr(const double* Z, int zs, int M, const double* Rl, int P, int top, Store store) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int row = lane & 15, kq = lane >> 4;
  int nt[CT], kmx[CT];
#pragma unroll
  for (int g = 0; g < CT; ++g) {
    nt[g] = top - (NWV * g + ((g & 1) ? NWV - 1 - w : w));  // uniform: costliest first, snake order
    kmx[g] = nt[g] >= 0 ? min(16 * nt[g] + 15, P - 1) : -1;
  }
  // The tiles are in decreasing k-extent (kmx[0] >= kmx[1] >= ..), so the k-steps split into
  // phases with a compile-time number ng of active tiles: every inner loop is branch-free (the
  // accumulators stay in place) and runs ng*MT independent MFMA chains.
  f64x4 acc[CT][MT];
#pragma unroll
  for (int g = 0; g < CT; ++g)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[g][m] = f64x4{0.0, 0.0, 0.0, 0.0};
  int i0 = 0;
  // raw R values of k-step i0n for every tile (inactive tiles read a valid clamped entry)
  auto load_b = [&](int i0n, double* b) {
    const int icn = min(i0n + kq, P - 1);
    const int tof = tri_off(icn, P) - icn;
#pragma unroll
    for (int g = 0; g < CT; ++g) {
      const int jc = min(max(16 * nt[g] + row, 0), P - 1);
      b[g] = Rl[tof + (jc >= icn ? jc : icn)];
    }
  };
  double bq[PF > 0 ? PF : 1][CT];  // bq[d]: k-step i0 + 4 d (rotated every step)
#pragma unroll
  for (int d = 0; d < PF; ++d) load_b(4 * d, bq[d]);
#pragma unroll
  for (int ng = CT; ng >= 1; --ng) {
    for (; i0 <= kmx[ng - 1]; i0 += 4) {  // tiles g < ng still need k-step i0
      const int i = i0 + kq;
      const int ic = i < P ? i : P - 1;
      double bcur[CT];
      if (PF > 0) {
#pragma unroll
        for (int g = 0; g < CT; ++g) bcur[g] = bq[0][g];
#pragma unroll
        for (int d = 0; d + 1 < PF; ++d)
#pragma unroll
          for (int g = 0; g < CT; ++g) bq[d][g] = bq[d + 1][g];
        load_b(i0 + 4 * PF, bq[PF > 0 ? PF - 1 : 0]);
      }
      double a[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int r = 16 * m + row;
        const double zv = Z[(r < M ? r : M - 1) * zs + ic];  // clamped: rows >= M read row M-1, zeroed
        a[m] = (r < M && i < P) ? zv : 0.0;
      }
      const int toff = tri_off(ic, P) - ic;
#pragma unroll
      for (int g = 0; g < ng; ++g) {
        const int j = 16 * nt[g] + row;
        const int jc = j < P ? j : P - 1;
        const double rv = PF > 0 ? bcur[g] : Rl[toff + (jc >= ic ? jc : ic)];
        const double b = (i <= j && j < P) ? rv : 0.0;
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[g][m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b, acc[g][m], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < CT; ++g) {
    const int j = 16 * nt[g] + row;
    if (kmx[g] < 0 || j >= P) continue;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * m + kq + 4 * q;
        if (r < M) store(r, j, acc[g][m][q]);
      }
  }
}
// k_draws' z*R with R in global memory (L2): mfma_zr's tiles, products and k order (the same
// bits) as a software pipeline. The R values of k-step i0 + 4 PF are loaded while k-step i0 runs,
// into a ring of PF register sets (no copies, so each load has PF k-steps to land); Z is read
// without exec-mask branches (rows past M read row M - 1, whose products are never stored; k past
// P reads finite LDS -- the zero-filled pads or the next row's normals -- and meets a zero R entry);
// the packed-R row offset advances by one addition per k-step. Phases run whole rings: the extra
// k-steps past a tile's last row multiply zero R entries and leave its accumulators' bits as they
// are (accumulators start at +0, products of finite values with 0 are +-0).
template <int MT, int CT, int NWV, int PF, class Store>
__device__ __forceinline__ void mfma_zr_pf(const double* Z, int zs, int M, const double* __restrict__ Rg, int P,
                                           int top, Store store) {
  static_assert(PF >= 1 && PF <= 4, "reads reach k = P + 4 PF - 2: draws_lds_bytes pads 16 doubles");
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int row = lane & 15, kq = lane >> 4;
  int nt[CT], kmx[CT], jv[CT], jc[CT];
#pragma unroll
  for (int g = 0; g < CT; ++g) {
    nt[g] = top - (NWV * g + ((g & 1) ? NWV - 1 - w : w));  // uniform: costliest first, snake order
    kmx[g] = nt[g] >= 0 ? min(16 * nt[g] + 15, P - 1) : -1;
    const int j = 16 * nt[g] + row;
    jv[g] = j < P ? j : -1;  // R row i contributes to column j while i <= jv (never past P)
    jc[g] = min(max(j, 0), P - 1);
  }
  // this lane's A entries at k-step 0 (k = kq)
  int za[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) za[m] = min(16 * m + row, M - 1) * zs + kq;
  // f(i) = tri_off(i, P) - i = i (2P - 1 - i) / 2: entry (i, j) of the packed R at f(i) + j. f rises
  // to i = P - 1, f(P) = f(P - 1), then falls (below 0 past 2P - 1), so max(f, 0) + j stays inside
  // [0, P(P+1)/2) for the loads past a tile's rows (their values are never used). f(i + 4) = f(i) +
  // 4P - 10 - 4i.
  int fl = kq * (P - 1) - (kq * (kq - 1)) / 2;  // f(il + kq) for the next load's k-step il
  int il = 0;
  auto load_next = [&](double* b) {
#pragma unroll
    for (int g = 0; g < CT; ++g) b[g] = Rg[max(fl, 0) + jc[g]];
    fl += 4 * P - 10 - 4 * il - 4 * kq;
    il += 4;
  };
  f64x4 acc[CT][MT];
#pragma unroll
  for (int g = 0; g < CT; ++g)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[g][m] = f64x4{0.0, 0.0, 0.0, 0.0};
  double bq[PF][CT];
#pragma unroll
  for (int d = 0; d < PF; ++d) load_next(bq[d]);
  int i0 = 0;
#pragma unroll
  for (int ng = CT; ng >= 1; --ng) {
    while (i0 <= kmx[ng - 1]) {  // uniform
#pragma unroll
      for (int d = 0; d < PF; ++d) {
        const int i = i0 + kq;
        double a[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) a[m] = Z[za[m] + i0];
#pragma unroll
        for (int g = 0; g < ng; ++g) {
          const double b = i <= jv[g] ? bq[d][g] : 0.0;
#pragma unroll
          for (int m = 0; m < MT; ++m) acc[g][m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b, acc[g][m], 0, 0, 0);
        }
        load_next(bq[d]);
        i0 += 4;
      }
    }
  }
#pragma unroll
  for (int g = 0; g < CT; ++g) {
    const int j = 16 * nt[g] + row;
    if (kmx[g] < 0 || j >= P) continue;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * m + kq + 4 * q;
        if (r < M) store(r, j, acc[g][m][q]);
      }
  }
}
constexpr int kZrCT = 5;  // column tiles per wave and call: 20 per 4-wave call (P <= 320 in one call)

// Dynamic LDS of the per-stage kernels (vector stride L = ld >= P): z, y, red and the chain's R
// as packed FP64.
struct Smem {
  double* z;
  double* y;
  double* red;
  double* Rl;
  int L;
};
// R is staged into LDS only while it fits (stage_r_lds); longer rows read the packed R from
// global memory in the same MFMA order (the same bits).
__host__ __device__ inline bool stage_r_lds(int64_t L) { return (2 * L + 8) * 8 + (L * (L + 1) / 2) * 8 + 16 <= 150 * 1024; }
__host__ __device__ inline int64_t stage_lds_bytes(int64_t L) {
  return (2 * L + 8) * 8 + (stage_r_lds(L) ? (L * (L + 1) / 2) * 8 : 0) + 16;
}
__device__ __forceinline__ Smem stage_smem(double* dyn, int L) {
  Smem m;
  m.z = dyn;
  m.y = dyn + L;
  m.red = dyn + 2 * L;
  m.Rl = dyn + 2 * L + 8;
  m.L = L;
  return m;
}

// Delayed-rejection proposal ratio q1 = exp(-0.5*(|(y2-y1) iR|^2 - |(x-y1) iR|^2)) from the
// normals: (y2-y1) iR = z2/drscale - z1 and (x-y1) iR = -z1 (z1, z2 in LDS).
__device__ double dr_q1(const double* z1, const double* z2, double inv_ds, int P, double* red) {
  if (threadIdx.x < 64) {
    const double2 q = wave_q(z1, z2, inv_ds, P, threadIdx.x);
    if (threadIdx.x == 0) red[0] = exp(-0.5 * (q.x - q.y));
  }
  __syncthreads();
  const double q1 = red[0];
  __syncthreads();
  return q1;
}

// Prior SS (wave_prior by wave 0), broadcast to the block.
__device__ double prior_block(const double* th, const double* mu, const double* sig, int P, double* red) {
  if (threadIdx.x < 64) {
    const double v = wave_prior(th, mu, sig, P, threadIdx.x);
    if (threadIdx.x == 0) red[0] = v;
  }
  __syncthreads();
  const double v = red[0];
  __syncthreads();
  return v;
}

// Draw z (stream `purpose`), y = base + scale * z*R into LDS and global `out`; returns in-bounds.
__device__ bool propose_block(const DramState& st, const DramParams& p, int64_t c, int64_t step, uint32_t purpose,
                              const double* base, double scale, int P, double* out, Smem& sm) {
  const int64_t ld = st.ld;
  draw_normals(p.seed, st.key[c], step, purpose, P, sm.z, threadIdx.x);
  const bool rl = stage_r_lds(st.ld);
  if (rl) load_R(sm.Rl, st, c, P);
  __syncthreads();
  double* U = sm.y;
  const int us = sm.L;
  const auto put = [=](int r, int j, double v) { U[r * us + j] = v; };
  for (int top = ((P + 15) >> 4) - 1; top >= 0; top -= 4 * kZrCT) {
    if (rl) mfma_zr<1, kZrCT, 4>(sm.z, sm.L, 1, sm.Rl, P, top, put);  // two calls: each one's R pointer has
    else mfma_zr<1, kZrCT, 4>(sm.z, sm.L, 1, st.Rd + c * tri_stride(st.ld), P, top, put);  // a known address space
  }
  __syncthreads();
  int inb = 1;
  for (int j = threadIdx.x; j < P; j += kThreads) {
    const double v = base[j] + scale * sm.y[j];
    out[j] = v;
    sm.y[j] = v;
    inb &= (v >= st.lower[c * ld + j] && v <= st.upper[c * ld + j]) ? 1 : 0;
  }
  return __syncthreads_and(inb) != 0;
}

__global__ __launch_bounds__(kThreads) void k_init(DramState st, const double* __restrict__ qdiag,
                                                   const double* __restrict__ s2_0) {
  __shared__ double red[8];
  const int64_t c = blockIdx.x;
  if (c >= st.n_chains) return;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  double* cv = st.cov + c * dram_cov_stride(ld);
  for (int64_t e = threadIdx.x; e < dram_cov_stride(ld); e += kThreads) cv[e] = 0.0;
  for (int64_t e = threadIdx.x; e < tri_stride(ld); e += kThreads) st.Rd[c * tri_stride(ld) + e] = 0.0;
  __syncthreads();
  for (int j = threadIdx.x; j < P; j += kThreads) {
    store_R(st, c, P, j, j, sqrt(qdiag[c * ld + j]));  // R = chol(qcov), qcov = J0 diagonal (:230)
    st.cmean[c * ld + j] = 0.0;
  }
  const double pr = prior_ss(st.theta + c * ld, st.pmu + c * ld, st.psig + c * ld, P, red);
  if (threadIdx.x == 0) {
    st.prior[c] = pr;
    st.sigma2[c] = s2_0[c];
    st.wsum[c] = 0.0;
    st.naccept[c] = 0;
    st.nrej_win[c] = 0;
    st.nevals[c] = 1;  // the initial ssfun call
  }
}

// ---- Chain records. Every engine LOGS each chain row: the state into its window slot
// (DramState::window, slot (row - 1) % p.win, the covupd window when adapting) and its s2 into the
// same slot of DramState::s2log. The records are kept window by window (p.win rows from row 1, the
// same partition for every engine):
//   * the window's column sums (the adaptation's batch mean);
//   * the posterior mean / M2 of rows >= stats_from (:276-301): the window's rows as one batch --
//     shifted sums S1 = sum(x - K), S2 = sum((x - K)^2) with K the running mean (or, before any
//     statistics row, the window's first row), batch mean K + S1/nb and M2 S2 - S1^2/nb -- merged
//     into the running values by the pairwise formula (Chan, Golub & LeVeque): the Welford
//     recurrence's result in exact arithmetic, with no per-row division;
//   * the same for sqrt(s2) over all rows and the sum of s2 (:302-303);
//   * the thinned output rows.
// Every sum runs over the window's rows in row order from 0.0, so every engine has the same bits:
// k_chain adds each row as it is decided (ColAcc / S2Acc on its record waves; a window that spans
// chunks continues from DramState::wsumv / wacc1 / wacc2 / s2acc), k_walk and k_stats read the
// window's logs back at its end (window_records, window_s2_records). (Summing the s2 log at the
// window's end in k_chain too: 226.9 -> 228.4 us per chunk, r04j.)
__device__ __forceinline__ int64_t log_slot(const DramParams& p, int64_t row) { return (row - 1) % p.win; }
// Whether the step that made the row in `slot` moved the chain (accepted a proposal): the
// adaptation's runs of equal rows (window_runs), recorded by the engines as they decide the rows
// instead of re-read and compared by the adaptation. (An accepted proposal equal to the state in
// every entry would split a run in two: the same sum in exact arithmetic.)
__device__ __forceinline__ void log_run(const DramState& st, const DramParams& p, int64_t c, int64_t slot, bool f) {
  st.runf[c * p.win + slot] = f ? 1 : 0;
}

// The batched engine's per-step log (one workgroup per chain).
__device__ void log_row_block(const DramState& st, const DramParams& p, int64_t c, int64_t row, int P, const double* th,
                              double s2, bool moved) {
  const int64_t slot = log_slot(p, row);
  double* w = st.window + (c * p.win + slot) * st.ld;
  for (int j = threadIdx.x; j < P; j += kThreads) w[j] = th[j];
  if (threadIdx.x == 0) {
    st.s2log[c * p.win + slot] = s2;
    log_run(st, p, c, slot, moved);
  }
}

struct S2Stats {
  double sum, qmean, qm2;
};

__global__ __launch_bounds__(kThreads) void k_init_stats(DramState st, DramParams p) {
  const int64_t c = blockIdx.x;
  if (c >= st.n_chains) return;
  const int P = st.npar[c];
  for (int j = threadIdx.x; j < P; j += kThreads) {
    st.smean[c * st.ld + j] = 0.0;
    st.sm2[c * st.ld + j] = 0.0;
  }
  if (threadIdx.x == 0) {
    st.s2sum[c] = 0.0;
    st.sq_mean[c] = 0.0;
    st.sq_m2[c] = 0.0;
  }
  log_row_block(st, p, c, 1, P, st.theta + c * st.ld, st.sigma2[c], true);  // chain row 1: the initial state
  // k_chain's running sums of the first window after row 1 (ColAcc / S2Acc::add of row 1, K = row 1)
  const bool in_stats = p.stats_from <= 1;
  for (int j = threadIdx.x; j < P; j += kThreads) {
    const double x = st.theta[c * st.ld + j], d = x - x;
    st.wsumv[c * st.ld + j] = 0.0 + x;
    st.wacc1[c * st.ld + j] = in_stats ? 0.0 + d : 0.0;
    st.wacc2[c * st.ld + j] = in_stats ? fma(d, d, 0.0) : 0.0;
  }
  if (st.chain_out != nullptr && p.thin > 0 && p.n_keep > 0)  // row 1 is always kept (k_chain writes rows >= 2)
    for (int j = threadIdx.x; j < P; j += kThreads) st.chain_out[c * st.ld + j] = st.theta[c * st.ld + j];
  if (threadIdx.x == 0) {
    if (st.s2_out != nullptr && p.thin > 0 && p.n_keep > 0) st.s2_out[c] = st.sigma2[c];
    const double s2 = st.sigma2[c], dq = sqrt(s2) - sqrt(s2);
    st.s2acc[3 * c + 0] = 0.0 + s2;
    st.s2acc[3 * c + 1] = 0.0 + dq;
    st.s2acc[3 * c + 2] = fma(dq, dq, 0.0);
  }
}

__global__ __launch_bounds__(kThreads) void k_propose1(DramState st, DramParams p) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  Smem sm = stage_smem(dyn, (int)st.ld);
  const int64_t c = blockIdx.x;
  if (c >= st.n_chains) return;
  const int64_t step = *st.step;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  const bool inb = propose_block(st, p, c, step, P_NORM1, st.theta + c * ld, 1.0, P, st.prop1 + c * ld, sm);
  if (threadIdx.x == 0) {
    st.act1[c] = inb ? 1 : 0;
    if (inb) st.nevals[c] += 1;
  }
}

__global__ __launch_bounds__(kThreads) void k_accept1(DramState st, DramParams p) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  Smem sm = stage_smem(dyn, (int)st.ld);
  const int64_t c = blockIdx.x;
  if (c >= st.n_chains) return;
  const int64_t step = *st.step;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  const bool inb = st.act1[c] != 0;
  double* th = st.theta + c * ld;
  const double* y1 = st.prop1 + c * ld;
  double a12 = 0.0, pr1 = 0.0;
  bool acc = false;
  if (inb) {
    pr1 = prior_block(y1, st.pmu + c * ld, st.psig + c * ld, P, sm.red);
    a12 = fmin(1.0, exp(dram_log_ratio(st.ss1[c], st.ss[c], pr1, st.prior[c], 1.0 / st.sigma2[c])));
    acc = uniform_at(p.seed, st.key[c], step, P_U1) < a12;
  }
  if (acc) {
    for (int j = threadIdx.x; j < P; j += kThreads) th[j] = y1[j];
    if (threadIdx.x == 0) {
      st.ss[c] = st.ss1[c];
      st.prior[c] = pr1;
      st.naccept[c] += 1;
    }
  }
  __syncthreads();
  bool inb2 = false;
  if (!acc && p.ntry >= 2)  // delayed rejection: second try with R / drscale
    inb2 = propose_block(st, p, c, step, P_NORM2, th, 1.0 / p.drscale, P, st.prop2 + c * ld, sm);
  if (threadIdx.x == 0) {
    st.a12[c] = a12;
    st.prior1[c] = pr1;
    st.acc1[c] = acc ? 1 : 0;
    st.act2[c] = inb2 ? 1 : 0;
    if (inb2) st.nevals[c] += 1;
  }
}

__global__ __launch_bounds__(kThreads) void k_accept2(DramState st, DramParams p) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  Smem sm = stage_smem(dyn, (int)st.ld);
  const int64_t c = blockIdx.x;
  if (c >= st.n_chains) return;
  const int64_t step = *st.step;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  double* th = st.theta + c * ld;
  bool acc2 = false;
  if (p.ntry >= 2 && st.act2[c] != 0) {  // stage 2 was proposed (stage 1 rejected) and is in bounds
    const double* y2 = st.prop2 + c * ld;
    const double pr2 = prior_block(y2, st.pmu + c * ld, st.psig + c * ld, P, sm.red);
    const double s2 = st.sigma2[c], ss2 = st.ss2[c], ss1 = st.ss1[c], a12 = st.a12[c];
    // ss1 = +Inf (stage 1 out of bounds) gives alpha32 = 0, alpha12 = 0
    const double ip = 1.0 / s2;
    const double a32 = fmin(1.0, exp(dram_log_ratio(ss1, ss2, st.prior1[c], pr2, ip)));
    const double l2 = exp(dram_log_ratio(ss2, st.ss[c], pr2, st.prior[c], ip));
    draw_normals(p.seed, st.key[c], step, P_NORM1, P, sm.z, threadIdx.x);
    draw_normals(p.seed, st.key[c], step, P_NORM2, P, sm.y, threadIdx.x);
    __syncthreads();
    const double q1 = dr_q1(sm.z, sm.y, 1.0 / p.drscale, P, sm.red);
    acc2 = dram_dr_accept(uniform_at(p.seed, st.key[c], step, P_U2), a12, a32, l2, q1);
    if (acc2) {
      for (int j = threadIdx.x; j < P; j += kThreads) th[j] = y2[j];
      if (threadIdx.x == 0) {
        st.ss[c] = ss2;
        st.prior[c] = pr2;
        st.naccept[c] += 1;
      }
    }
  }
  if (threadIdx.x == 0) {
    if (!(st.acc1[c] != 0 || acc2)) st.nrej_win[c] += 1;  // no stage moved the chain
    // sigma2 Gibbs update (updatesigma = 1, :265): 1/sigma2 ~ Gamma(N/2, scale 2/oldss)
    if (p.updatesigma) st.sigma2[c] = 1.0 / gamma_at(p.seed, st.key[c], step, 0.5 * (double)st.nobs[c], 2.0 / st.ss[c]);
  }
  __syncthreads();
  log_row_block(st, p, c, step, P, st.theta + c * st.ld, st.sigma2[c], st.acc1[c] != 0 || acc2);
}

__global__ void k_step_incr(int64_t* step) {
  if (threadIdx.x == 0) *step += 1;
}



// ---- Fused chain engine. Per chunk of chain rows between two adaptations (R fixed):
//   k_draws  every random quantity of the chunk that does not depend on the chain state, for all
//            chains and steps in one wide launch: the proposal offsets u1 = z1*R and u2 = z2*R
//            (MFMA tiles of 8 steps x 2 stages), the delayed-rejection norms |z2/drscale - z1|^2
//            and |z1|^2, the two acceptance uniforms and the unit Gamma variate of the sigma2 draw;
//   k_chain  one workgroup per chain walks the chunk's rows with ONE workgroup barrier per step:
//            waves 0 and 1 evaluate ssfun at the stage-1 and stage-2 proposals concurrently (stage
//            2 is used only when stage 1 rejects, so only the latency changes), wave 2 computes the
//            priors and records the previous row, wave 3 records the previous sigma2. Every wave
//            keeps its own copy of theta in registers and takes the same acceptance decision from
//            the values exchanged at the barrier; the next step's draws are prefetched meanwhile.
// Same RNG keys, reductions and operation order as the batched engine above: the two engines
// produce identical chains (tests/test_dram_gpu.py).

// Normals of both stages for `ns` steps from `step` into rows 2 k (stage 1, P_NORM1) and 2 k + 1
// (stage 2, P_NORM2) of Z (row stride L), one Philox call per thread and round.
template <int NTH>
__device__ __forceinline__ void draw_block_normals(uint64_t seed, int64_t c, int64_t step, int ns, int P, bool two,
                                                   double* Z, int L) {
  const int np = (P + kNPer - 1) / kNPer;
  const int rows = 2 * ns;
  for (int k = threadIdx.x; k < rows * np; k += NTH) {
    const int r = k / np, q = k - r * np;
    double* z = Z + r * L;
    double n[kNPer];
    if ((r & 1) && !two) {
#pragma unroll
      for (int h = 0; h < kNPer; ++h) n[h] = 0.0;
    } else {
      normals_at(seed, c, step + (r >> 1), (r & 1) ? P_NORM2 : P_NORM1, q, n);
    }
#pragma unroll
    for (int h = 0; h < kNPer; ++h)
      if (kNPer * q + h < P) z[kNPer * q + h] = n[h];
  }
}

constexpr int kDrawsWPE = 3;             // waves per SIMD k_draws is compiled for (<= 168 VGPRs): at 4
                                          // (128 VGPRs) it spilled 34 VGPRs, 76.9 -> 75.5 us per TestData
                                          // chunk at 3 (r05dw; three 37 KB workgroups per CU)
constexpr int kDrawsPF = 4;               // R values prefetched this many k-steps ahead (mfma_zr PF): 4 against
                                          // 2, per launch, split z*R (TestData) 53.3 -> 51.3 us, WALK (config
                                          // 4) 4,300 -> 4,119 us (r06pfd, r06pfc4); the extra k-steps of a
                                          // whole ring multiply zero R entries (the same bits)
constexpr int kDrawMT = 2;                // MFMA row tiles per pass (16 rows each), 4-wave workgroups
enum DrawSlot { D_Q1 = 0, D_U1 = 1, D_U2 = 2, D_G = 3 };  // scalar slots of a draws row

// Dynamic LDS of k_draws: one pass's normals (2 x 8 x MT rows of stride L). The chain's packed
// FP64 R is read from global memory (L2) with a kDrawsPF-deep prefetch: staging it in LDS beside the
// normals (74 KB at P = 136) left one workgroup per CU, and that layout took 144 us per TestData
// chunk against 105 us with R from L2 and four 35 KB workgroups per CU (r03n/r03o).
// (+ 8 doubles: mfma_zr_pf's reads past the last row's P entries, zeroed with the pads)
__host__ __device__ inline int64_t draws_lds_bytes(int64_t L, int mt = kDrawMT) { return (2 * 8 * mt * L + 16) * 8; }
// WALK (thousands of chains): their R triangles (171 KB per chain at P = 207, 1.7 GB for config
// 4) stream from HBM, once per pass, so the passes there are twice as long -- 4 row tiles (64 rows)
// in an 8-wave workgroup of 256-VGPR waves, one per CU (106 KB of normals): the R traffic per row
// halves (config 4 ablations, r04t: z*R 1.51 ms of the pass's 2.31 ms per launch).
constexpr int kDrawMTWalk = 4;
__host__ __device__ inline bool draws_walk_wide(int64_t L) { return draws_lds_bytes(L, kDrawMTWalk) <= 150 * 1024; }
// Passes per workgroup: every workgroup reads the chain's R once per pass. FUSED (a few hundred
// chains): 2 (1: 108.8, 2: 104.7, 4: 123.7 us per TestData chunk); WALK (thousands of chains, P =
// 207): 4, fewer and longer workgroups reading R fewer times.
// fused engine: 1 pass per k_draws workgroup (2: 80.4 vs 77.9 us per chunk, r04np); WALK: 4
__host__ __device__ inline int draws_passes(bool walk) { return walk ? 4 : 1; }

// The split draws pass (k_chain's engine, DramParams::split). The draws that do not depend on R --
// the normals, the delayed-rejection ratio q1, the two uniforms and the unit Gamma variate -- are
// written into the NEXT chunk's draws buffer (two buffers, alternating) by extra workgroups of the
// k_chain launch that walks the current chunk: k_chain's 299 chain workgroups leave a CU's second
// workgroup slot free on 213 of 256 CUs and their rounds are latency-bound. The extra workgroups
// come after the chain workgroups in the grid (dispatched in order, so they only take slots the
// chains left) and loop over the (chain, kRngSteps-step) units. k_draws<.., FromBuf> then only copies
// the normals into its LDS tile and multiplies them by the chain's new R, in place. (The first chunk's
// units: k_draws_rng, one launch before the loop.) Same normals_at / wave_q / uniform_at /
// gamma_unit_t calls as k_draws: the same bits.
constexpr int kRngSteps = 8;
__host__ __device__ inline int64_t draws_rng_lds_bytes(int64_t L) { return (2 * kRngSteps * L + 16) * 8; }
// Units first_unit, first_unit + stride, .. of chain rows s_begin..s_end into `draws` (that chunk's
// buffer), by one kThreads workgroup; Z: 2 kRngSteps L doubles of LDS.
__device__ __forceinline__ void draws_rng_units(const DramState& st, const DramParams& p, double* draws,
                                                int64_t s_begin, int64_t s_end, int64_t first_unit, int64_t stride,
                                                double* Z) {
  constexpr int NW = kThreads / 64;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t ld = st.ld;
  const int L = (int)ld;
  const int64_t DW = draw_stride(ld);
  const double inv_ds = 1.0 / p.drscale;
  const int64_t nb = (s_end - s_begin + kRngSteps) / kRngSteps;  // units per chain
  const int64_t nunits = st.n_chains * nb;
  for (int64_t u = first_unit; u < nunits; u += stride) {
    const int64_t c = u / nb;
    const int64_t step0 = s_begin + (u - c * nb) * kRngSteps;
    const int ns = (int)min<int64_t>(kRngSteps, s_end - step0 + 1);
    const int P = st.npar[c];
    const int64_t key = st.key[c];
    double* d0 = draws + (c * p.chunk - s_begin + step0) * DW;  // row of step step0 + k: d0 + k * DW
    draw_block_normals<kThreads>(p.seed, key, step0, ns, P, p.ntry >= 2, Z, L);
    __syncthreads();
    for (int r = w; r < 2 * ns; r += NW) {
      double* dz = d0 + (r >> 1) * DW + (r & 1) * ld;
      for (int j = lane; j < P; j += 64) dz[j] = Z[r * L + j];
    }
    for (int k = w; k < ns; k += NW) {
      const double2 q = wave_q(Z + 2 * k * L, Z + (2 * k + 1) * L, inv_ds, P, lane);
      if (lane == 0) d0[k * DW + 2 * ld + D_Q1] = exp(-0.5 * (q.x - q.y));  // as dr_q1
    }
    if ((int)threadIdx.x < ns) {
      const int64_t step = step0 + threadIdx.x;
      double* sc = d0 + threadIdx.x * DW + 2 * ld;
      sc[D_U1] = uniform_at(p.seed, key, step, P_U1);
      sc[D_U2] = uniform_at(p.seed, key, step, P_U2);
      sc[D_G] = p.updatesigma ? gamma_unit_t(p.seed, key, step, 0.5 * (double)st.nobs[c]) : 1.0;
    }
    __syncthreads();  // Z is rewritten by the next unit
  }
}
__global__ __launch_bounds__(kThreads) void k_draws_rng(DramState st, DramParams p, int64_t s_begin, int64_t s_end) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  draws_rng_units(st, p, st.draws, s_begin, s_end, blockIdx.x, gridDim.x, dyn);
}

// The split form's normals, already in the draws rows (k_draws_rng), into the pass's LDS tile: one
// row per wave and loop, coalesced over j (entries past P keep the tile's zeros).
template <int NWD>
__device__ __forceinline__ void load_block_normals(const double* d0, int64_t DW, int64_t ld, int ns, int P, double* Z,
                                                   int L) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  for (int r = w; r < 2 * ns; r += NWD) {
    const double* dz = d0 + (r >> 1) * DW + (r & 1) * ld;
    for (int j = lane; j < P; j += 64) Z[r * L + j] = dz[j];
  }
}

// NWD waves per workgroup, CT column tiles per wave and MFMA call (launch_chain_t: 4 and 2); longer
// rows loop over calls. The wave count and CT only move column tiles between waves and calls: same
// bits. FromBuf: the split form (k_draws_rng above wrote the normals and scalars; z*R only).
template <int NWD, int CT, int MT = kDrawMT, int WPE = kDrawsWPE, bool FromBuf = false>
__global__ __launch_bounds__(64 * NWD) __attribute__((amdgpu_waves_per_eu(WPE))) void k_draws(DramState st, DramParams p, int64_t s_begin, int64_t s_end, int npass) {
  constexpr int kDrawWaves = NWD, kDrawThreads = 64 * NWD;
  constexpr int kDrawCT = CT;
  constexpr int kDrawSteps = 8 * MT;  // steps per pass
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  const int64_t c = blockIdx.x, by = blockIdx.y;
  if (c >= st.n_chains) return;
  const int64_t ld = st.ld;
  const int L = (int)ld;
  const int P = st.npar[c];
  const int64_t key = st.key[c];
  const int64_t DW = draw_stride(ld);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  double* Z = dyn;
  // finite LDS under every z*R read (mfma_zr_pf): the pads past P and past the last row stay zero
  for (int e = threadIdx.x; e < 2 * kDrawSteps * L + 16; e += kDrawThreads) Z[e] = 0.0;
  __syncthreads();
  const double* Rg = st.Rd + c * tri_stride(ld);
  const double a = 0.5 * (double)st.nobs[c];
  const double inv_ds = 1.0 / p.drscale;
  double* drow = st.draws + (c * p.chunk - s_begin) * DW;  // row of step s: drow + s * DW
  for (int pass = 0; pass < npass; ++pass) {
    const int64_t step0 = s_begin + (by * npass + pass) * kDrawSteps;
    if (step0 > s_end) break;  // uniform over the workgroup
    const int ns = (int)min<int64_t>(kDrawSteps, s_end - step0 + 1);
    // z*R straight to the draws rows: row r of Z is step step0 + r/2, stage r&1
    double* d0 = drow + step0 * DW;
    if (FromBuf) load_block_normals<kDrawWaves>(d0, DW, ld, ns, P, Z, L);
    else if (!(TCI_DRAWS_ABLATE & 1)) draw_block_normals<kDrawThreads>(p.seed, key, step0, ns, P, p.ntry >= 2, Z, L);
    __syncthreads();
    const auto put = [=](int r, int j, double v) { d0[(r >> 1) * DW + (r & 1) * ld + j] = v; };
    // WALK's short pass (a 100-step chunk's last: 3 x 32 + 4 steps) runs only the row tiles it fills
    // -- an instance with fewer tiles, the same products (each depends only on its row of Z and the k
    // order): config 4 2,381 -> 2,289 us per launch (r05p); the fused engine's one-launch instance
    // spilled more with it (77.4 -> 78.1 us per TestData chunk) and keeps one instance; its split
    // (FromBuf, 117 VGPRs) form has the room: 54.6 -> 53.5 us per chunk (r06t1; XCD-grouped chain
    // blocks, cdna_hip_programming.md T1, measured slower: 54.9 -> 60.5, r06t2)
    if (!(TCI_DRAWS_ABLATE & 2))
      for (int top = ((P + 15) >> 4) - 1; top >= 0; top -= kDrawWaves * kDrawCT) {
        if ((MT > 2 || FromBuf) && 2 * ns <= 16)
          mfma_zr_pf<1, kDrawCT, kDrawWaves, kDrawsPF>(Z, L, 2 * ns, Rg, P, top, put);
        else if (MT > 2 && 2 * ns <= 32)
          mfma_zr_pf<(MT > 2 ? 2 : MT), kDrawCT, kDrawWaves, kDrawsPF>(Z, L, 2 * ns, Rg, P, top, put);
        else
          mfma_zr_pf<MT, kDrawCT, kDrawWaves, kDrawsPF>(Z, L, 2 * ns, Rg, P, top, put);
      }
    if (!FromBuf)
      for (int k = w; k < ns; k += kDrawWaves) {
        const double2 q = wave_q(Z + 2 * k * L, Z + (2 * k + 1) * L, inv_ds, P, lane);
        if (lane == 0) d0[k * DW + 2 * ld + D_Q1] = exp(-0.5 * (q.x - q.y));  // as dr_q1
      }
    __syncthreads();  // Z is rewritten by the next pass
  }
  // the scalar draws of the workgroup's steps, one step per thread
  const int64_t step = s_begin + by * npass * kDrawSteps + threadIdx.x;
  if (!FromBuf && !(TCI_DRAWS_ABLATE & 4) && threadIdx.x < npass * kDrawSteps && step <= s_end) {
    double* sc = drow + step * DW + 2 * ld;
    sc[D_U1] = uniform_at(p.seed, key, step, P_U1);
    sc[D_U2] = uniform_at(p.seed, key, step, P_U2);
    sc[D_G] = p.updatesigma ? gamma_unit_t(p.seed, key, step, a) : 1.0;
  }
}

// wave_prior on register-held vectors (entry k of lane l is j = l + 64 k; rs[k] = prior_prec of
// its sig): the same per-lane order and shuffle tree, so the same bits.
template <int NJ>
__device__ __forceinline__ double prior_part(const double* y, const double* mu, const double* rs, int P, int lane) {
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    if (lane + 64 * k < P) {
      const double z = (y[k] - mu[k]) * rs[k];
      s += z * z;
    }
  }
  return s;
}
template <int NJ>
__device__ __forceinline__ double wave_prior_reg(const double* y, const double* mu, const double* rs, int P, int lane) {
  return wsum64(prior_part<NJ>(y, mu, rs, P, lane));
}

// The fused engines' per-row logs (k_chain / k_walk: one wave writes a row).
template <int NJ>
__device__ __forceinline__ void log_row(const DramState& st, const DramParams& p, int64_t c, int64_t slot, int P,
                                        const double* th, int lane) {
  double* w = st.window + (c * p.win + slot) * st.ld;
#pragma unroll
  for (int k = 0; k < NJ; ++k)
    if (lane + 64 * k < P) w[lane + 64 * k] = th[k];
}
__device__ __forceinline__ void log_s2(const DramState& st, const DramParams& p, int64_t c, int64_t slot, double s2) {
  st.s2log[c * p.win + slot] = s2;
}


// Pairwise merge of a batch (nb values, shifted sums S1, S2 about K) into running (n, mean, M2).
__device__ __forceinline__ void stats_merge(double na, double nb, double K, double S1, double S2, double& mean,
                                            double& m2) {
  if (nb <= 0.0) return;
  const double db = S1 / nb;                 // batch mean - K
  const double m2b = fma(-S1, db, S2);       // sum (x - mean_b)^2
  if (na <= 0.0) {
    mean = K + db;
    m2 = m2b;
    return;
  }
  const double n = na + nb, d = (K - mean) + db;  // batch mean - running mean
  mean = fma(d, nb / n, mean);
  m2 = m2 + m2b + d * d * (na * nb / n);
}

__device__ __forceinline__ int64_t win_first(const DramParams& p, int64_t row) { return (row - 1) / p.win * p.win + 1; }
__device__ __forceinline__ bool kept_row(const DramParams& p, int64_t row, int64_t& k) {
  if (p.thin <= 0 || (row - 1) % p.thin != 0) return false;
  k = (row - 1) / p.thin;
  return k < p.n_keep;
}

// A window's column sums (lanes: columns j = lane + 64 k, k < NJ), added row by row in row order.
template <int NJ>
struct ColAcc {
  double ws[NJ], S1[NJ], S2[NJ], K[NJ];
  int64_t first, sf;
  bool kfirst;  // no statistics row before the window: K = the window's first statistics row (row sf:
                // a sample of the rows summed, so S2 - S1^2/nb cancels no more than a variance does; the
                // window's first row, which may precede stats_from, gave a chain stuck far from it an M2
                // of rounding noise, even negative)
  __device__ void setup(const DramParams& p, int64_t row) {
    first = win_first(p, row);
    sf = max(first, p.stats_from);
    kfirst = first <= p.stats_from;
  }
  __device__ void zero() {
#pragma unroll
    for (int k = 0; k < NJ; ++k) ws[k] = S1[k] = S2[k] = K[k] = 0.0;
  }
  __device__ __forceinline__ void add(int64_t row, const double* x) {
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      if (kfirst && row == sf) K[k] = x[k];
      ws[k] = ws[k] + x[k];
      if (row >= sf) {
        const double d = x[k] - K[k];
        S1[k] = S1[k] + d;
        S2[k] = fma(d, d, S2[k]);
      }
    }
  }
  // the window's records at its last row `last` (columns jl + 64 k): merged into the running
  // statistics, the column sums kept for the adaptation
  __device__ void finish(const DramState& st, const DramParams& p, int64_t c, int64_t last, int P, int jl) {
    const int64_t ld = st.ld;
    const double na = (double)max<int64_t>(first - p.stats_from, 0), nb = (double)max<int64_t>(last - sf + 1, 0);
    double mean[NJ], m2[NJ];
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const int j = jl + 64 * k;
      mean[k] = j < P ? st.smean[c * ld + j] : 0.0;
      m2[k] = j < P ? st.sm2[c * ld + j] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const int j = jl + 64 * k;
      stats_merge(na, nb, K[k], S1[k], S2[k], mean[k], m2[k]);
      if (j < P) {
        st.smean[c * ld + j] = mean[k];
        st.sm2[c * ld + j] = m2[k];
        st.wsumv[c * ld + j] = ws[k];
      }
    }
  }
};

// The same for s2 (one value per row; lane 0 of k_chain's kSigWave, uniform in window_records).
struct S2Acc {
  double sum, S1, S2, K;
  __device__ __forceinline__ void add(double s2) { add_dq(s2, sqrt(s2) - K); }
  __device__ __forceinline__ void add_dq(double s2, double dq) {  // dq = sqrt(s2) - K
    sum = sum + s2;
    S1 = S1 + dq;
    S2 = fma(dq, dq, S2);
  }
  __device__ void finish(const DramState& st, int64_t c, int64_t first, int64_t last) {
    double qmean = st.sq_mean[c], qm2 = st.sq_m2[c];
    stats_merge((double)(first - 1), (double)(last - first + 1), K, S1, S2, qmean, qm2);
    st.s2sum[c] += sum;
    st.sq_mean[c] = qmean;
    st.sq_m2[c] = qm2;
  }
};

// The s2 records of the window ending at row `last` from its log, by one wave (k_chain, k_walk): 64
// rows per pass in lanes, sqrt(s2) - K lane-parallel, then added in row order through lane
// broadcasts (S2Acc::add's arithmetic); with_out: also the thinned s2 rows.
__device__ void window_s2_records(const DramState& st, const DramParams& p, int64_t c, int64_t last, int lane,
                                  bool with_out) {
  const int64_t first = win_first(p, last);
  const int nrow = (int)(last - first + 1);
  const double* lg = st.s2log + c * p.win;
  S2Acc q{0.0, 0.0, 0.0, first > 1 ? st.sq_mean[c] : sqrt(lg[0])};
  for (int r0 = 0; r0 < nrow; r0 += 64) {
    const int r = r0 + lane;
    const double v = lg[min(r, nrow - 1)];
    int64_t k;
    if (with_out && st.s2_out != nullptr && r < nrow && kept_row(p, first + r, k)) st.s2_out[k * st.n_chains + c] = v;
    const double dq = sqrt(v) - q.K;
    const int m = min(64, nrow - r0);
    for (int l = 0; l < m; ++l) q.add_dq(lane_bcast(v, l), lane_bcast(dq, l));
  }
  if (lane == 0) q.finish(st, c, first, last);
}

// The records of the window ending at row `last` from its logs, by one wave (k_stats): the rows in
// row order, kStatsRows loads in flight per column block.
constexpr int kStatsRows = 32;
__device__ void window_records(const DramState& st, const DramParams& p, int64_t c, int64_t last, int lane) {
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  const int64_t first = win_first(p, last);
  const int nrow = (int)(last - first + 1);
  const double* win = st.window + c * p.win * ld;
  ColAcc<1> a;
  a.setup(p, first);
  for (int j0 = 0; j0 < P; j0 += 64) {  // uniform
    const int j = j0 + lane;
    const int jj = j < P ? j : 0;
    a.zero();
    a.K[0] = a.kfirst ? 0.0 : (j < P ? st.smean[c * ld + j] : 0.0);
    for (int rb = 0; rb < nrow; rb += kStatsRows) {
      double x[kStatsRows];  // every load issued together (clamped rows: no branch between them)
#pragma unroll
      for (int u = 0; u < kStatsRows; ++u) x[u] = win[(int64_t)min(rb + u, nrow - 1) * ld + jj];
#pragma unroll
      for (int u = 0; u < kStatsRows; ++u) {
        if (rb + u >= nrow) break;  // uniform
        const int64_t row = first + rb + u;
        a.add(row, &x[u]);
        int64_t k;
        if (st.chain_out != nullptr && j < P && kept_row(p, row, k)) st.chain_out[(k * st.n_chains + c) * ld + j] = x[u];
      }
    }
    a.finish(st, p, c, last, P, j);
  }
  window_s2_records(st, p, c, last, lane, true);
}

// The batched engine's records (and a run's first or last window outside a chunk): one wave per
// chain, the window ending at row *st.step.
__global__ __launch_bounds__(kThreads) void k_stats(DramState st, DramParams p) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * (kThreads / 64) + w;
  if (c >= st.n_chains) return;
  window_records(st, p, c, *st.step, lane);
}

__device__ __forceinline__ uint64_t stamp() {
#if TCI_CHAIN_PROFILE || TCI_ADAPT_PROFILE
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
#else
  return 0;
#endif
}

// Which waves keep the chain records. Both are stage-1 waves: a stage-1 proposal is more often out
// of bounds (it skips ssfun), so these waves reach the barrier first and have slack before it.
//   kRecWave: the window-slot log of the decided rows (log_row; k_stats keeps their records);
//   kSigWave: the s2 of each decided row (log_s2) and the precisions 1/s2 the next decisions use.
constexpr int kRecWave = 0, kSigWave = 2;  // (six placements measured within 1 %: r02u_record_wave_placement)
// k_chain / k_walk loop heads: the lane index is re-laundered every round/step (launder_lane), so
// the 64-bit lane masks derived from it are recomputed (one compare each) instead of living in
// scalar pairs across the loop. Register allocation only (same bits): it removes k_walk's VGPR
// spill at RPL = 4 (config 5: 199.7 -> 191-193 us per step) and trims k_chain<2,1>'s SGPR spill.
__device__ __forceinline__ void launder_lane(int& lane) { asm volatile("" : "+v"(lane)); }

// Evaluations per wave and round of k_chain: EPW = 1 speculates 2 steps per round, EPW = 2 four
// (each wave evaluates its stage's proposals of two steps, one after the other). EPW = 2 decides
// 3.02 steps per round instead of 1.82 on the 299 TestData chains, but its rounds are ~1.75x as
// long and the 43 CUs that hold two chains become the long pole: k_chain 411 vs 260 us per 100
// steps (r03y). Only EPW = 1 is instantiated; the EPW = 2 instance was bitwise equal to the other
// engines (tests/test_dram_gpu.py green with it).
constexpr int kChainEPW = 1;


template <int RPL, int NSEG, int EPW>
__global__ __launch_bounds__(kThreads) void k_chain(DramState st, DramParams p, KParams kp, int64_t s_begin,
                                                    int64_t s_end, int with_records, double* nx_draws,
                                                    int64_t nx_begin, int64_t nx_end) {
  // Round structure (one workgroup barrier per round). At the start of a round the state after
  // row s-1 is known. The round speculates D = 2 EPW steps: proposal slot 2h + stage holds the
  // stage-1/2 proposal of step s + h, drawn around the SAME state, i.e. speculating that steps
  // s .. s + h - 1 do not move the chain (the common case: mcmcstat's DRAM accepts a minority of
  // steps). Wave w evaluates its stage (w & 1) of steps s + (w >> 1) + 2e, e < EPW. After the
  // barrier every wave takes the decisions of steps s, s + 1, .. from the exchanged values until
  // one moves the chain: up to D steps are decided per round, each exactly as the step-by-step
  // sampler (and the batched engine) decides it, bit for bit.
  //
  // After the barrier only the decisions run: one lane-parallel exp and the compares. Everything
  // that does not depend on the exchanged values happens before the barrier, on the stage-1
  // waves (kRecWave, kSigWave), one round late for the records:
  //   * the precisions the decisions use: 1/s2 of the current state (step s) and, for step s + h
  //     after unmoved steps s .. s + h - 1, 1/s2 with s2 = 1/(G_{s+h-1}*(2/ss)) -- known before
  //     the round;
  //   * the s2 of the rows the previous round decided (1/(G*(2/ss)) of the state after them)
  //     and the logs and window sums of those rows.
  constexpr int NJ = RPL + 1;  // vector entries per lane: P = 7 + N <= 64 RPL + 8 <= 64 NJ
  constexpr int EV = eval_lds_doubles<RPL>();
  constexpr int NW = kThreads / 64;
  constexpr int D = 2 * EPW;                // steps per round
  constexpr int NS = 2 * D;                 // proposal slots
  // candidate rows for the next round: row s + a1 + 1 + k for k < D + 2 (EPW - 1). EPW = 1: both (k = 0, 1);
  // EPW = 2: the rows of an advance by 1 or 4 (k = 0, 2, 3, 5) -- an advance by 2 or 3 loads its
  // missing row (k = 1 or 4) after the decisions: six prefetched rows exceeded the 256-register
  // budget of two chains per CU
  constexpr int NPF = EPW == 1 ? 2 : 4;
  constexpr int kPf[4] = {0, EPW == 1 ? 1 : 2, 3, 5};  // prefetched k (the first NPF)
  __shared__ __attribute__((aligned(16))) double evl[NW][EV];  // each evaluating wave's tables
  __shared__ double yl[2][NS][64 * NJ];                         // by round parity: every proposal
  __shared__ double xch[2][NS][4];                              // by round parity: ss, prior, in-bounds
  __shared__ double xip[2][D];                                  // by round parity: precisions of steps s + h
  const int64_t c = blockIdx.x;
  if (c >= st.n_chains) {  // the split draws' workgroups: the next chunk's units (nx_draws, rows nx_begin..nx_end)
    extern __shared__ __attribute__((aligned(16))) double dyn[];
    if (nx_draws != nullptr) draws_rng_units(st, p, nx_draws, nx_begin, nx_end, c - st.n_chains, gridDim.x - st.n_chains, dyn);
    return;
  }
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int lane = threadIdx.x & 63;  // re-laundered every round (launder_lane)
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  const int64_t DW = draw_stride(ld);
  // this chain's draws rows (row of step s at (s - s_begin) * DW) and window logs (slot r at r * ld):
  // 32-bit offsets from per-chain bases, no 64-bit multiplies in the loop -- tci_dram_run checks that
  // chunk * draw_stride(ld) and adaptint * ld fit in an int (the draws buffer's GiB cap bounds the
  // first for every chain count)
  const double* const dchain = st.draws + c * p.chunk * DW;
  double* const wlog = st.window + c * p.win * ld;
  double* const s2lg = st.s2log + c * p.win;
  const int DWi = (int)DW, ldi = (int)ld;
  const int stage = w & 1, a1 = w >> 1;                           // this wave's slots: steps s + a1 + 2e
  const double scale = stage ? 1.0 / p.drscale : 1.0;
  double th[NJ], lo[NJ], hi[NJ], mu[NJ], sg[NJ], thp[NJ];
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    const int j = lane + 64 * k;
    const bool in = j < P;
    th[k] = in ? st.theta[c * ld + j] : 0.0;
    thp[k] = th[k];
    lo[k] = in ? st.lower[c * ld + j] : 0.0;
    hi[k] = in ? st.upper[c * ld + j] : 0.0;
    mu[k] = in ? st.pmu[c * ld + j] : 0.0;
    sg[k] = in ? prior_prec(st.psig[c * ld + j]) : 0.0;  // the precision (prior_prec)
  }
  EvalIn<RPL> e;  // the chain's cell records stay in registers
  {
    load_cell<RPL, false>(kp, st.cell[c], lane, e);
  }
  double ss = st.ss[c], prior = st.prior[c];
  // sigma2 chain (kSigWave): s2 of the last decided row, or its Gamma variate Gl while that s2
  // (1/(Gl*(2/ss)), ss of the state after the row) is pending; s2f[i]: s2 of row s + i if the
  // round's steps s .. s + i do not move the chain
  double s2c = st.sigma2[c], Gl = 0.0, s2f[D - 1];
#pragma unroll
  for (int i = 0; i < D - 1; ++i) s2f[i] = 0.0;
  bool gpend = false;
  int32_t nacc = st.naccept[c], nrej = st.nrej_win[c];
  int64_t nev = st.nevals[c];
  int64_t prow = 0;  // rows prow .. prow + padv - 1 were decided by the previous round (logs pending);
  int padv = 0;      // all but the last did not move the chain (their state is thp)
  bool pmov = false;  // the last of them moved the chain
  // Loads one round ahead. The next round starts at step s + 1 .. s + D, so a round loads every
  // candidate at its START (this wave's offsets of rows s + a1 + 1 .. s + a1 + D + 2 (EPW - 1), and the scalar
  // draws of rows s + 1 .. s + 2D - 1) and the next round picks its rows: a whole round hides the
  // latency. The scalar draws are vector loads (lane j: row r0 + j / 4, slot j % 4) read by
  // readlane: scalar loads would also be waited for at the evaluation's first LDS wait.
  // Unconditional loads (indices clamped into the row: no exec-mask branches), zeros selected past P.
  auto load_u = [&](double* u, int64_t row) {
    const double* src = dchain + (int)(min(row, s_end) - s_begin) * DWi + stage * ldi;
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const double v = src[min(lane + 64 * k, P - 1)];
      u[k] = lane + 64 * k < P ? v : 0.0;
    }
  };
  auto load_sc = [&](int64_t r0) {  // lanes >= 4 (2D - 1) load a valid entry that is never read
    return dchain[(int)(min(r0 + (lane >> 2), s_end) - s_begin) * DWi + 2 * ldi + (lane & 3)];
  };
  double ucur[EPW][NJ], cand[NPF][NJ];
#pragma unroll
  for (int q = 0; q < EPW; ++q) load_u(ucur[q], s_begin + a1 + 2 * q);
  double dsc = load_sc(s_begin), dscn = 0.0;
  int sbase = 0;  // lane of step s's first scalar draw in dsc (4 (adv - 1) of the previous round)
  int par = 0;
  // the logs and window sums of the rows as they are decided ("Chain records"): kRecWave's column
  // sums, kSigWave's s2 sums (lane 0), continuing a window begun by an earlier chunk (or by
  // k_init_stats); slots are consecutive within a chunk (log_slot)
  const int64_t slot0 = log_slot(p, s_begin) - s_begin;  // slot of row r: slot0 + r
  ColAcc<NJ> ca;
  ca.setup(p, s_begin);
  S2Acc qa{0.0, 0.0, 0.0, 0.0};
  const bool cont = s_begin != ca.first;
  if (w == kRecWave) {
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const int j = lane + 64 * k;
      const bool in = j < P;
      ca.ws[k] = cont && in ? st.wsumv[c * ld + j] : 0.0;
      ca.S1[k] = cont && in ? st.wacc1[c * ld + j] : 0.0;
      ca.S2[k] = cont && in ? st.wacc2[c * ld + j] : 0.0;
      // a window continued from an earlier chunk whose row sf is already logged: K = that row
      ca.K[k] = !in ? 0.0 : !ca.kfirst ? st.smean[c * ld + j]
                                         : ca.sf < s_begin ? st.window[(c * p.win + log_slot(p, ca.sf)) * ld + j] : 0.0;
    }
  }
  if (w == kSigWave) {
    qa.sum = cont ? st.s2acc[3 * c + 0] : 0.0;
    qa.S1 = cont ? st.s2acc[3 * c + 1] : 0.0;
    qa.S2 = cont ? st.s2acc[3 * c + 2] : 0.0;
    qa.K = ca.first > 1 ? st.sq_mean[c] : sqrt(st.s2log[c * p.win]);
  }
  // thinned output rows: the next kept row >= s_begin and its index, advanced as rows are recorded
  // (no division per row); never matched when nothing is kept
  const bool keep_rows = (st.chain_out != nullptr || st.s2_out != nullptr) && p.thin > 0;
  int64_t kkeep = keep_rows ? (s_begin - 1 + p.thin - 1) / p.thin : 0;
  int64_t next_keep = keep_rows ? kkeep * p.thin + 1 : INT64_MAX;
  auto rec_row = [&](int64_t row, const double* x, bool f) {  // kRecWave; f: the row's step moved the chain
    double* wr = wlog + (int)(slot0 + row) * ldi;
    if (lane == 0) log_run(st, p, c, slot0 + row, f);
#pragma unroll
    for (int k = 0; k < NJ; ++k)
      if (lane + 64 * k < P) wr[lane + 64 * k] = x[k];
    ca.add(row, x);
    if (row == next_keep) {  // uniform
      if (st.chain_out != nullptr && kkeep < p.n_keep) {
#pragma unroll
        for (int q = 0; q < NJ; ++q)
          if (lane + 64 * q < P) st.chain_out[(kkeep * st.n_chains + c) * ld + lane + 64 * q] = x[q];
      }
      ++kkeep;
      next_keep += p.thin;
    }
  };
  auto rec_s2 = [&](int64_t row, double v) {  // kSigWave: the row bookkeeping in every lane, stores by lane 0
    if (lane == 0) s2lg[(int)(slot0 + row)] = v;
    if (lane == 0) qa.add(v);
    if (row == next_keep) {  // uniform
      if (lane == 0 && st.s2_out != nullptr && kkeep < p.n_keep) st.s2_out[kkeep * st.n_chains + c] = v;
      ++kkeep;
      next_keep += p.thin;
    }
  };
  auto flush_vec = [&]() {  // unrolled: a bounded store count (a runtime loop made the compiler
                            // wait for every store before the next round's loads were used)
    // the round's unmoved rows repeat the state before it; its last row moved the chain or not (pmov)
#pragma unroll
    for (int i = 0; i < D - 1; ++i)
      if (i + 1 < padv) rec_row(prow + i, thp, false);  // uniform
    if (padv >= 1) rec_row(prow + padv - 1, th, pmov);
  };
  auto flush_s2 = [&](double x0) {
#pragma unroll
    for (int i = 0; i < D - 1; ++i)
      if (i + 1 < padv) rec_s2(prow + i, s2f[i]);  // uniform
    if (padv >= 1) rec_s2(prow + padv - 1, x0);
  };
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t0 = stamp(), t1;
#define TCI_PHASE(k) \
  if (TCI_CHAIN_PROFILE) { t1 = stamp(); ph[k] += t1 - t0; t0 = t1; }
  for (int64_t s = s_begin; s <= s_end; par ^= 1) {
    launder_lane(lane);
    // ---- this wave's proposals, their bounds (wave vote) and evaluations
#pragma unroll
    for (int q = 0; q < EPW; ++q) {
      const int h = a1 + 2 * q;  // step s + h
      double y[NJ];
      uint64_t outm = 0;  // lanes with an entry outside its bounds: votes on the compare masks, no branches
#pragma unroll
      for (int k = 0; k < NJ; ++k) {
        y[k] = th[k] + scale * ucur[q][k];
        outm |= (wave_ballot(!(y[k] >= lo[k])) | wave_ballot(!(y[k] <= hi[k]))) & wave_ballot(lane + 64 * k < P);
      }
      const bool active = (stage == 0 || p.ntry >= 2) && s + h <= s_end;
      const bool inb = active && outm == 0;
      if (q == 0) {  // the next round's candidates (see load_u)
#pragma unroll
        for (int k = 0; k < NPF; ++k) load_u(cand[k], s + a1 + 1 + kPf[k]);
        dscn = load_sc(s + 1);
        // the record / s2 waves' work on the previous round's rows (it reads only the state at the
        // round's start) ahead of the evaluation, whose latencies it fills: k_chain 220.7 -> 216.4
        // us per chunk against after the evaluation (r04early)
        if (w == kSigWave) {
          // lanes 0 .. D-1: s2 of the last decided row (pending: 1/(Gl*(2/ss))), then after the steps
          // s .. s + i - 1 unmoved (1/(G_{s+i-1}*(2/ss))); their precisions are the decisions' of
          // steps s .. s + D - 1
          double gv = Gl;
#pragma unroll
          for (int i = 1; i < D; ++i) {
            const double Gi = lane_bcast(dsc, sbase + 4 * (i - 1) + D_G);
            gv = lane == i ? Gi : gv;
          }
          double x = 1.0 / (gv * (2.0 / ss));
          if (!p.updatesigma || (lane == 0 && !gpend)) x = s2c;
          const double ipv = 1.0 / x;
          if (lane < D) xip[par][lane] = ipv;
          const double x0 = lane_bcast(x, 0);
          flush_s2(x0);
          s2c = x0;
          gpend = false;
#pragma unroll
          for (int i = 0; i < D - 1; ++i) s2f[i] = lane_bcast(x, i + 1);  // the s2 of row s + i if unmoved
        }
        if (w == kRecWave) flush_vec();
        if (w == kRecWave) {
#pragma unroll
          for (int k = 0; k < NJ; ++k) thp[k] = th[k];  // the state before this round's rows
        }
      }
      double r = INFINITY, pr = 0.0;
      TCI_PHASE(0)
      if (inb) {
        double* yb = yl[par][2 * h + stage];
#pragma unroll
        for (int k = 0; k < NJ; ++k) yb[lane + 64 * k] = y[k];
        wave_sync();
        e.v = yb[0];
        e.tau = yb[1];
        e.ton = yb[2];
        e.b1 = yb[3];
        e.b2 = yb[4];
        e.A = yb[5];
        e.R = yb[6];
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
          const int g = RPL * lane + k;
          e.dr[k] = 7 + g < P ? yb[7 + g] : 0.0;
        }
        if (RPL <= 2) {  // the prior's wave sum rides on the evaluation's final scan (same bits)
          pr = prior_part<NJ>(y, mu, sg, P, lane);
          r = eval_wave<RPL, NSEG, MODE_SS>(kp, e, lane, evl[w], 0, nullptr, nullptr, 0, &pr);
          TCI_PHASE(1)
        } else {
          r = eval_wave<RPL, NSEG, MODE_SS>(kp, e, lane, evl[w], 0, nullptr, nullptr, 0);
          TCI_PHASE(1)
          pr = wave_prior_reg<NJ>(y, mu, sg, P, lane);
        }
      }
      if (lane == 0) {
        xch[par][2 * h + stage][0] = r;
        xch[par][2 * h + stage][1] = pr;
        xch[par][2 * h + stage][2] = inb ? 1.0 : 0.0;
      }
    }
    TCI_PHASE(2)
    __syncthreads();
    TCI_PHASE(3)
    // ---- decisions: step s, then (while the chain did not move) s + 1, .. s + D - 1 from the
    // speculation. The three exponentials each step can need -- a12, a32, l2 (dram_log_ratio) --
    // for every step are ONE lane-parallel exp (lanes 3h .. 3h + 2: step s + h), picked by readlane.
    const double (*X)[4] = xch[par];
    double av;
    {
      const int h = min(lane / 3, D - 1), k3 = lane - 3 * (lane / 3);  // lanes >= 3D compute junk
      const double* x1 = X[2 * h];
      const double* x2 = X[2 * h + 1];
      const double ssA = x1[0], ssB = x2[0];
      const double prA = x1[1], prB = x2[1];  // 0.0 for a candidate out of bounds (never evaluated)
      const double ipu = xip[par][h];
      // one expression, per-lane operands: a12 (k3 = 0), a32 (k3 = 1), l2 (k3 = 2)
      const double eA = k3 == 2 ? ssB : ssA, eB = k3 == 1 ? ssB : ss;
      const double eC = k3 == 2 ? prB : prA, eD = k3 == 1 ? prB : prior;
      const double ev = exp(dram_log_ratio(eA, eB, eC, eD, ipu));
      av = k3 == 2 ? ev : fmin(1.0, ev);
    }
    TCI_PHASE(4)
    int adv = 0;
    bool rmov = false;
#pragma unroll
    for (int hh = 0; hh < D; ++hh) {  // uniform
      if (hh >= 1 && s + hh > s_end) break;
      const double* x1 = X[2 * hh];
      const double* x2 = X[2 * hh + 1];
      const bool inb1 = x1[2] != 0.0, inb2 = x2[2] != 0.0;
      const double a12 = lane_bcast(av, 3 * hh), a32 = lane_bcast(av, 3 * hh + 1), l2 = lane_bcast(av, 3 * hh + 2);
      const double Q1 = lane_bcast(dsc, sbase + 4 * hh + D_Q1), U1 = lane_bcast(dsc, sbase + 4 * hh + D_U1);
      const double U2 = lane_bcast(dsc, sbase + 4 * hh + D_U2);
      bool acc = false, acc2 = false;
      if (inb1) {
        nev += 1;
        acc = U1 < a12;
      }
      if (!acc && inb2) {
        nev += 1;
        acc2 = dram_dr_accept(U2, a12, a32, l2, Q1);
      }
      const bool moved = acc || acc2;
      adv = hh + 1;
      if (moved) {
        const double* yb = yl[par][2 * hh + (acc ? 0 : 1)];
#pragma unroll
        for (int k = 0; k < NJ; ++k) th[k] = yb[lane + 64 * k];
        ss = acc ? x1[0] : x2[0];
        prior = acc ? x1[1] : x2[1];  // an accepted candidate was in bounds
        nacc += 1;
        rmov = true;
        break;  // step s + hh + 1 must be re-proposed around the new state
      }
      nrej += 1;
    }
    // the rows s .. s + adv - 1 are recorded next round (s2 of the last: 1/(G*(2/ss)), ss after it)
    prow = s;
    padv = adv;
    pmov = rmov;
    Gl = lane_bcast(dsc, sbase + 4 * (adv - 1) + D_G);
    gpend = p.updatesigma != 0;
    TCI_PHASE(6)
    // ---- advance by adv rows: the candidates loaded at the start of this round (row
    // s + adv + a1 + 2q is candidate adv + 2q - 1), or a load now
#pragma unroll
    for (int q = 0; q < EPW; ++q) {
      bool have = false;
#pragma unroll
      for (int i = 0; i < NPF; ++i) have = have || adv + 2 * q - 1 == kPf[i];
      if (have) {  // uniform
#pragma unroll
        for (int k = 0; k < NJ; ++k) {
          double v = cand[0][k];
#pragma unroll
          for (int i = 1; i < NPF; ++i) v = adv + 2 * q - 1 == kPf[i] ? cand[i][k] : v;
          ucur[q][k] = v;
        }
      } else {
        load_u(ucur[q], s + adv + a1 + 2 * q);
      }
    }
    dsc = dscn;
    sbase = 4 * (adv - 1);
    s += adv;
    TCI_PHASE(5)
    if (TCI_CHAIN_PROFILE) ph[5] += 1ull << 40;  // round count in the high bits
  }
#undef TCI_PHASE
#if TCI_CHAIN_PROFILE == 3  // every phase of every wave: slot 8 w + k
  if (lane == 0 && st.prof != nullptr)
    for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long*)&st.prof[8 * w + k], (unsigned long long)ph[k]);
#elif TCI_CHAIN_PROFILE == 2  // per wave: barrier wait (slot w) and eval + prior + exchange (slot 4 + w)
  if (lane == 0 && st.prof != nullptr) {
    atomicAdd((unsigned long long*)&st.prof[w], (unsigned long long)ph[3]);
    atomicAdd((unsigned long long*)&st.prof[4 + w], (unsigned long long)(ph[1] + ph[2]));
  }
#else
  if (TCI_CHAIN_PROFILE && w == 0 && lane == 0 && st.prof != nullptr)
    for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long*)&st.prof[k], (unsigned long long)ph[k]);
#endif
  // the last round's rows
  if (w == kRecWave) {
    flush_vec();
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const int j = lane + 64 * k;
      if (j < P) st.theta[c * ld + j] = th[k];
    }
    if (lane == 0) {
      st.ss[c] = ss;
      st.prior[c] = prior;
      st.naccept[c] = nacc;
      st.nrej_win[c] = nrej;
      st.nevals[c] = nev;
      if (c == 0) *st.step = s_end;  // the adaptation reads the row it follows
    }
    if (with_records) {  // the chunk ends a window (or the run): its records
      ca.finish(st, p, c, s_end, P, lane);
    } else {  // the window goes on in the next chunk
#pragma unroll
      for (int k = 0; k < NJ; ++k) {
        const int j = lane + 64 * k;
        if (j < P) {
          st.wsumv[c * ld + j] = ca.ws[k];
          st.wacc1[c * ld + j] = ca.S1[k];
          st.wacc2[c * ld + j] = ca.S2[k];
        }
      }
    }
  }
  if (w == kSigWave) {
    const double x0 = (p.updatesigma && gpend) ? 1.0 / (Gl * (2.0 / ss)) : s2c;
    flush_s2(x0);
    if (lane == 0) {
      st.sigma2[c] = x0;
      if (with_records) {
        qa.finish(st, c, ca.first, s_end);
      } else {
        st.s2acc[3 * c + 0] = qa.sum;
        st.s2acc[3 * c + 1] = qa.S1;
        st.s2acc[3 * c + 2] = qa.S2;
      }
    }
  }
}

// One wavefront per chain (the WALK engine: many chains, e.g. configs 4/5's 10,000): the same
// chunk of rows as k_chain, step by step, stage 2 evaluated only when stage 1 is rejected. No
// workgroup barriers; one chain per 64-thread workgroup (a CU holds 8 of them at the register
// budget, 2x the chains k_chain's 4-wave layout does). Every value is computed by the same expressions as
// k_chain (its step-s lanes) and the batched engine: identical chains (tests/test_dram_gpu.py).
// Register budget: two waves per SIMD (229 -> 188 us per config-4 step).
// One chain (wave) per workgroup: a 4-chain workgroup kept its 74 KB of LDS until its slowest chain
// ended (config 4: k_walk 2,189 -> 2,135 us per chunk, bitwise equal, profiles/r05/r05ic4_*).
constexpr int kWalkWaves = 1;
template <int RPL, int NSEG>
__global__ __launch_bounds__(64 * kWalkWaves) __attribute__((amdgpu_waves_per_eu(2))) void k_walk(DramState st, DramParams p, KParams kp, int64_t s_begin,
                                                                int64_t s_end, int with_records) {
  constexpr int NJ = RPL + 1;
  constexpr int EV = eval_lds_doubles<RPL>();
  constexpr int NW = kWalkWaves;
  __shared__ __attribute__((aligned(16))) double evl[NW][EV];  // each wave's {K,J} tables / rows
  __shared__ double yl[NW][64 * NJ];                            // each wave's proposal (theta broadcast)
  __shared__ double racc[NW][3][64 * NJ];  // each wave's window column sums ws, S1, S2 (ColAcc, in LDS)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int lane = threadIdx.x & 63;  // re-laundered every step (launder_lane)
  const int64_t c = (int64_t)blockIdx.x * NW + w;
  if (c >= st.n_chains) return;  // uniform per wave; no workgroup barriers below
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  const int64_t DW = draw_stride(ld);
  const double* drow = st.draws + (c * p.chunk - s_begin) * DW;  // row of step s: drow + s * DW
  const double inv_ds = 1.0 / p.drscale;
  // Bounds and prior vectors: held in registers for up to two segments per dye; re-read from
  // global memory at every evaluation for NSEG >= 3, whose larger evaluation spills at the
  // 2-waves/SIMD budget. (Round 3 re-read them for NSEG = 2 too, when its evaluation spilled 108 B
  // per lane; with round 4-5's shorter evaluation NSEG = 2 fits 256 VGPRs without a spill and
  // holding them took config 5's walk from 3,150 to 2,521 us per launch, bitwise equal, r05gb.)
  constexpr bool kGB = NSEG >= 3;
  double th[NJ], lo[NJ], hi[NJ], mu[NJ], sg[NJ];
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    const int j = lane + 64 * k;
    const bool in = j < P;
    th[k] = in ? st.theta[c * ld + j] : 0.0;
    if (!kGB) {
      lo[k] = in ? st.lower[c * ld + j] : 0.0;
      hi[k] = in ? st.upper[c * ld + j] : 0.0;
      mu[k] = in ? st.pmu[c * ld + j] : 0.0;
      sg[k] = in ? prior_prec(st.psig[c * ld + j]) : 0.0;  // the precision (prior_prec)
    }
  }
  EvalIn<RPL> e;  // the chain's cell records stay in registers
  {
    load_cell<RPL, false>(kp, st.cell[c], lane, e);
  }
  double ss = st.ss[c], prior = st.prior[c], s2 = st.sigma2[c];
  int32_t nacc = st.naccept[c], nrej = st.nrej_win[c];
  int64_t nev = st.nevals[c];
  double* yb = yl[w];
  const int64_t slot0 = log_slot(p, s_begin) - s_begin;  // log slot of row s: slot0 + s
  // the window's column sums as the rows are decided, k_chain's ColAcc arithmetic ("Chain
  // records"): the sums in this wave's LDS (registers are at the 2-waves/SIMD budget), their shift K
  // in registers, continuing a window begun by an earlier chunk (or by k_init_stats); the s2 sums
  // from the window's s2 log at its end (S2Acc over 100 values)
  ColAcc<NJ> ca;  // only first / sf / kfirst / K live in the loop
  ca.setup(p, s_begin);
  const bool cont = s_begin != ca.first;
  double* ra = racc[w][0];
  double* rb = racc[w][1];
  double* rc = racc[w][2];
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    const int j = lane + 64 * k;
    const bool in = j < P;
    ra[64 * k + lane] = cont && in ? st.wsumv[c * ld + j] : 0.0;
    rb[64 * k + lane] = cont && in ? st.wacc1[c * ld + j] : 0.0;
    rc[64 * k + lane] = cont && in ? st.wacc2[c * ld + j] : 0.0;
    ca.K[k] = !in ? 0.0 : !ca.kfirst ? st.smean[c * ld + j]
                                       : ca.sf < s_begin ? st.window[(c * p.win + log_slot(p, ca.sf)) * ld + j] : 0.0;
  }
  // ssfun and prior of the proposal th + scale * u (k_chain's per-wave evaluation); an in-bounds
  // proposal is left in yb (a move copies it from there)
  auto evaluate = [&](const double* u, double scale, double& r, double& pr) {
    double y[NJ];
    bool out = false;
    if constexpr (kGB) {
#pragma unroll
      for (int k = 0; k < NJ; ++k) {
        const int j = lane + 64 * k;
        const bool in = j < P;
        lo[k] = in ? st.lower[c * ld + j] : 0.0;
        hi[k] = in ? st.upper[c * ld + j] : 0.0;
        mu[k] = in ? st.pmu[c * ld + j] : 0.0;
        sg[k] = in ? prior_prec(st.psig[c * ld + j]) : 0.0;  // the precision (prior_prec)
      }
    }
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      y[k] = th[k] + scale * u[k];
      if (lane + 64 * k < P) out |= !(y[k] >= lo[k] && y[k] <= hi[k]);
    }
    r = INFINITY;
    pr = 0.0;
    if (wave_ballot(out) != 0) return false;
#pragma unroll
    for (int k = 0; k < NJ; ++k) yb[lane + 64 * k] = y[k];
    wave_sync();
    e.v = yb[0];
    e.tau = yb[1];
    e.ton = yb[2];
    e.b1 = yb[3];
    e.b2 = yb[4];
    e.A = yb[5];
    e.R = yb[6];
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      const int g = RPL * lane + q;
      e.dr[q] = 7 + g < P ? yb[7 + g] : 0.0;
    }
    r = eval_wave<RPL, NSEG, MODE_SS>(kp, e, lane, evl[w], 0, nullptr, nullptr, 0);
    pr = wave_prior_reg<NJ>(y, mu, sg, P, lane);
    return true;
  };
  // the row's proposal offsets of one stage (loaded when needed: registers, not prefetch, are short)
  auto load_u = [&](double* u, int64_t s, int stage) {
    const double* src = drow + s * DW + stage * ld;
#pragma unroll
    for (int k = 0; k < NJ; ++k) u[k] = lane + 64 * k < P ? src[lane + 64 * k] : 0.0;
  };
  // the records of row r (the chain state th, s2 after it): the window log, the window sums in LDS
  // and the thinned outputs
  auto record_row = [&](int64_t r, bool f) {  // f: the step moved the chain
    log_row<NJ>(st, p, c, slot0 + r, P, th, lane);
    if (lane == 0) {
      log_s2(st, p, c, slot0 + r, s2);
      log_run(st, p, c, slot0 + r, f);
    }
    int64_t kk;
    const bool keep = st.chain_out != nullptr && kept_row(p, r, kk);
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      if (ca.kfirst && r == ca.sf) ca.K[k] = th[k];
      const int i = 64 * k + lane;
      ra[i] = ra[i] + th[k];
      if (r >= ca.sf) {
        const double d = th[k] - ca.K[k];
        rb[i] = rb[i] + d;
        rc[i] = fma(d, d, rc[i]);
      }
      if (keep && lane + 64 * k < P) st.chain_out[(kk * st.n_chains + c) * ld + lane + 64 * k] = th[k];
    }
    if (st.s2_out != nullptr && lane == 0 && kept_row(p, r, kk)) st.s2_out[kk * st.n_chains + c] = s2;
  };
  // row decided by the previous step, recorded after this step's loads are issued (its latency
  // hides the records: config 4 2,230 -> 2,178 us per chunk against recording it at once, r04wearly)
  int64_t prow = s_begin - 1;
  bool pmv = false;  // the step of row prow moved the chain
  for (int64_t s = s_begin; s <= s_end; ++s) {
    launder_lane(lane);
    double u[NJ];
    load_u(u, s, 0);
    const double* sc = drow + s * DW + 2 * ld;
    const double q1 = sc[D_Q1], U1 = sc[D_U1], U2 = sc[D_U2], G = sc[D_G];
    if (prow >= s_begin) record_row(prow, pmv);
    double r1, pr1, r2 = INFINITY, pr2 = 0.0;
    const bool inb1 = evaluate(u, 1.0, r1, pr1);
    // a12 (k_chain lane 0): ssA = r1 (+Inf out of bounds), prA = pr1 (0 out of bounds)
    const double ip = 1.0 / s2;  // k_chain's xip
    const double a12 = fmin(1.0, exp(dram_log_ratio(r1, ss, pr1, prior, ip)));
    bool acc = false, acc2 = false;
    if (inb1) {
      nev += 1;
      acc = U1 < a12;
    }
    if (!acc && p.ntry >= 2) {
      load_u(u, s, 1);
      const bool inb2 = evaluate(u, inv_ds, r2, pr2);
      if (inb2) {
        nev += 1;
        // a32 (lane 1), l2 (lane 2) and the stage-2 test as k_chain computes them
        const double a32 = fmin(1.0, exp(dram_log_ratio(r1, r2, pr1, pr2, ip)));
        const double l2 = exp(dram_log_ratio(r2, ss, pr2, prior, ip));
        acc2 = dram_dr_accept(U2, a12, a32, l2, q1);
      }
    }
    const bool mv = acc || acc2;
    if (acc || acc2) {  // the accepted proposal is the last one evaluated: it is in yb
#pragma unroll
      for (int k = 0; k < NJ; ++k) th[k] = yb[lane + 64 * k];
      ss = acc ? r1 : r2;
      prior = acc ? pr1 : pr2;
      nacc += 1;
    } else {
      nrej += 1;
    }
    // sigma2 Gibbs update of this row (updatesigma = 1, :265): 1/sigma2 ~ Gamma(N/2, scale 2/ss)
    if (p.updatesigma) s2 = 1.0 / (G * (2.0 / ss));
    wave_sync();  // yb reads are done before the next evaluation rewrites it
    prow = s;  // recorded under the next step's loads
    pmv = mv;
  }
  if (prow >= s_begin) record_row(prow, pmv);
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    const int j = lane + 64 * k;
    if (j < P) st.theta[c * ld + j] = th[k];
  }
  if (lane == 0) {
    st.ss[c] = ss;
    st.prior[c] = prior;
    st.sigma2[c] = s2;
    st.naccept[c] = nacc;
    st.nrej_win[c] = nrej;
    st.nevals[c] = nev;
    if (c == 0) *st.step = s_end;  // the adaptation reads the row it follows
  }
  if (with_records) {  // the chunk ends a window (or the run): its records
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      ca.ws[k] = ra[64 * k + lane];
      ca.S1[k] = rb[64 * k + lane];
      ca.S2[k] = rc[64 * k + lane];
    }
    ca.finish(st, p, c, s_end, P, lane);
    __threadfence_block();  // lane 0's s2 logs before the other lanes read them
    window_s2_records(st, p, c, s_end, lane, false);  // the s2 sums from the window's log (100 values)
  } else {  // the window goes on in the next chunk
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const int j = lane + 64 * k;
      if (j < P) {
        st.wsumv[c * ld + j] = ra[64 * k + lane];
        st.wacc1[c * ld + j] = rb[64 * k + lane];
        st.wacc2[c * ld + j] = rc[64 * k + lane];
      }
    }
  }
}

template <int RPL, int NSEG>
int launch_chain_t(const DramState& st, const DramParams& p, const KParams& kp, int64_t s_begin, int64_t s_end,
                   int with_records, hipStream_t stream, LaunchTimer* timer, const ChainNext* nx) {
  const bool wide = p.walk != 0 && draws_walk_wide(st.ld);  // WALK: 64-row draws passes (k_draws<8, 2, 4, 2>)
  const size_t lds = (size_t)draws_lds_bytes(st.ld, wide ? kDrawMTWalk : kDrawMT);
  // 4-wave workgroups, 2 column tiles x 2 row tiles per wave and MFMA call (168 VGPRs: three
  // workgroups per CU, kDrawsWPE). Config 4 (WALK, P = 207): 72.7 ms per 1,000 steps with the 8-wave, 2-tile
  // form -> 53.6 (3 tiles: 58.0, 5: 56.4); TestData (FUSED): 105.3 -> 99.8 us per chunk against
  // 3 tiles (r03t4, r03u); the pipelined z*R loop (mfma_zr_pf) 97.6 -> 86.5 (r04g).
  auto kd = wide ? k_draws<8, 2, kDrawMTWalk, 2> : p.split ? k_draws<4, 2, kDrawMT, kDrawsWPE, true> : k_draws<4, 2>;
  const int nwd = wide ? 8 : 4;
  if (ensure_dyn_lds((const void*)kd, lds) != TCI_OK) return TCI_EHIP;
  const int npass = draws_passes(p.walk != 0);
  const int64_t per_wg = (int64_t)8 * (wide ? kDrawMTWalk : kDrawMT) * npass;  // <= the threads (scalar draws)
  const unsigned gy = (unsigned)((s_end - s_begin + per_wg) / per_wg);
  if (timer) timer->begin(stream);
  hipLaunchKernelGGL(kd, dim3((unsigned)st.n_chains, gy), dim3(64 * nwd), lds, stream, st, p, s_begin, s_end, npass);
  if (timer) {
    timer->end(0, stream);
    timer->begin(stream);
  }
  if (p.walk)
    hipLaunchKernelGGL((k_walk<RPL, NSEG>), dim3((unsigned)((st.n_chains + kWalkWaves - 1) / kWalkWaves)),
                       dim3(64 * kWalkWaves), 0, stream, st, p,
                       kp, s_begin, s_end, with_records);
  else {
    auto kc = k_chain<RPL, NSEG, (RPL <= 2 ? kChainEPW : 1)>;
    const bool rng = nx != nullptr && nx->draws != nullptr && nx->wgs > 0;
    const size_t clds = rng ? (size_t)draws_rng_lds_bytes(st.ld) : 0;
    if (rng && ensure_dyn_lds((const void*)kc, clds) != TCI_OK) return TCI_EHIP;
    hipLaunchKernelGGL(kc, dim3((unsigned)(st.n_chains + (rng ? nx->wgs : 0))), dim3(kThreads), clds, stream, st, p, kp,
                       s_begin, s_end, with_records, rng ? nx->draws : nullptr, rng ? nx->s_begin : 0,
                       rng ? nx->s_end : -1);
  }
  if (timer) timer->end(1, stream);
  return hipGetLastError() == hipSuccess ? TCI_OK : TCI_EHIP;
}

template <int RPL>
int launch_chain_r(const DramState& st, const DramParams& p, const KParams& kp, int64_t a, int64_t b, int rec,
                   hipStream_t s, LaunchTimer* timer, const ChainNext* dd) {
  switch (kp.n_seg) {
    case 1: return launch_chain_t<RPL, 1>(st, p, kp, a, b, rec, s, timer, dd);
    case 2: return launch_chain_t<RPL, 2>(st, p, kp, a, b, rec, s, timer, dd);
    case 3: return launch_chain_t<RPL, 3>(st, p, kp, a, b, rec, s, timer, dd);
    case 4: return launch_chain_t<RPL, 4>(st, p, kp, a, b, rec, s, timer, dd);
    default: return TCI_EINVAL;
  }
}



// ---- Adaptation on matrix cores, for P <= 16 * MAXT (every TestData cell; configs 4/5). One
// workgroup per chain. The upper triangle of cov + qcovadj I is held as 16 x 16 tiles in the MFMA
// accumulator layout, in REGISTERS: wave w owns every NW-th tile of the row-major tile order for the
// kernel. LDS holds only one batch of window rows (scatter) or, aliased onto it, two panel
// buffers (Cholesky): ~39 KB, so two chains' workgroups share a CU and all 299 TestData chains are
// resident at once (a 131 KB tile-in-LDS layout ran them in two rounds on 256 CUs).
//   covupd: the window's rows, centred on their batch mean and staged through LDS (the next batch
//     is loaded while the current one is multiplied), give the scatter S = Xc' Xc as
//     v_mfma_f64_16x16x4_f64 products into the owned tiles, merged with (cov, mean, wsum) by the
//     pairwise-update formula (mcmcstat's row-by-row recurrence in exact arithmetic);
//   Cholesky cov + qcovadj I = U'U, right-looking by 16-column panels: the owners copy panel row pk
//     to LDS (the diagonal tile factored on the way, in its owner's registers: chol16),
//     one wave per row tile solves the panel (solve16), the owners take their U
//     tiles back and every trailing tile takes the rank-16 update as 4 MFMAs on its owner's
//     registers. R = U * adascale, stored only when the
//     whole factorization succeeded (a singular matrix keeps the previous R, as mcmcstat).
// Instances: NW waves per workgroup (one chain), MAXT = max tiles per dimension, kAdOwn output tiles
// per wave (MAXT (MAXT + 1) / 2 <= NW kAdOwn): <8, 9, 6> for P <= 144 (two chains per CU at 128
// VGPRs), <8, 13, 12> for P <= 208 (configs 4/5: 200 points, P = 207; one chain per CU).
// The runs of equal rows among a window's nb rows (k_adapt_mfma, k_adapt_gt): a rejected step
// repeats the row before it, which adds the same outer product to the scatter again, so the
// scatter runs once per run, weighted by its length -- about 1 + 100 x the acceptance rate of the
// 100 rows; the same sum in exact arithmetic, rounded differently from row-by-row sums (and the
// same in every engine). A row starts a run when it is the window's first or its step moved the
// chain -- the engines record that flag as they log the row
// (DramState::runf; re-reading and comparing the window's rows here took 38k of the 261k cycles of
// a config-4 adaptation, profiles/r05/r05y_aprof4.json). Wave 0 lists the run starts in row order:
// rs[0..m) = start rows, rs[m] = nb.
__device__ int window_runs(const uint8_t* runf, int nb, int* rs, int* nrun) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w == 0) {  // run starts in row order (a ballot prefix per 64 rows)
    int m = 0;
    for (int r0 = 0; r0 < nb; r0 += 64) {
      const int r = r0 + lane;
      const bool f = r < nb && (r == 0 || runf[r] != 0);
      const uint64_t bal = wave_ballot(f);
      if (f) rs[m + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0))] = r;
      m += __builtin_popcountll(bal);
    }
    if (lane == 0) {
      rs[m] = nb;
      *nrun = m;
    }
  }
  __syncthreads();
  return *nrun;
}

constexpr int kAdRB = 16;  // window runs per LDS batch
__host__ __device__ inline int64_t adapt_mfma_lds_bytes(int64_t P, int64_t nb) {
  const int64_t NT = (P + 15) / 16, LX = 16 * NT;
  const int64_t shared = 2 * kAdRB * LX > 2 * NT * 256 ? 2 * kAdRB * LX : 2 * NT * 256;  // X, Xw | panel buffers
  return (shared + 2 * LX) * 8 + ((nb + 1) * 4 + 7) / 8 * 8;  // + the run starts
}

template <int NW, int MAXT, int kAdOwn, int WPE = (NW <= 8 ? 2 : NW / 4)>  // kAdOwn: output tiles per wave (a
                                                                        // multiple of the merge group); WPE: waves/SIMD
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(WPE))) void k_adapt_mfma(
    DramState st, DramParams p) {
  constexpr int kAdM = MAXT;
  constexpr bool kFresh = WPE >= 4;  // the 128-VGPR instance spills lane-derived indices otherwise
  constexpr int NTH = 64 * NW;
  static_assert(MAXT * (MAXT + 1) / 2 <= NW * kAdOwn, "owned tiles per wave");
  // merge groups: the old covariance values of kAdMG tiles in flight at once (the register budget)
  constexpr int kAdMG = kAdOwn <= 6 ? 3 : 6;
  static_assert(kAdOwn % kAdMG == 0, "owned tiles come in whole merge groups");
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ int fail, nrun;
  __shared__ double rdg[16];  // 1 / U[k][k] of the current diagonal tile
  const int t = threadIdx.x, lane = t & 63;  // lane-derived tile indices: lane_idx<kFresh>() where used
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t c = blockIdx.x;
  const int64_t step = *st.step;
  if (c >= st.n_chains || p.adaptint <= 0 || step % p.adaptint != 0) return;  // uniform exit
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  const int NT = (P + 15) >> 4, LX = 16 * NT;
  const int shared = max(2 * kAdRB * LX, 2 * NT * 256);
  double* X = dyn;                // scatter: a batch of centred window rows [kAdRB][LX]
  double* Xw = dyn + kAdRB * LX;  //   and the same rows times their run lengths
  double* Pb = dyn;               // Cholesky: panel buffers [2][NT][256] (aliases X)
  double* mb = dyn + shared;      // batch mean
  double* mo = mb + LX;           // old mean
  double* cvg = st.cov + c * dram_cov_stride(ld);
  double* mu = st.cmean + c * ld;
  const int nb = (TCI_ADAPT_ABLATE & 2) ? 0 : (int)p.adaptint;
  const double* win = st.window + c * p.win * ld;
  int* rs = (int*)(mo + LX);  // [nb + 1] the window's runs of equal rows: start rows, then nb
  uint64_t aph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a0 = stamp(), a1;
#define TCI_APHASE(k) \
  if (TCI_ADAPT_PROFILE) { a1 = stamp(); aph[k] += a1 - a0; a0 = a1; }
  // ---- batch mean from the window's column sums (kept by the engines as rows are recorded)
  for (int j = t; j < LX; j += NTH) {
    mb[j] = j < P ? st.wsumv[c * ld + j] / (double)p.adaptint : 0.0;
    mo[j] = j < P ? mu[j] : 0.0;
  }
  // owned tiles (ti <= tj): wave w's slots from kAdMap (tci_adapt_map.h: the diagonal tile a panel
  // factors goes to a wave with few trailing tiles in the panel before it). Slots past the wave's
  // last tile compute on tile (0, 0) and are discarded, so the code is straight-line and every array
  // index is a compile-time constant (the tiles stay in registers, no scratch memory).
  static_assert(NW == 8 && kAdOwn <= kAdMapSlots && MAXT <= kAdMapMaxT, "tile map shape");
  int sti[kAdOwn], stj[kAdOwn], stk[kAdOwn];  // tile row, column, row-major index (the cov layout)
  int nown = 0;                               // valid slots (a wave's tiles fill its first slots)
#pragma unroll
  for (int o = 0; o < kAdOwn; ++o) {
    int k = kAdMap[NT - 1][w][o], ti = 0;
    if (k >= 0) nown = o + 1;  // uniform
    if (k < 0) k = 0;
    stk[o] = k;
    while (k >= NT - ti) {  // uniform
      k -= NT - ti;
      ++ti;
    }
    sti[o] = ti;
    stj[o] = ti + k;
  }
  // ---- the window's runs of equal rows (window_runs)
  const int M = window_runs(st.runf + c * p.win, nb, rs, &nrun);
  TCI_APHASE(6)
  // ---- scatter of the centred runs on MFMA: sum over runs of len * d d' (A operand: the rows
  //      times their lengths, B: the rows); batch m0 + kAdRB is loaded while m0 is multiplied
  f64x4 acc[kAdOwn];
#pragma unroll
  for (int o = 0; o < kAdOwn; ++o) acc[o] = f64x4{0.0, 0.0, 0.0, 0.0};
  constexpr int kPer = (kAdRB * 16 * kAdM + NTH - 1) / NTH;
  double v[kPer];
  auto load_batch = [&](int m0) {
    const int n = min(kAdRB, M - m0);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = t + u * NTH, r = e / LX, j = e - r * LX;
      v[u] = (e < kAdRB * LX && r < n && j < P) ? win[(int64_t)rs[m0 + r] * ld + j] : 0.0;
    }
  };
  if (M > 0) load_batch(0);
  for (int m0 = 0; m0 < M; m0 += kAdRB) {
    const int n = min(kAdRB, M - m0);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = t + u * NTH, r = e / LX, j = e - r * LX;
      if (e < kAdRB * LX) {
        const double d = (r < n && j < P) ? v[u] - mb[j] : 0.0;
        X[e] = d;
        Xw[e] = r < n ? (double)(rs[m0 + r + 1] - rs[m0 + r]) * d : 0.0;
      }
    }
    __syncthreads();
    if (m0 + kAdRB < M) load_batch(m0 + kAdRB);
    const int lnx = lane_idx<kFresh>();
    for (int k0 = 0; k0 < n; k0 += 4) {
      const int ro = (k0 + (lnx >> 4)) * LX + (lnx & 15);
      double xa[kAdOwn], xb[kAdOwn];
#pragma unroll
      for (int o = 0; o < kAdOwn; ++o) {
        xa[o] = Xw[ro + 16 * sti[o]];
        xb[o] = X[ro + 16 * stj[o]];
      }
#pragma unroll
      for (int o = 0; o < kAdOwn; ++o) acc[o] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[o], xb[o], acc[o], 0, 0, 0);
    }
    __syncthreads();
  }
  TCI_APHASE(1)
  // ---- merge (cov, mean, wsum) with the batch: n = na + nb, d = m_batch - m_old; the owned tiles
  //      become the matrix to factor: cov + qcovadj I (identity in the padding)
  const double na = st.wsum[c], nn = na + (double)p.adaptint;
  const double fcross = na * (double)p.adaptint / nn;
  // cov in the owned-tile layout: tile k (row-major upper-tile order; wave w's slot o is tile
  // stk[o]) at cvg + 256 k, accumulator entry q of lane l at 64 q + l -- four 512-byte reads per
  // tile, and a diagonal tile keeps both triangles (the scatter, the update and hence the stored
  // values are symmetric bit for bit: the products and sums of (i, j) and (j, i) are the same)
  const double rn1 = 1.0 / (nn - 1.0);
#pragma unroll
  for (int o0 = 0; o0 < kAdOwn; o0 += kAdMG) {
    if (o0 >= nown) break;  // uniform
    const int ln = lane_idx<kFresh>(), row = ln & 15, kq = ln >> 4;
    double old[kAdMG][4];
#pragma unroll
    for (int u = 0; u < kAdMG; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int o = o0 + u;
        old[u][q] = (o < nown && na > 0.0) ? cvg[256 * stk[o] + 64 * q + ln] : 0.0;
      }
#pragma unroll
    for (int u = 0; u < kAdMG; ++u) {
      const int o = o0 + u;
      if (o >= nown) continue;  // uniform
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 16 * sti[o] + kq + 4 * q, j = 16 * stj[o] + row;
        double a, cv = 0.0;
        if (i < P && j < P) {
          if (nn <= 1.0) {
            cv = 0.0;  // a single row so far: covariance 0 (the recurrence's first row)
          } else if (na == 0.0) {
            cv = acc[o][q] * rn1;
          } else {
            const double di = mb[i] - mo[i], dj = mb[j] - mo[j];
            cv = (old[u][q] * (na - 1.0) + acc[o][q] + di * dj * fcross) * rn1;
          }
          a = cv + (i == j ? p.qcovadj : 0.0);
        } else {
          a = i == j ? 1.0 : 0.0;
        }
        cvg[256 * stk[o] + 64 * q + ln] = cv;
        acc[o][q] = a;
      }
    }
  }
  __syncthreads();  // mb / mo reads
  for (int j = t; j < P; j += NTH)
    mu[j] = na == 0.0 ? mb[j] : mo[j] + (mb[j] - mo[j]) * ((double)p.adaptint / nn);
  if (t == 0) {
    st.wsum[c] = nn;
    fail = 0;
  }
  if (step < p.burnintime) {
    // burn-in: no covariance adaptation, only scaling by the window's rejection rate
    const double rate = (double)st.nrej_win[c] / (double)p.adaptint;
    double s = 1.0;
    if (rate > 0.95) s = 1.0 / p.burnin_scale;
    else if (rate < 0.05) s = p.burnin_scale;
    if (s != 1.0) scale_R(st, c, P, s, t, NTH);
    __syncthreads();
    if (t == 0) st.nrej_win[c] = 0;
    return;
  }
  __syncthreads();
  TCI_APHASE(2)
  // ---- blocked Cholesky U'U of the owned tiles; panel row pk goes through LDS buffer pk & 1.
  // Look-ahead: the trailing update of panel pk ends with row pk + 1 -- the owners store its tiles
  // to the next buffer and the owner of the diagonal tile factors it right away, while the other
  // waves still apply their updates (the one-wave factorization no longer waits for them).
  const bool chol = !(TCI_ADAPT_ABLATE & 1);
  // row pr's tiles to LDS buffer pr & 1; the diagonal one (slot od) factored by its owner
  auto panel_row = [&](int pr) {
    double* Bn = Pb + (pr & 1) * NT * 256;
    const int ln = lane_idx<kFresh>(), row = ln & 15, kq = ln >> 4;
    int od = -1;
#pragma unroll
    for (int o = 0; o < kAdOwn; ++o) {
      if (o >= nown || sti[o] != pr) continue;  // uniform
      if (stj[o] == pr) {
        od = o;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) Bn[256 * stj[o] + (kq + 4 * q) * 16 + row] = acc[o][q];
      }
    }
    if (od >= 0) {  // uniform
      double dt[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double v = acc[0][q];
#pragma unroll
        for (int o = 1; o < kAdOwn; ++o) v = od == o ? acc[o][q] : v;
        dt[q] = v;
      }
      bool bad = false;
      chol16<kFresh>(dt, rdg, bad);
#pragma unroll
      for (int q = 0; q < 4; ++q) Bn[256 * pr + (kq + 4 * q) * 16 + row] = dt[q];
      if (bad && lane == 0) fail = 1;
    }
  };
  bool ok = true;
  if (chol) panel_row(0);
  __syncthreads();
  TCI_APHASE(3)
  for (int pk = 0; pk < (chol ? NT : 0); ++pk) {
    if (fail) {  // uniform (read after a barrier)
      ok = false;
      break;
    }
    double* B = Pb + (pk & 1) * NT * 256;  // tile (pk, tj) at B + 256 tj
    const double* D = B + 256 * pk;
    // (2) the panel's row tiles (pk, tj > pk): U_pk' X = A -> X, one tile per wave (solve16)
    for (int tj = pk + 1 + w; tj < NT; tj += NW) {  // uniform
      const int ln = lane_idx<kFresh>(), row = ln & 15, kq = ln >> 4;
      double* A = B + 256 * tj;
      double x[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = A[(kq + 4 * q) * 16 + row];
      solve16<kFresh>(x, D, rdg);
#pragma unroll
      for (int q = 0; q < 4; ++q) A[(kq + 4 * q) * 16 + row] = x[q];
    }
    __syncthreads();
    TCI_APHASE(5)
    // (3) the owners take row pk of U back; trailing tiles (ti, tj), pk < ti <= tj: A -= X_ti' X_tj;
    //     then row pk + 1 to the other buffer, its diagonal tile factored (look-ahead)
    const int ln3 = lane_idx<kFresh>(), row = ln3 & 15, kq = ln3 >> 4;
#pragma unroll
    for (int o = 0; o < kAdOwn; ++o) {
      if (o >= nown) continue;  // uniform
      if (sti[o] == pk) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[o][q] = B[256 * stj[o] + (kq + 4 * q) * 16 + row];
      } else if (sti[o] > pk) {
        const double* Xi = B + 256 * sti[o];
        const double* Xj = B + 256 * stj[o];
#pragma unroll
        for (int k4 = 0; k4 < 16; k4 += 4)
          acc[o] = __builtin_amdgcn_mfma_f64_16x16x4f64(-Xi[(k4 + kq) * 16 + row], Xj[(k4 + kq) * 16 + row], acc[o], 0,
                                                        0, 0);
      }
    }
    if (pk + 1 < NT) panel_row(pk + 1);
    __syncthreads();
    TCI_APHASE(0)
  }
  if (ok && !(TCI_ADAPT_ABLATE & 1)) {  // singular: keep the previous R (mcmcstat: "cmat singular, not adapting")
    const double sc = p.adascale > 0.0 ? p.adascale : 2.4 / sqrt((double)P);
    const int ln = lane_idx<kFresh>(), row = ln & 15, kq = ln >> 4;
#pragma unroll
    for (int o = 0; o < kAdOwn; ++o) {
      if (o >= nown) continue;  // uniform
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 16 * sti[o] + kq + 4 * q, j = 16 * stj[o] + row;
        if (i < P && j < P && j >= i) store_R(st, c, P, i, j, acc[o][q] * sc);
      }
    }
  }
  __syncthreads();
  TCI_APHASE(4)
#undef TCI_APHASE
  if (TCI_ADAPT_PROFILE && t == 0 && st.prof != nullptr)
    for (int q = 0; q < 8; ++q) atomicAdd((unsigned long long*)&st.prof[q], (unsigned long long)aph[q]);
  if (t == 0) st.nrej_win[c] = 0;
}

// ---- Adaptation for P > 208 (past k_adapt_mfma's register-resident tiles): the same covupd merge
// and right-looking blocked Cholesky by 16 x 16 tiles on the matrix cores, with the tiles in global
// memory -- st.work as an NT x NT grid of 16 x 16 tiles per chain (tile (ti, tj) at (ti NT + tj) 256,
// element (r, col) at r 16 + col), L2-resident while the chain's workgroup works on it. One
// workgroup of kGtWaves waves per chain:
//   covupd: passes of kGtTiles tiles per wave; each pass streams the window's centred rows through
//     LDS in batches of rb rows (as many as fit 96 KB, a multiple of 4) and accumulates the owned
//     tiles' scatter with v_mfma_f64_16x16x4_f64, then merges them into (cov, mean, wsum) with
//     k_adapt_mfma's formula and writes cov + qcovadj I to the tile grid;
//   Cholesky: per panel pk, wave 0 factors the diagonal tile in registers (chol16), one wave
//     per row tile solves the panel (solve16), every wave takes trailing tiles (pk < ti <= tj) round-robin
//     and applies the rank-16 update as 4 MFMAs. R = U * adascale, stored only when every pivot
//     was positive (a singular matrix keeps the previous R, as mcmcstat).
// The tile arithmetic is k_adapt_mfma's, so both kernels give the same R up to the order of the
// scatter's k-steps (rows in batches here).
constexpr int kGtWaves = 8, kGtTiles = 8;  // waves per chain; scatter tiles per wave and pass
constexpr int kGtBatch = 2;   // trailing / R-store tiles whose loads are issued together
constexpr int kGtPer = 8;     // window loads in flight per thread
constexpr int kGtPanels = 3;  // Cholesky panels per trailing pass (1 .. 4; 4 spill at the 128-VGPR budget)
__host__ __device__ inline int64_t gt_lt(int64_t ld) { return (ld + 15) / 16 * 16; }  // tile-grid side
__host__ __device__ inline int gt_rows(int64_t P) {  // window rows per LDS batch
  const int64_t LX = (P + 15) / 16 * 16;
  const int64_t rb = (96 * 1024 / 8 - 2 * LX) / LX;
  return (int)std::min<int64_t>(16, std::max<int64_t>(4, rb & ~(int64_t)3));
}
__host__ __device__ inline int64_t adapt_gt_lds_bytes(int64_t P, int64_t nb) {
  const int64_t LX = (P + 15) / 16 * 16;
  return ((int64_t)gt_rows(P) * LX + 2 * LX) * 8 + ((nb + 1) * 4 + 7) / 8 * 8;  // + the window's run starts
}
// tile k of the row-major upper triangle of an n x n tile grid starting at tile row r0 -> (ti, tj)
__device__ __forceinline__ void tri_tile(int k, int n, int r0, int& ti, int& tj) {
  int i = 0;
  while (k >= n - i) {  // uniform
    k -= n - i;
    ++i;
  }
  ti = r0 + i;
  tj = r0 + i + k;
}

__global__ __launch_bounds__(64 * kGtWaves) __attribute__((amdgpu_waves_per_eu(4))) void k_adapt_gt(DramState st,
                                                                                                    DramParams p) {
  constexpr int NW = kGtWaves, NTH = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ int fail, nrun;
  __shared__ double rdg[16];
  __shared__ double Dt[256];  // U of the current panel's diagonal tile
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int row = lane & 15, kq = lane >> 4;
  const int64_t c = blockIdx.x;
  const int64_t step = *st.step;
  if (c >= st.n_chains || p.adaptint <= 0 || step % p.adaptint != 0) return;  // uniform exit
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  const int NT = (P + 15) >> 4, LX = 16 * NT, T = NT * (NT + 1) / 2;
  const int rb = gt_rows(P);
  double* X = dyn;           // a batch of centred window rows [rb][LX]
  double* mb = X + rb * LX;  // batch mean
  double* mo = mb + LX;      // old mean
  double* cvg = st.cov + c * dram_cov_stride(ld);
  double* mu = st.cmean + c * ld;
  const int64_t LT = gt_lt(ld);
  double* Wt = st.work + c * LT * LT;
  auto tile = [&](int ti, int tj) { return Wt + ((int64_t)ti * NT + tj) * 256; };
  const int nb = (int)p.adaptint;
  const double* win = st.window + c * p.win * ld;
  int* rs = (int*)(mo + LX);  // [nb + 1] the window's runs: start rows, then nb
  // TCI_ADAPT_PROFILE: thread 0's s_memtime cycles per phase: scatter, merge, diagonal tiles,
  // panel solves, trailing updates, R store
  uint64_t aph[6] = {0, 0, 0, 0, 0, 0}, a0 = stamp(), a1;
#define TCI_GPHASE(k) \
  if (TCI_ADAPT_PROFILE) { a1 = stamp(); aph[k] += a1 - a0; a0 = a1; }
  for (int j = t; j < LX; j += NTH) {
    mb[j] = j < P ? st.wsumv[c * ld + j] / (double)p.adaptint : 0.0;
    mo[j] = j < P ? mu[j] : 0.0;
  }
  const double na = st.wsum[c], nn = na + (double)p.adaptint;
  const double fcross = na * (double)p.adaptint / nn;
  const double rn1 = 1.0 / (nn - 1.0);
  const int M = window_runs(st.runf + c * p.win, nb, rs, &nrun);
  // ---- covupd: scatter of the centred window runs (each row once, times its run length) + merge,
  //      kGtTiles tiles per wave and pass
  for (int base = 0; base < T; base += NW * kGtTiles) {
    int ti[kGtTiles], tj[kGtTiles];
    bool val[kGtTiles];
#pragma unroll
    for (int g = 0; g < kGtTiles; ++g) {
      const int k = base + w * kGtTiles + g;
      val[g] = k < T;
      tri_tile(val[g] ? k : 0, NT, 0, ti[g], tj[g]);
    }
    f64x4 acc[kGtTiles];
#pragma unroll
    for (int g = 0; g < kGtTiles; ++g) acc[g] = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int r0 = 0; r0 < M; r0 += rb) {
      const int n = min(rb, M - r0);
      __syncthreads();  // the previous batch is consumed (and mb is written, first time)
      // the batch's window entries, kGtPer loads in flight per thread before their LDS stores (a
      // plain strided loop waited for each load in turn)
      for (int e0 = t; e0 < rb * LX; e0 += kGtPer * NTH) {
        double v[kGtPer];
#pragma unroll
        for (int u = 0; u < kGtPer; ++u) {
          const int e = e0 + u * NTH, r = e / LX, j = e - r * LX;
          v[u] = (e < rb * LX && r < n && j < P) ? win[(int64_t)rs[r0 + r] * ld + j] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kGtPer; ++u) {
          const int e = e0 + u * NTH, r = e / LX, j = e - r * LX;
          if (e < rb * LX) X[e] = (r < n && j < P) ? v[u] - mb[j] : 0.0;
        }
      }
      __syncthreads();
      for (int k0 = 0; k0 < n; k0 += 4) {
        const double* xr = X + (k0 + kq) * LX + row;
        const int kr = k0 + kq;  // this lane's run: its length weights the A operand (rows past n are 0)
        const double len = kr < n ? (double)(rs[r0 + kr + 1] - rs[r0 + kr]) : 0.0;
#pragma unroll
        for (int g = 0; g < kGtTiles; ++g)
          if (val[g])
            acc[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(len * xr[16 * ti[g]], xr[16 * tj[g]], acc[g], 0, 0, 0);
      }
    }
    TCI_GPHASE(0)
#pragma unroll
    for (int g = 0; g < kGtTiles; ++g) {
      // every old value of the tile before any write (a diagonal tile reads the mirrors of its own
      // elements)
      double old[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 16 * ti[g] + kq + 4 * q, j = 16 * tj[g] + row;
        old[q] = (val[g] && i < P && j < P && na > 0.0) ? cvg[i <= j ? (int64_t)i * ld + j : (int64_t)j * ld + i] : 0.0;
      }
      if (!val[g]) continue;  // uniform
      double* A = tile(ti[g], tj[g]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 16 * ti[g] + kq + 4 * q, j = 16 * tj[g] + row;
        double a;
        if (i < P && j < P) {
          double cv;
          if (nn <= 1.0) {
            cv = 0.0;  // a single row so far: covariance 0 (the recurrence's first row)
          } else if (na == 0.0) {
            cv = acc[g][q] * rn1;
          } else {
            const double di = mb[i] - mo[i], dj = mb[j] - mo[j];
            cv = (old[q] * (na - 1.0) + acc[g][q] + di * dj * fcross) * rn1;
          }
          if (i <= j) cvg[(int64_t)i * ld + j] = cv;
          a = cv + (i == j ? p.qcovadj : 0.0);
        } else {
          a = i == j ? 1.0 : 0.0;
        }
        A[(kq + 4 * q) * 16 + row] = a;
      }
    }
  }
  TCI_GPHASE(1)
  __syncthreads();  // mb / mo reads, tile writes
  for (int j = t; j < P; j += NTH) mu[j] = na == 0.0 ? mb[j] : mo[j] + (mb[j] - mo[j]) * ((double)p.adaptint / nn);
  if (t == 0) {
    st.wsum[c] = nn;
    fail = 0;
  }
  if (step < p.burnintime) {
    // burn-in: no covariance adaptation, only scaling by the window's rejection rate
    const double rate = (double)st.nrej_win[c] / (double)p.adaptint;
    double s = 1.0;
    if (rate > 0.95) s = 1.0 / p.burnin_scale;
    else if (rate < 0.05) s = p.burnin_scale;
    if (s != 1.0) scale_R(st, c, P, s, t, NTH);
    __syncthreads();
    if (t == 0) st.nrej_win[c] = 0;
    return;
  }
  __syncthreads();
  // ---- blocked Cholesky U'U of the tile grid, kGtPanels (3) panels per trailing pass: panel pk is
  //      factored, row pk + 1 takes its update, panel pk + 1 is factored, ..., and every tile below
  //      takes all the group's rank-16 updates in one read-modify-write (4 MFMAs per panel, in panel
  //      order: the same bits as one pass per panel, 1/kGtPanels of the trailing tile traffic)
  // (1) + (2): the diagonal tile of panel pk in wave 0's registers, then the panel's row tiles
  //     (pk, tj > pk): U_pk' X = A -> X, one column per lane; false if a pivot failed
  auto factor_panel = [&](int pk) -> bool {
    if (w == 0) {
      double* A = tile(pk, pk);
      double dt[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) dt[q] = A[(kq + 4 * q) * 16 + row];
      bool bad = false;
      chol16(dt, rdg, bad);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        A[(kq + 4 * q) * 16 + row] = dt[q];
        Dt[(kq + 4 * q) * 16 + row] = dt[q];
      }
      if (bad && lane == 0) fail = 1;
    }
    __syncthreads();
    TCI_GPHASE(2)
    if (fail) return false;
    for (int tj = pk + 1 + w; tj < NT; tj += NW) {  // one tile per wave (solve16)
      double* A = tile(pk, tj);
      double x[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = A[(kq + 4 * q) * 16 + row];
      solve16(x, Dt, rdg);
#pragma unroll
      for (int q = 0; q < 4; ++q) A[(kq + 4 * q) * 16 + row] = x[q];
    }
    __syncthreads();
    TCI_GPHASE(3)
    return true;
  };
  // (3) trailing tiles (ti, tj), r0 <= ti <= tj (ti < r1), A -= X_ti' X_tj by panels pa .. pa + NP - 1,
  //     round-robin over waves, kGtBatch tiles at a time: every load of the batch is issued before
  //     the first store (one memory round trip per batch, not per tile: the stores may alias later
  //     loads)
  auto trail = [&](auto np_c, int pa, int r0, int r1) {
    constexpr int NP = decltype(np_c)::value;
    constexpr int BT = NP <= 2 ? kGtBatch : 1;  // tiles per batch (register budget)
    const int m = NT - r0, Ttr = (r1 - r0) * (2 * m - (r1 - r0) + 1) / 2;  // rows r0 .. r1 - 1 of the triangle
    for (int k0 = w; k0 < Ttr; k0 += NW * BT) {
      double* Ap[BT];
      f64x4 acc[BT];
      double xi[BT][NP][4], xj[BT][NP][4];
#pragma unroll
      for (int g = 0; g < BT; ++g) {
        const int k = k0 + g * NW;
        if (k >= Ttr) break;  // uniform
        int ti, tj;
        tri_tile(k, m, r0, ti, tj);
        Ap[g] = tile(ti, tj);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[g][q] = Ap[g][(kq + 4 * q) * 16 + row];
#pragma unroll
        for (int h = 0; h < NP; ++h) {
          const double* Xi = tile(pa + h, ti);
          const double* Xj = tile(pa + h, tj);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            xi[g][h][q] = Xi[(4 * q + kq) * 16 + row];
            xj[g][h][q] = Xj[(4 * q + kq) * 16 + row];
          }
        }
      }
#pragma unroll
      for (int g = 0; g < BT; ++g) {
        if (k0 + g * NW >= Ttr) break;
#pragma unroll
        for (int h = 0; h < NP; ++h)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(-xi[g][h][q], xj[g][h][q], acc[g], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) Ap[g][(kq + 4 * q) * 16 + row] = acc[g][q];
      }
    }
    __syncthreads();
    TCI_GPHASE(4)
  };
  auto trail_n = [&](int np, int pa, int r0, int r1) {  // np panels pa .. pa + np - 1
    if (np <= 0 || r0 >= r1) return;
    const auto go = [&](auto np_c) {
      trail(np_c, pa, r0, r1);
    };
    switch (np) {
      case 1: go(std::integral_constant<int, 1>{}); break;
      case 2: go(std::integral_constant<int, 2>{}); break;
      case 3: go(std::integral_constant<int, 3>{}); break;
      default: go(std::integral_constant<int, 4>{}); break;
    }
  };
  static_assert(kGtPanels >= 1 && kGtPanels <= 4, "panels per trailing pass (4 spills at the 128-VGPR budget)");
  bool ok = true;
  for (int pk = 0; pk < NT && ok; pk += kGtPanels) {
    const int np = min(kGtPanels, NT - pk);
    for (int j = 0; j < np && ok; ++j) {
      trail_n(j, pk, pk + j, pk + j + 1);  // row pk + j by panels pk .. pk + j - 1
      ok = factor_panel(pk + j);
    }
    if (ok) trail_n(np, pk, pk + np, NT);  // the rows below by all np panels
  }
  if (ok) {  // singular: keep the previous R (mcmcstat: "cmat singular, not adapting")
    const double sc = p.adascale > 0.0 ? p.adascale : 2.4 / sqrt((double)P);
    for (int k0 = w; k0 < T; k0 += NW * kGtBatch) {  // batches of loads, as in (3)
      double a[kGtBatch][4];
      int tis[kGtBatch], tjs[kGtBatch];
#pragma unroll
      for (int g = 0; g < kGtBatch; ++g) {
        const int k = k0 + g * NW;
        if (k >= T) break;  // uniform
        tri_tile(k, NT, 0, tis[g], tjs[g]);
        const double* A = tile(tis[g], tjs[g]);
#pragma unroll
        for (int q = 0; q < 4; ++q) a[g][q] = A[(kq + 4 * q) * 16 + row];
      }
#pragma unroll
      for (int g = 0; g < kGtBatch; ++g) {
        if (k0 + g * NW >= T) break;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = 16 * tis[g] + kq + 4 * q, j = 16 * tjs[g] + row;
          if (i < P && j < P && j >= i) store_R(st, c, P, i, j, a[g][q] * sc);
        }
      }
    }
  }
  __syncthreads();
  TCI_GPHASE(5)
#undef TCI_GPHASE
  if (TCI_ADAPT_PROFILE && t == 0 && st.prof != nullptr)
    for (int q = 0; q < 6; ++q) atomicAdd((unsigned long long*)&st.prof[q], (unsigned long long)aph[q]);
  if (t == 0) st.nrej_win[c] = 0;
}

inline int finish() { return hipGetLastError() == hipSuccess ? TCI_OK : TCI_EHIP; }
inline dim3 chain_grid(int64_t n) { return dim3((unsigned)n); }

int launch_stage(void (*k)(DramState, DramParams), const DramState& st, const DramParams& p, void* stream) {
  const size_t lds = (size_t)stage_lds_bytes(st.ld);
  if (ensure_dyn_lds((const void*)k, lds) != TCI_OK) return TCI_EHIP;
  hipLaunchKernelGGL(k, chain_grid(st.n_chains), dim3(kThreads), lds, (hipStream_t)stream, st, p);
  return finish();
}

template <int NW, int MAXT, int OWN, int WPE = (NW <= 8 ? 2 : NW / 4)>
int launch_adapt_mfma(const DramState& st, const DramParams& p, void* stream) {
  const size_t bytes = (size_t)adapt_mfma_lds_bytes(p.pmax, p.adaptint);
  auto k = k_adapt_mfma<NW, MAXT, OWN, WPE>;
  if (ensure_dyn_lds((const void*)k, bytes) != TCI_OK) return TCI_EHIP;
  hipLaunchKernelGGL(k, chain_grid(st.n_chains), dim3(64 * NW), bytes, (hipStream_t)stream, st, p);
  return finish();
}

}  // namespace

int dram_launch_init(const DramState& st, const double* qcov_diag, const double* sigma2_0, void* stream) {
  hipLaunchKernelGGL(k_init, chain_grid(st.n_chains), dim3(kThreads), 0, (hipStream_t)stream, st, qcov_diag, sigma2_0);
  return finish();
}
int dram_launch_init_stats(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_init_stats, chain_grid(st.n_chains), dim3(kThreads), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_propose1(const DramState& st, const DramParams& p, void* stream) {
  return launch_stage(k_propose1, st, p, stream);
}
int dram_launch_accept1(const DramState& st, const DramParams& p, void* stream) {
  return launch_stage(k_accept1, st, p, stream);
}
int dram_launch_accept2(const DramState& st, const DramParams& p, void* stream) {
  return launch_stage(k_accept2, st, p, stream);
}
int dram_launch_adapt(const DramState& st, const DramParams& p, void* stream, LaunchTimer* timer) {
  if (timer) timer->begin((hipStream_t)stream);
  int rc;
  // P <= 144: 8 waves x 6 tiles at <= 128 VGPRs (two chains per CU): 109.3 -> 105.2 us per
  // TestData adaptation against 4 waves x 12 tiles (r03af; 28 VGPRs spilled, still faster)
  if (p.pmax <= 16 * 9) {
    rc = launch_adapt_mfma<8, 9, 6, 4>(st, p, stream);
  } else if (p.pmax <= 16 * 13 && p.pmax <= kAdaptGtFrom) {
    // P <= 208: 8 waves x 12 tiles (16 waves x 6 tiles measured slower)
    rc = launch_adapt_mfma<8, 13, 12>(st, p, stream);
  } else {
    const size_t lds = (size_t)adapt_gt_lds_bytes(p.pmax, p.adaptint);
    if (ensure_dyn_lds((const void*)k_adapt_gt, lds) != TCI_OK) return TCI_EHIP;
    hipLaunchKernelGGL(k_adapt_gt, chain_grid(st.n_chains), dim3(64 * kGtWaves), lds, (hipStream_t)stream, st, p);
    rc = finish();
  }
  if (timer) timer->end(2, (hipStream_t)stream);
  return rc;
}
int dram_launch_draws_rng(const DramState& st, const DramParams& p, int64_t s_begin, int64_t s_end, int wgs,
                          void* stream, LaunchTimer* timer) {
  const size_t lds = (size_t)draws_rng_lds_bytes(st.ld);
  if (ensure_dyn_lds((const void*)k_draws_rng, lds) != TCI_OK) return TCI_EHIP;
  if (timer) timer->begin((hipStream_t)stream);
  hipLaunchKernelGGL(k_draws_rng, dim3((unsigned)std::max(wgs, 1)), dim3(kThreads), lds, (hipStream_t)stream, st, p, s_begin,
                     s_end);
  if (timer) timer->end(3, (hipStream_t)stream);
  return finish();
}
int64_t dram_draws_rng_lds_bytes(int64_t ld) { return draws_rng_lds_bytes(ld); }
int dram_launch_chain(const DramState& st, const DramParams& p, const KParams& kp, int rpl, int64_t s_begin,
                      int64_t s_end, int with_records, void* stream, LaunchTimer* timer, const ChainNext* nx) {
  hipStream_t s = (hipStream_t)stream;
  switch (rpl) {
    case 1: return launch_chain_r<1>(st, p, kp, s_begin, s_end, with_records, s, timer, nx);
    case 2: return launch_chain_r<2>(st, p, kp, s_begin, s_end, with_records, s, timer, nx);
    case 4: return launch_chain_r<4>(st, p, kp, s_begin, s_end, with_records, s, timer, nx);
    case 8: return launch_chain_r<8>(st, p, kp, s_begin, s_end, with_records, s, timer, nx);
    default: return TCI_EINVAL;
  }
}
int64_t dram_adapt_lds_bytes(int64_t pmax, int64_t adaptint) {
  if (adaptint <= 0) return 0;
  // the kernel dram_launch_adapt picks, its dynamic LDS, plus its static __shared__ (read from the code
  // object, so a later change to the kernel's static arrays is counted)
  const void* k;
  int64_t dyn;
  if (pmax <= 16 * 9) {
    k = (const void*)k_adapt_mfma<8, 9, 6, 4>;
    dyn = adapt_mfma_lds_bytes(pmax, adaptint);
  } else if (pmax <= 16 * 13 && pmax <= kAdaptGtFrom) {
    k = (const void*)k_adapt_mfma<8, 13, 12>;
    dyn = adapt_mfma_lds_bytes(pmax, adaptint);
  } else {
    k = (const void*)k_adapt_gt;
    dyn = adapt_gt_lds_bytes(pmax, adaptint);
  }
  hipFuncAttributes a{};
  const int64_t stat = hipFuncGetAttributes(&a, k) == hipSuccess ? (int64_t)a.sharedSizeBytes : 4096;
  return dyn + stat;
}
int64_t dram_chain_lds_bytes(int64_t ld, int rpl) {
  const int64_t ns = 4 * (rpl <= 2 ? kChainEPW : 1);  // k_chain: evl, yl, xch, xip (and slack)
  const int64_t chain = (4 * (4 * 64 * rpl + 4 * rpl) + 2 * ns * 64 * (rpl + 1) + 2 * ns * 4 + 2 * ns + 16) * 8;
  return std::max<int64_t>(chain, draws_lds_bytes(ld));                                  // k_draws (dynamic)
}
int dram_launch_stats(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_stats, dim3((unsigned)((st.n_chains + 3) / 4)), dim3(kThreads), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_step_incr(const DramState& st, void* stream) {
  hipLaunchKernelGGL(k_step_incr, dim3(1), dim3(64), 0, (hipStream_t)stream, st.step);
  return finish();
}

}  // namespace tci
