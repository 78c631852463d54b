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
//             q1 = exp(-0.5*(|(newpar2-newpar)*iR|^2 - |(oldpar-newpar)*iR|^2))
//             alpha13 = l2*q1*(1-alpha32)/(1-alpha12)
//   sigma2    1/sigma2 ~ Gamma((N0+N)/2, scale 2/(N0*S20 + oldss)), N0 = 0, N = length(ydata)
//   adapt     every adaptint steps: burn-in (step < burnintime): R scaled by 1/burnin_scale or
//             burnin_scale when the window's rejection rate is > 0.95 or < 0.05; afterwards
//             covupd over all chain rows so far, R = chol(cov + qcovadj*I) * adascale
//   prior     sum(((theta - mu)./sig).^2) over parameters with finite sig (dR: N(0, 50), :254)
// Randomness: Philox4x32-10 keyed by (seed), counter (chain, step, purpose, index) -- the
// stream is reproducible and independent of launch geometry (MATLAB's MT19937 is not
// reproducible here, so chain parity with the reference is statistical only).
//
// Kernels: one wavefront per chain for propose/accept (4 chains per 256-thread block), one
// 256-thread workgroup per chain for adaptation. The SS of the proposals is the batched
// likelihood kernel (tci_kernels.hip), launched between these kernels on device buffers.
#include <hip/hip_runtime.h>
#include <math.h>

#include "tci_dram_internal.h"

namespace tci {

namespace {

constexpr int kWaves = 4;

enum Purpose : uint32_t { P_NORM1 = 1, P_U1 = 2, P_NORM2 = 3, P_U2 = 4, P_GAMMA = 5 };

__device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

// Philox4x32-10 (Salmon et al. 2011).
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = mulhi32(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
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

// Standard normal number `j` of the stream (chain, step, purpose): Box-Muller on pairs.
__device__ __forceinline__ double normal_at(uint64_t seed, int64_t c, int64_t step, uint32_t purpose, int j) {
  const uint4 r = rng(seed, c, step, purpose, (uint32_t)(j >> 1));
  const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
  const double rad = sqrt(-2.0 * log(u1));
  return (j & 1) ? rad * sin(2.0 * M_PI * u2) : rad * cos(2.0 * M_PI * u2);
}

__device__ __forceinline__ double uniform_at(uint64_t seed, int64_t c, int64_t step, uint32_t purpose) {
  const uint4 r = rng(seed, c, step, purpose, 0);
  return u01(r.x, r.y);
}

// Gamma(a, scale) by Marsaglia & Tsang (a >= 1 here: a = N/2 >= 2).
__device__ double gamma_at(uint64_t seed, int64_t c, int64_t step, double a, double scale) {
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
    if (log(u) < 0.5 * x * x + d - d * v + d * log(v)) return d * v * scale;
  }
  return a * scale;  // unreachable in practice (acceptance > 0.95 per try)
}

__device__ __forceinline__ double wsum64(double x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
  return x;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// prior SS: sum(((th - mu) ./ sig).^2) (mcmcstat default priorfun)
__device__ double prior_ss(const double* th, const double* mu, const double* sig, int P, int lane) {
  double s = 0.0;
  for (int j = lane; j < P; j += 64) {
    const double sg = sig[j];
    if (isfinite(sg)) {
      const double z = (th[j] - mu[j]) / sg;
      s += z * z;
    }
  }
  return wsum64(s);
}

// Column j of the row-vector product (v * M)_j = sum_{i<=j} v_i M[i][j] for an upper-triangular
// row-major M (stride ld), for the 64 columns j0..j0+63 (one per lane). v in LDS. Eight
// independent loads are issued per round so the L2/MALL latency overlaps (the wave is otherwise
// latency-bound on one dependent load per term).
__device__ __forceinline__ double tri_col(const double* v, const double* M, int64_t ld, int j0, int j, int P) {
  const int imax = (j0 + 63 < P - 1 ? j0 + 63 : P - 1);  // uniform
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int i = 0;
  for (; i + 7 <= imax; i += 8) {
    double r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = (i + u <= j && j < P) ? M[(int64_t)(i + u) * ld + j] : 0.0;
    a0 = fma(v[i + 0], r[0], a0);
    a1 = fma(v[i + 1], r[1], a1);
    a2 = fma(v[i + 2], r[2], a2);
    a3 = fma(v[i + 3], r[3], a3);
    a0 = fma(v[i + 4], r[4], a0);
    a1 = fma(v[i + 5], r[5], a1);
    a2 = fma(v[i + 6], r[6], a2);
    a3 = fma(v[i + 7], r[7], a3);
  }
  for (; i <= imax; ++i)
    if (i <= j && j < P) a0 = fma(v[i], M[(int64_t)i * ld + j], a0);
  return (a0 + a1) + (a2 + a3);
}

// out[j] = base[j] + scale * sum_i z_i R[i][j] (R upper triangular, row-major ld); returns whether
// every out[j] is inside [lo, hi]. z in LDS.
__device__ bool propose(const double* base, const double* R, int64_t ld, const double* z, double scale, int P,
                        const double* lo, const double* hi, double* out, int lane) {
  bool inb = true;
  for (int j0 = 0; j0 < P; j0 += 64) {
    const int j = j0 + lane;
    const double acc = tri_col(z, R, ld, j0, j, P);
    if (j < P) {
      const double v = base[j] + scale * acc;
      out[j] = v;
      inb = inb && v >= lo[j] && v <= hi[j];
    }
  }
  return __all(inb);
}

// |d * iR|^2 with d = a - b (row vector), iR upper triangular.
__device__ double mahal(const double* a, const double* b, const double* iR, int64_t ld, int P, double* dl, int lane) {
  for (int j = lane; j < P; j += 64) dl[j] = a[j] - b[j];
  wave_sync();
  double s = 0.0;
  for (int j0 = 0; j0 < P; j0 += 64) {
    const int j = j0 + lane;
    const double acc = tri_col(dl, iR, ld, j0, j, P);
    if (j < P) s += acc * acc;
  }
  wave_sync();
  return wsum64(s);
}

__global__ __launch_bounds__(256) void k_init(DramState st, const double* __restrict__ qdiag,
                                              const double* __restrict__ s2_0) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (c >= st.n_chains) return;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  double* R = st.R + c * ld * ld;
  double* iR = st.iR + c * ld * ld;
  double* cv = st.cov + c * ld * ld;
  for (int64_t e = lane; e < ld * ld; e += 64) {
    R[e] = 0.0;
    iR[e] = 0.0;
    cv[e] = 0.0;
  }
  for (int j = lane; j < P; j += 64) {
    const double sd = sqrt(qdiag[c * ld + j]);  // R = chol(qcov), qcov = J0 diagonal (:230)
    R[(int64_t)j * ld + j] = sd;
    iR[(int64_t)j * ld + j] = 1.0 / sd;
    st.cmean[c * ld + j] = 0.0;
  }
  const double pr = prior_ss(st.theta + c * ld, st.pmu + c * ld, st.psig + c * ld, P, lane);
  if (lane == 0) {
    st.prior[c] = pr;
    st.sigma2[c] = s2_0[c];
    st.wsum[c] = 0.0;
    st.naccept[c] = 0;
    st.nrej_win[c] = 0;
    st.nevals[c] = 1;  // the initial ssfun call
  }
}

// Row 1 of the chain (the initial state): window, stats, thinned output.
__device__ void record_row(const DramState& st, const DramParams& p, int64_t c, int64_t row, int P, int lane) {
  const int64_t ld = st.ld;
  const double* th = st.theta + c * ld;
  if (p.adaptint > 0) {
    double* w = st.window + (c * p.adaptint + (row - 1) % p.adaptint) * ld;
    for (int j = lane; j < P; j += 64) w[j] = th[j];
  }
  if (row >= p.stats_from) {  // posterior mean / population std over chain(stats_from:end, :) (:276-301)
    const double n = (double)(row - p.stats_from + 1);
    for (int j = lane; j < P; j += 64) {
      const double x = th[j];
      double m = st.smean[c * ld + j];
      const double d = x - m;
      m += d / n;
      st.smean[c * ld + j] = m;
      st.sm2[c * ld + j] += d * (x - m);
    }
  }
  if (lane == 0) {  // s2 statistics over the whole s2chain (:302-303)
    const double s2 = st.sigma2[c];
    st.s2sum[c] += s2;
    const double q = sqrt(s2), n = (double)row;
    const double d = q - st.sq_mean[c];
    st.sq_mean[c] += d / n;
    st.sq_m2[c] += d * (q - st.sq_mean[c]);
  }
  if (st.chain_out != nullptr && p.thin > 0 && (row - 1) % p.thin == 0) {
    const int64_t k = (row - 1) / p.thin;
    if (k < p.n_keep) {
      for (int j = lane; j < P; j += 64) st.chain_out[(k * st.n_chains + c) * ld + j] = th[j];
      if (lane == 0 && st.s2_out) st.s2_out[k * st.n_chains + c] = st.sigma2[c];
    }
  }
}

__global__ __launch_bounds__(256) void k_init_stats(DramState st, DramParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (c >= st.n_chains) return;
  const int P = st.npar[c];
  for (int j = lane; j < P; j += 64) {
    st.smean[c * st.ld + j] = 0.0;
    st.sm2[c * st.ld + j] = 0.0;
  }
  if (lane == 0) {
    st.s2sum[c] = 0.0;
    st.sq_mean[c] = 0.0;
    st.sq_m2[c] = 0.0;
  }
  wave_sync();
  record_row(st, p, c, 1, P, lane);
}

__global__ __launch_bounds__(256) void k_propose1(DramState st, DramParams p) {
  __shared__ double zs[kWaves][TCI_MAX_POINTS + 8];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * kWaves + w;
  if (c >= st.n_chains) return;
  const int64_t step = *st.step;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  for (int j = lane; j < P; j += 64) zs[w][j] = normal_at(p.seed, c, step, P_NORM1, j);
  wave_sync();
  const bool inb = propose(st.theta + c * ld, st.R + c * ld * ld, ld, zs[w], 1.0, P, st.lower + c * ld,
                           st.upper + c * ld, st.prop1 + c * ld, lane);
  if (lane == 0) {
    st.act1[c] = inb ? 1 : 0;
    if (inb) st.nevals[c] += 1;
  }
}

__global__ __launch_bounds__(256) void k_accept1(DramState st, DramParams p) {
  __shared__ double zs[kWaves][TCI_MAX_POINTS + 8];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * kWaves + w;
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
    pr1 = prior_ss(y1, st.pmu + c * ld, st.psig + c * ld, P, lane);
    const double e = -0.5 * (st.ss1[c] - st.ss[c]) / st.sigma2[c] - 0.5 * (pr1 - st.prior[c]);
    a12 = fmin(1.0, exp(e));
    acc = uniform_at(p.seed, c, step, P_U1) < a12;
  }
  if (acc) {
    for (int j = lane; j < P; j += 64) th[j] = y1[j];
    if (lane == 0) {
      st.ss[c] = st.ss1[c];
      st.prior[c] = pr1;
      st.naccept[c] += 1;
    }
  }
  if (lane == 0) {
    st.a12[c] = a12;
    st.prior1[c] = pr1;
  }
  bool inb2 = false;
  if (!acc && p.ntry >= 2) {  // delayed rejection: second try with R / drscale
    for (int j = lane; j < P; j += 64) zs[w][j] = normal_at(p.seed, c, step, P_NORM2, j);
    wave_sync();
    inb2 = propose(th, st.R + c * ld * ld, ld, zs[w], 1.0 / p.drscale, P, st.lower + c * ld, st.upper + c * ld,
                   st.prop2 + c * ld, lane);
  }
  if (lane == 0) {
    st.acc1[c] = acc ? 1 : 0;
    st.act2[c] = inb2 ? 1 : 0;
    if (inb2) st.nevals[c] += 1;
  }
}

__global__ __launch_bounds__(256) void k_accept2(DramState st, DramParams p) {
  __shared__ double dl[kWaves][TCI_MAX_POINTS + 8];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * kWaves + w;
  if (c >= st.n_chains) return;
  const int64_t step = *st.step;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  double* th = st.theta + c * ld;
  bool acc2 = false;
  if (p.ntry >= 2 && st.act2[c] != 0) {  // stage 2 was proposed (stage 1 rejected) and is in bounds
    const double* y1 = st.prop1 + c * ld;
    const double* y2 = st.prop2 + c * ld;
    const double pr2 = prior_ss(y2, st.pmu + c * ld, st.psig + c * ld, P, lane);
    const double s2 = st.sigma2[c], ss2 = st.ss2[c], ss1 = st.ss1[c], a12 = st.a12[c];
    // ss1 = +Inf (stage 1 out of bounds) gives alpha32 = 0, alpha12 = 0
    const double a32 = fmin(1.0, exp(-0.5 * (ss1 - ss2) / s2 - 0.5 * (st.prior1[c] - pr2)));
    const double l2 = exp(-0.5 * (ss2 - st.ss[c]) / s2 - 0.5 * (pr2 - st.prior[c]));
    const double* iR = st.iR + c * ld * ld;
    const double m21 = mahal(y2, y1, iR, ld, P, dl[w], lane);
    const double m01 = mahal(th, y1, iR, ld, P, dl[w], lane);
    const double q1 = exp(-0.5 * (m21 - m01));
    const double a13 = l2 * q1 * (1.0 - a32) / (1.0 - a12);
    acc2 = uniform_at(p.seed, c, step, P_U2) < a13;
    if (acc2) {
      for (int j = lane; j < P; j += 64) th[j] = y2[j];
      if (lane == 0) {
        st.ss[c] = ss2;
        st.prior[c] = pr2;
        st.naccept[c] += 1;
      }
    }
  }
  if (lane == 0 && !(st.acc1[c] != 0 || acc2)) st.nrej_win[c] += 1;  // no stage moved the chain
  // sigma2 Gibbs update (updatesigma = 1, :265): 1/sigma2 ~ Gamma(N/2, scale 2/oldss)
  if (p.updatesigma && lane == 0) {
    const double a = 0.5 * (double)st.nobs[c];
    st.sigma2[c] = 1.0 / gamma_at(p.seed, c, step, a, 2.0 / st.ss[c]);
  }
  wave_sync();
  record_row(st, p, c, step, P, lane);
}

__global__ void k_step_incr(int64_t* step) {
  if (threadIdx.x == 0) *step += 1;
}

// Adaptation (one 256-thread workgroup per chain).
__global__ __launch_bounds__(256) void k_adapt(DramState st, DramParams p) {
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t step = *st.step;
  if (c >= st.n_chains || p.adaptint <= 0 || step % p.adaptint != 0) return;  // uniform exit
  double* work = st.work;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  double* cv = st.cov + c * ld * ld;
  double* mu = st.cmean + c * ld;
  double* R = st.R + c * ld * ld;
  double* iR = st.iR + c * ld * ld;
  double* A = work + c * ld * ld;
  __shared__ double xs[TCI_MAX_POINTS + 8];
  __shared__ double dm[TCI_MAX_POINTS + 8];
  __shared__ int fail;
  // ---- covupd: fold the window rows (chain rows step-adaptint+1 .. step) into (mean, cov, wsum)
  const int64_t nrows = p.adaptint;
  double ws = st.wsum[c];
  for (int64_t r = 0; r < nrows; ++r) {
    const double* x = st.window + (c * p.adaptint + r) * ld;
    for (int j = t; j < P; j += 256) xs[j] = x[j];
    __syncthreads();
    if (ws == 0.0) {  // first row: mean = x, cov = 0
      for (int j = t; j < P; j += 256) mu[j] = xs[j];
      __syncthreads();
      ws = 1.0;
      continue;
    }
    for (int j = t; j < P; j += 256) dm[j] = xs[j] - mu[j];
    __syncthreads();
    // xcov = oldcov + w/(w+oldwsum-1) * (oldwsum/(w+oldwsum) * d'd - oldcov), w = 1
    const double f1 = 1.0 / ws, f2 = ws / (ws + 1.0);
    for (int64_t e = t; e < (int64_t)P * P; e += 256) {
      const int i = (int)(e / P), j = (int)(e % P);
      if (j < i) continue;
      const double old = cv[(int64_t)i * ld + j];
      cv[(int64_t)i * ld + j] = old + f1 * (f2 * dm[i] * dm[j] - old);
    }
    for (int j = t; j < P; j += 256) mu[j] = mu[j] + dm[j] / (ws + 1.0);
    ws += 1.0;
    __syncthreads();
  }
  if (t == 0) st.wsum[c] = ws;
  if (step < p.burnintime) {
    // burn-in: no covariance adaptation, only scaling by the window's rejection rate
    const double rate = (double)st.nrej_win[c] / (double)p.adaptint;
    double s = 1.0;
    if (rate > 0.95) s = 1.0 / p.burnin_scale;
    else if (rate < 0.05) s = p.burnin_scale;
    if (s != 1.0) {
      for (int64_t e = t; e < (int64_t)P * P; e += 256) {
        const int i = (int)(e / P), j = (int)(e % P);
        R[(int64_t)i * ld + j] *= s;
        iR[(int64_t)i * ld + j] /= s;
      }
    }
    __syncthreads();
    if (t == 0) st.nrej_win[c] = 0;
    return;
  }
  // ---- R = chol(cov + qcovadj*I) * adascale (upper, A = R'R), then iR = inv(R)
  for (int64_t e = t; e < (int64_t)P * P; e += 256) {
    const int i = (int)(e / P), j = (int)(e % P);
    A[(int64_t)i * ld + j] = j >= i ? cv[(int64_t)i * ld + j] + (i == j ? p.qcovadj : 0.0) : 0.0;
  }
  if (t == 0) fail = 0;
  __syncthreads();
  for (int k = 0; k < P; ++k) {
    if (t == 0) {
      const double d = A[(int64_t)k * ld + k];
      if (!(d > 0.0) || !isfinite(d)) fail = 1;
      A[(int64_t)k * ld + k] = sqrt(d);
    }
    __syncthreads();
    if (fail) break;
    const double dk = A[(int64_t)k * ld + k];
    for (int j = k + 1 + t; j < P; j += 256) A[(int64_t)k * ld + j] /= dk;
    __syncthreads();
    const int m = P - k - 1;
    for (int64_t e = t; e < (int64_t)m * m; e += 256) {
      const int i = k + 1 + (int)(e / m), j = k + 1 + (int)(e % m);
      if (j >= i) A[(int64_t)i * ld + j] -= A[(int64_t)k * ld + i] * A[(int64_t)k * ld + j];
    }
    __syncthreads();
  }
  if (!fail) {  // singular: keep the previous R (mcmcstat: "cmat singular, not adapting")
    const double sc = p.adascale > 0.0 ? p.adascale : 2.4 / sqrt((double)P);
    for (int64_t e = t; e < (int64_t)P * P; e += 256) {
      const int i = (int)(e / P), j = (int)(e % P);
      R[(int64_t)i * ld + j] = j >= i ? A[(int64_t)i * ld + j] * sc : 0.0;
    }
    __syncthreads();
    // iR = R \ I : column j by back substitution (one thread per column)
    for (int j = t; j < P; j += 256) {
      for (int i = P - 1; i >= 0; --i) {
        double v;
        if (i > j) {
          v = 0.0;
        } else {
          double s = i == j ? 1.0 : 0.0;
          for (int k = i + 1; k <= j; ++k) s -= R[(int64_t)i * ld + k] * iR[(int64_t)k * ld + j];
          v = s / R[(int64_t)i * ld + i];
        }
        iR[(int64_t)i * ld + j] = v;
      }
    }
  }
  __syncthreads();
  if (t == 0) st.nrej_win[c] = 0;
}

inline int finish() { return hipGetLastError() == hipSuccess ? TCI_OK : TCI_EHIP; }
inline dim3 wave_grid(int64_t n) { return dim3((unsigned)((n + kWaves - 1) / kWaves)); }

}  // namespace

int dram_launch_init(const DramState& st, const double* qcov_diag, const double* sigma2_0, void* stream) {
  hipLaunchKernelGGL(k_init, wave_grid(st.n_chains), dim3(256), 0, (hipStream_t)stream, st, qcov_diag, sigma2_0);
  return finish();
}
int dram_launch_init_stats(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_init_stats, wave_grid(st.n_chains), dim3(256), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_propose1(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_propose1, wave_grid(st.n_chains), dim3(256), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_accept1(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_accept1, wave_grid(st.n_chains), dim3(256), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_accept2(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_accept2, wave_grid(st.n_chains), dim3(256), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_adapt(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_adapt, dim3((unsigned)st.n_chains), dim3(256), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_step_incr(const DramState& st, void* stream) {
  hipLaunchKernelGGL(k_step_incr, dim3(1), dim3(64), 0, (hipStream_t)stream, st.step);
  return finish();
}

}  // namespace tci
