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
#include "tci_eval.h"

namespace tci {

namespace {

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

constexpr int kThreads = 256;  // one workgroup (4 waves) per chain
constexpr int kVec = TCI_MAX_POINTS + 8;

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
    const double sg = sig[j];
    if (isfinite(sg)) {
      const double z = (th[j] - mu[j]) / sg;
      s += z * z;
    }
  }
  return block_sum(s, red);
}

// Row-vector times upper-triangular matrix, out_j = sum_{i<=j} v_i M[i][j] (M row-major, stride
// ld, in global memory), for up to two vectors sharing each load of M. Wave w takes the rows
// i == w (mod 4) (balanced over the triangle); lanes take columns; 8 loads in flight per lane.
// v0/v1 and the outputs are in LDS; part = LDS [2][4][ps] (ps >= P).
template <int NV>
__device__ void tri_vecmat(const double* v0, const double* v1, const double* M, int64_t ld, int P, double* part,
                           double* out0, double* out1, int ps = kVec) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int j0 = 0; j0 < P; j0 += 64) {
    const int j = j0 + lane;
    const int imax = (j0 + 63 < P - 1 ? j0 + 63 : P - 1);  // uniform
    double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
    int i = w;
    for (; i + 28 <= imax; i += 32) {
      double r[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int ii = i + 4 * u;
        r[u] = (ii <= j && j < P) ? M[(int64_t)ii * ld + j] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        a0 = fma(v0[i + 4 * u], r[u], a0);
        a1 = fma(v0[i + 4 * u + 4], r[u + 1], a1);
        if (NV == 2) {
          b0 = fma(v1[i + 4 * u], r[u], b0);
          b1 = fma(v1[i + 4 * u + 4], r[u + 1], b1);
        }
      }
    }
    for (; i <= imax; i += 4) {
      const double r = (i <= j && j < P) ? M[(int64_t)i * ld + j] : 0.0;
      a0 = fma(v0[i], r, a0);
      if (NV == 2) b0 = fma(v1[i], r, b0);
    }
    if (j < P) {
      part[(0 * 4 + w) * ps + j] = a0 + a1;
      if (NV == 2) part[(1 * 4 + w) * ps + j] = b0 + b1;
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < P; j += kThreads) {
    out0[j] = (part[0 * ps + j] + part[1 * ps + j]) + (part[2 * ps + j] + part[3 * ps + j]);
    if (NV == 2) out1[j] = (part[4 * ps + j] + part[5 * ps + j]) + (part[6 * ps + j] + part[7 * ps + j]);
  }
  __syncthreads();
}

struct Smem {
  double z[kVec];
  double y[kVec];
  double d0[kVec];
  double d1[kVec];
  double part[8 * kVec];
  double red[8];
  int flag;
};

// Draw z (stream `purpose`), y = base + scale * z*R into LDS and global `out`; returns in-bounds.
__device__ bool propose_block(const DramState& st, const DramParams& p, int64_t c, int64_t step, uint32_t purpose,
                              const double* base, double scale, int P, double* out, Smem& sm) {
  const int64_t ld = st.ld;
  for (int j = threadIdx.x; j < P; j += kThreads) sm.z[j] = normal_at(p.seed, c, step, purpose, j);
  __syncthreads();
  tri_vecmat<1>(sm.z, nullptr, st.R + c * ld * ld, ld, P, sm.part, sm.y, nullptr);
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
  double* R = st.R + c * ld * ld;
  double* iR = st.iR + c * ld * ld;
  double* cv = st.cov + c * ld * ld;
  for (int64_t e = threadIdx.x; e < ld * ld; e += kThreads) {
    R[e] = 0.0;
    iR[e] = 0.0;
    cv[e] = 0.0;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < P; j += kThreads) {
    const double sd = sqrt(qdiag[c * ld + j]);  // R = chol(qcov), qcov = J0 diagonal (:230)
    R[(int64_t)j * ld + j] = sd;
    iR[(int64_t)j * ld + j] = 1.0 / sd;
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

// Chain row `row` (1-based) = the current state th (global or LDS) with error variance s2:
// covupd window, posterior stats, thinned output.
__device__ void record_row(const DramState& st, const DramParams& p, int64_t c, int64_t row, int P, const double* th,
                           double s2) {
  const int64_t ld = st.ld;
  const int t = threadIdx.x;
  if (p.adaptint > 0) {
    double* w = st.window + (c * p.adaptint + (row - 1) % p.adaptint) * ld;
    for (int j = t; j < P; j += kThreads) w[j] = th[j];
  }
  if (row >= p.stats_from) {  // posterior mean / population std over chain(stats_from:end, :) (:276-301)
    const double n = (double)(row - p.stats_from + 1);
    for (int j = t; j < P; j += kThreads) {
      const double x = th[j];
      double m = st.smean[c * ld + j];
      const double d = x - m;
      m += d / n;
      st.smean[c * ld + j] = m;
      st.sm2[c * ld + j] += d * (x - m);
    }
  }
  if (t == 0) {  // s2 statistics over the whole s2chain (:302-303)
    st.s2sum[c] += s2;
    const double q = sqrt(s2), n = (double)row;
    const double d = q - st.sq_mean[c];
    st.sq_mean[c] += d / n;
    st.sq_m2[c] += d * (q - st.sq_mean[c]);
  }
  if (st.chain_out != nullptr && p.thin > 0 && (row - 1) % p.thin == 0) {
    const int64_t k = (row - 1) / p.thin;
    if (k < p.n_keep) {
      for (int j = t; j < P; j += kThreads) st.chain_out[(k * st.n_chains + c) * ld + j] = th[j];
      if (t == 0 && st.s2_out) st.s2_out[k * st.n_chains + c] = s2;
    }
  }
}

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
  __syncthreads();
  record_row(st, p, c, 1, P, st.theta + c * st.ld, st.sigma2[c]);
}

__global__ __launch_bounds__(kThreads) void k_propose1(DramState st, DramParams p) {
  __shared__ Smem sm;
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
  __shared__ Smem sm;
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
    pr1 = prior_ss(y1, st.pmu + c * ld, st.psig + c * ld, P, sm.red);
    const double e = -0.5 * (st.ss1[c] - st.ss[c]) / st.sigma2[c] - 0.5 * (pr1 - st.prior[c]);
    a12 = fmin(1.0, exp(e));
    acc = uniform_at(p.seed, c, step, P_U1) < a12;
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
  __shared__ Smem sm;
  const int64_t c = blockIdx.x;
  if (c >= st.n_chains) return;
  const int64_t step = *st.step;
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  double* th = st.theta + c * ld;
  bool acc2 = false;
  if (p.ntry >= 2 && st.act2[c] != 0) {  // stage 2 was proposed (stage 1 rejected) and is in bounds
    const double* y1 = st.prop1 + c * ld;
    const double* y2 = st.prop2 + c * ld;
    const double pr2 = prior_ss(y2, st.pmu + c * ld, st.psig + c * ld, P, sm.red);
    const double s2 = st.sigma2[c], ss2 = st.ss2[c], ss1 = st.ss1[c], a12 = st.a12[c];
    // ss1 = +Inf (stage 1 out of bounds) gives alpha32 = 0, alpha12 = 0
    const double a32 = fmin(1.0, exp(-0.5 * (ss1 - ss2) / s2 - 0.5 * (st.prior1[c] - pr2)));
    const double l2 = exp(-0.5 * (ss2 - st.ss[c]) / s2 - 0.5 * (pr2 - st.prior[c]));
    for (int j = threadIdx.x; j < P; j += kThreads) {
      sm.d1[j] = y2[j] - y1[j];
      sm.d0[j] = th[j] - y1[j];
    }
    __syncthreads();
    tri_vecmat<2>(sm.d1, sm.d0, st.iR + c * ld * ld, ld, P, sm.part, sm.z, sm.y);
    double q21 = 0.0, q01 = 0.0;
    for (int j = threadIdx.x; j < P; j += kThreads) {
      q21 += sm.z[j] * sm.z[j];
      q01 += sm.y[j] * sm.y[j];
    }
    q21 = block_sum(q21, sm.red);
    q01 = block_sum(q01, sm.red);
    const double q1 = exp(-0.5 * (q21 - q01));  // |(y2-y1) iR|^2 - |(x-y1) iR|^2
    const double a13 = l2 * q1 * (1.0 - a32) / (1.0 - a12);
    acc2 = uniform_at(p.seed, c, step, P_U2) < a13;
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
    if (p.updatesigma) st.sigma2[c] = 1.0 / gamma_at(p.seed, c, step, 0.5 * (double)st.nobs[c], 2.0 / st.ss[c]);
  }
  __syncthreads();
  record_row(st, p, c, step, P, st.theta + c * st.ld, st.sigma2[c]);
}

__global__ void k_step_incr(int64_t* step) {
  if (threadIdx.x == 0) *step += 1;
}

// Adaptation, one workgroup per chain (launched only at steps that are multiples of adaptint).
// Matrices live in LDS when P*P*8 bytes fit (every TestData cell: P <= 136), else in global.
__global__ __launch_bounds__(kThreads) void k_adapt(DramState st, DramParams p) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ double xs[kVec];
  __shared__ double dm[kVec];
  __shared__ int fail;
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t step = *st.step;
  if (c >= st.n_chains || p.adaptint <= 0 || step % p.adaptint != 0) return;  // uniform exit
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  double* cvg = st.cov + c * ld * ld;
  double* mu = st.cmean + c * ld;
  double* R = st.R + c * ld * ld;
  double* iR = st.iR + c * ld * ld;
  const bool in_lds = p.lds_matrix != 0;
  double* A = in_lds ? dyn : st.work + c * ld * ld;
  const int64_t lda = in_lds ? P : ld;
  // ---- covupd: fold the window rows (chain rows step-adaptint+1 .. step) into (mean, cov, wsum)
  for (int64_t e = t; e < (int64_t)P * P; e += kThreads) {
    const int i = (int)(e / P), j = (int)(e % P);
    if (j >= i) A[(int64_t)i * lda + j] = cvg[(int64_t)i * ld + j];
  }
  double ws = st.wsum[c];
  __syncthreads();
  for (int64_t r = 0; r < p.adaptint; ++r) {
    const double* x = st.window + (c * p.adaptint + r) * ld;
    for (int j = t; j < P; j += kThreads) xs[j] = x[j];
    __syncthreads();
    if (ws == 0.0) {  // first row: mean = x, cov = 0
      for (int j = t; j < P; j += kThreads) mu[j] = xs[j];
      __syncthreads();
      ws = 1.0;
      continue;
    }
    for (int j = t; j < P; j += kThreads) dm[j] = xs[j] - mu[j];
    __syncthreads();
    // xcov = oldcov + w/(w+oldwsum-1) * (oldwsum/(w+oldwsum) * d'd - oldcov), w = 1
    const double f1 = 1.0 / ws, f2 = ws / (ws + 1.0);
    for (int64_t e = t; e < (int64_t)P * P; e += kThreads) {
      const int i = (int)(e / P), j = (int)(e % P);
      if (j < i) continue;
      const double old = A[(int64_t)i * lda + j];
      A[(int64_t)i * lda + j] = old + f1 * (f2 * dm[i] * dm[j] - old);
    }
    for (int j = t; j < P; j += kThreads) mu[j] = mu[j] + dm[j] / (ws + 1.0);
    ws += 1.0;
    __syncthreads();
  }
  for (int64_t e = t; e < (int64_t)P * P; e += kThreads) {
    const int i = (int)(e / P), j = (int)(e % P);
    if (j >= i) cvg[(int64_t)i * ld + j] = A[(int64_t)i * lda + j];
  }
  if (t == 0) st.wsum[c] = ws;
  __syncthreads();  // the copy-back must read A before the Cholesky below modifies it
  if (step < p.burnintime) {
    // burn-in: no covariance adaptation, only scaling by the window's rejection rate
    const double rate = (double)st.nrej_win[c] / (double)p.adaptint;
    double s = 1.0;
    if (rate > 0.95) s = 1.0 / p.burnin_scale;
    else if (rate < 0.05) s = p.burnin_scale;
    if (s != 1.0) {
      for (int64_t e = t; e < (int64_t)P * P; e += kThreads) {
        const int i = (int)(e / P), j = (int)(e % P);
        R[(int64_t)i * ld + j] *= s;
        iR[(int64_t)i * ld + j] /= s;
      }
    }
    __syncthreads();
    if (t == 0) st.nrej_win[c] = 0;
    return;
  }
  // ---- R = chol(cov + qcovadj*I) * adascale (upper, A = R'R), in place on A
  for (int i = t; i < P; i += kThreads) A[(int64_t)i * lda + i] += p.qcovadj;
  if (t == 0) fail = 0;
  __syncthreads();
  for (int k = 0; k < P; ++k) {
    if (t == 0) {
      const double d = A[(int64_t)k * lda + k];
      if (!(d > 0.0) || !isfinite(d)) fail = 1;
      A[(int64_t)k * lda + k] = sqrt(d);
    }
    __syncthreads();
    if (fail) break;
    const double dk = A[(int64_t)k * lda + k];
    for (int j = k + 1 + t; j < P; j += kThreads) A[(int64_t)k * lda + j] /= dk;
    __syncthreads();
    const int m = P - k - 1;
    for (int64_t e = t; e < (int64_t)m * m; e += kThreads) {
      const int i = k + 1 + (int)(e / m), j = k + 1 + (int)(e % m);
      if (j >= i) A[(int64_t)i * lda + j] -= A[(int64_t)k * lda + i] * A[(int64_t)k * lda + j];
    }
    __syncthreads();
  }
  if (!fail) {  // singular: keep the previous R (mcmcstat: "cmat singular, not adapting")
    const double sc = p.adascale > 0.0 ? p.adascale : 2.4 / sqrt((double)P);
    for (int64_t e = t; e < (int64_t)P * P; e += kThreads) {
      const int i = (int)(e / P), j = (int)(e % P);
      const double r = j >= i ? A[(int64_t)i * lda + j] * sc : 0.0;
      A[(int64_t)i * lda + j] = r;  // A now holds R (upper), lower part zero
      R[(int64_t)i * ld + j] = r;
    }
    __syncthreads();
    // iR = R \ I, in place on A, row by row from the bottom: X(i,j) = (d_ij - sum_{k=i+1..j} R(i,k) X(k,j)) / R(i,i)
    for (int i = P - 1; i >= 0; --i) {
      const double rii = A[(int64_t)i * lda + i];
      // row i of R (k > i) is read before being overwritten by row i of X: stage it
      for (int k = i + 1 + t; k < P; k += kThreads) xs[k] = A[(int64_t)i * lda + k];
      __syncthreads();
      for (int j = i + t; j < P; j += kThreads) {
        double s = (i == j) ? 1.0 : 0.0;
        for (int k = i + 1; k <= j; ++k) s -= xs[k] * A[(int64_t)k * lda + j];
        A[(int64_t)i * lda + j] = s / rii;
      }
      __syncthreads();
    }
    for (int64_t e = t; e < (int64_t)P * P; e += kThreads) {
      const int i = (int)(e / P), j = (int)(e % P);
      iR[(int64_t)i * ld + j] = j >= i ? A[(int64_t)i * lda + j] : 0.0;
    }
  }
  __syncthreads();
  if (t == 0) st.nrej_win[c] = 0;
}


// ---- Fused chain engine: one workgroup runs chain rows s_begin..s_end of its chain with every
// ssfun evaluation inside the loop (no launch per step). Waves 0 and 1 evaluate the stage-1
// proposal and the stage-2 proposal concurrently (stage 2 is drawn up front from its own stream
// and used only when stage 1 rejects, so nothing changes but the latency). Adaptation stays the
// k_adapt launch between chunks. Same RNG keys, reductions and operation order as the batched
// engine above: the two engines produce identical chains (tests/test_dram_gpu.py).

// Prior SS from LDS copies of mu / sig (same arithmetic as prior_ss).
__device__ double prior_lds(const double* th, const double* mu, const double* sig, int P, double* red) {
  double s = 0.0;
  for (int j = threadIdx.x; j < P; j += kThreads) {
    const double sg = sig[j];
    if (isfinite(sg)) {
      const double z = (th[j] - mu[j]) / sg;
      s += z * z;
    }
  }
  return block_sum(s, red);
}

#ifndef TCI_CHAIN_PROFILE
#define TCI_CHAIN_PROFILE 0  // diagnostics: per-phase s_memtime cycles of k_chain into st.prof
#endif
__device__ __forceinline__ uint64_t stamp() {
#if TCI_CHAIN_PROFILE
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
#else
  return 0;
#endif
}

// Dynamic LDS doubles of k_chain for vector stride L (>= P): 11 vectors, 8 partial rows, red.
__host__ __device__ inline int64_t chain_lds_doubles(int64_t L) { return 19 * L + 8; }

template <int RPL, int NSEG>
__global__ __launch_bounds__(kThreads) void k_chain(DramState st, DramParams p, KParams kp, int64_t s_begin,
                                                    int64_t s_end) {
  constexpr int EV = eval_lds_doubles<RPL>();
  __shared__ __attribute__((aligned(16))) double evl[2][EV];
  __shared__ double ssv[2];
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  const int64_t c = blockIdx.x;
  if (c >= st.n_chains) return;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int64_t ld = st.ld;
  const int L = (int)ld;
  const int P = st.npar[c];
  double* z = dyn;
  double* y = z + L;
  double* d0 = y + L;
  double* d1 = d0 + L;
  double* y1 = d1 + L;
  double* y2 = y1 + L;
  double* th = y2 + L;
  double* lo = th + L;
  double* hi = lo + L;
  double* mu = hi + L;
  double* sg = mu + L;
  double* part = sg + L;
  double* red = part + 8 * L;
  for (int j = t; j < P; j += kThreads) {
    th[j] = st.theta[c * ld + j];
    lo[j] = st.lower[c * ld + j];
    hi[j] = st.upper[c * ld + j];
    mu[j] = st.pmu[c * ld + j];
    sg[j] = st.psig[c * ld + j];
  }
  // the chain's cell records stay in the registers of the two evaluating waves
  EvalIn<RPL> e;
  if (w < 2) {
    const int cell = st.cell[c];
    const int64_t cbase = (int64_t)cell * kp.cell_stride;
    e.cm = kp.cells[cell];
#pragma unroll
    for (int q = 0; q < RPL; ++q) e.st[q] = kp.steps[cbase + RPL * lane + q];
#pragma unroll
    for (int k = 0; k <= RPL; ++k) {
      const int j = lane + 64 * k;
      e.pt[k] = j <= 64 * RPL ? kp.points[cbase + j] : PointRec{NAN, NAN, NAN, 0, 0};
    }
  }
  double ss = st.ss[c], prior = st.prior[c], s2 = st.sigma2[c];
  int32_t nacc = st.naccept[c], nrej = st.nrej_win[c];
  int64_t nev = st.nevals[c];
  const double half_nobs = 0.5 * (double)st.nobs[c];
  const double* Rm = st.R + c * ld * ld;
  const double* iRm = st.iR + c * ld * ld;
  const double scale2 = 1.0 / p.drscale;
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t t0 = stamp(), t1;
#define TCI_PHASE(k) \
  if (TCI_CHAIN_PROFILE) { t1 = stamp(); ph[k] += t1 - t0; t0 = t1; }
  __syncthreads();
  for (int64_t step = s_begin; step <= s_end; ++step) {
    // ---- proposals: stage 1 theta + z1*R, stage 2 theta + z2*R/drscale (both drawn now)
    for (int j = t; j < P; j += kThreads) {
      z[j] = normal_at(p.seed, c, step, P_NORM1, j);
      d0[j] = p.ntry >= 2 ? normal_at(p.seed, c, step, P_NORM2, j) : 0.0;
    }
    __syncthreads();
    TCI_PHASE(0)
    tri_vecmat<2>(z, d0, Rm, ld, P, part, y, d1, L);
    TCI_PHASE(1)
    int ok1 = 1, ok2 = 1;
    for (int j = t; j < P; j += kThreads) {
      const double a = th[j] + 1.0 * y[j];
      const double b = th[j] + scale2 * d1[j];
      y1[j] = a;
      y2[j] = b;
      ok1 &= (a >= lo[j] && a <= hi[j]) ? 1 : 0;
      ok2 &= (b >= lo[j] && b <= hi[j]) ? 1 : 0;
    }
    const bool inb1 = __syncthreads_and(ok1) != 0;
    const bool inb2 = __syncthreads_and(ok2) != 0 && p.ntry >= 2;
    TCI_PHASE(2)
    // ---- ssfun of both proposals, one wavefront each (out of bounds: not called, +Inf)
    if (w < 2) {
      const double* yy = w == 0 ? y1 : y2;
      double r = INFINITY;
      if (w == 0 ? inb1 : inb2) {
        e.v = yy[0];
        e.tau = yy[1];
        e.ton = yy[2];
        e.b1 = yy[3];
        e.b2 = yy[4];
        e.A = yy[5];
        e.R = yy[6];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
          const int g = RPL * lane + q;
          e.dr[q] = 7 + g < P ? yy[7 + g] : 0.0;
        }
        r = eval_wave<RPL, NSEG, MODE_SS>(kp, e, lane, evl[w], 0, nullptr, nullptr, 0);
      }
      if (lane == 0) ssv[w] = r;
    }
    __syncthreads();
    TCI_PHASE(3)
    const double ss1 = ssv[0], ss2 = ssv[1];
    // ---- stage 1 (k_accept1)
    double a12 = 0.0, pr1 = 0.0;
    bool acc = false;
    if (inb1) {
      nev += 1;
      pr1 = prior_lds(y1, mu, sg, P, red);
      const double ex = -0.5 * (ss1 - ss) / s2 - 0.5 * (pr1 - prior);
      a12 = fmin(1.0, exp(ex));
      acc = uniform_at(p.seed, c, step, P_U1) < a12;
    }
    if (acc) {
      for (int j = t; j < P; j += kThreads) th[j] = y1[j];
      ss = ss1;
      prior = pr1;
      nacc += 1;
    }
    TCI_PHASE(4)
    // ---- stage 2 (k_accept2)
    bool acc2 = false;
    if (!acc && inb2) {
      nev += 1;
      const double pr2 = prior_lds(y2, mu, sg, P, red);
      const double a32 = fmin(1.0, exp(-0.5 * (ss1 - ss2) / s2 - 0.5 * (pr1 - pr2)));
      const double l2 = exp(-0.5 * (ss2 - ss) / s2 - 0.5 * (pr2 - prior));
      for (int j = t; j < P; j += kThreads) {
        d1[j] = y2[j] - y1[j];
        d0[j] = th[j] - y1[j];
      }
      __syncthreads();
      tri_vecmat<2>(d1, d0, iRm, ld, P, part, z, y, L);
      double q21 = 0.0, q01 = 0.0;
      for (int j = t; j < P; j += kThreads) {
        q21 += z[j] * z[j];
        q01 += y[j] * y[j];
      }
      q21 = block_sum(q21, red);
      q01 = block_sum(q01, red);
      const double q1 = exp(-0.5 * (q21 - q01));
      const double a13 = l2 * q1 * (1.0 - a32) / (1.0 - a12);
      acc2 = uniform_at(p.seed, c, step, P_U2) < a13;
      if (acc2) {
        for (int j = t; j < P; j += kThreads) th[j] = y2[j];
        ss = ss2;
        prior = pr2;
        nacc += 1;
      }
    }
    TCI_PHASE(5)
    if (!(acc || acc2)) nrej += 1;
    if (p.updatesigma) s2 = 1.0 / gamma_at(p.seed, c, step, half_nobs, 2.0 / ss);
    __syncthreads();
    TCI_PHASE(6)
    record_row(st, p, c, step, P, th, s2);
    __syncthreads();
    TCI_PHASE(7)
  }
#undef TCI_PHASE
  if (TCI_CHAIN_PROFILE && t == 0 && st.prof != nullptr)
    for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long*)&st.prof[k], (unsigned long long)ph[k]);
  for (int j = t; j < P; j += kThreads) st.theta[c * ld + j] = th[j];
  if (t == 0) {
    st.ss[c] = ss;
    st.prior[c] = prior;
    st.sigma2[c] = s2;
    st.naccept[c] = nacc;
    st.nrej_win[c] = nrej;
    st.nevals[c] = nev;
    if (c == 0) *st.step = s_end;  // k_adapt reads the row it follows
  }
}

template <int RPL, int NSEG>
int launch_chain_t(const DramState& st, const DramParams& p, const KParams& kp, int64_t s_begin, int64_t s_end,
                   hipStream_t stream) {
  const size_t lds = (size_t)chain_lds_doubles(st.ld) * sizeof(double);
  if (lds > 48 * 1024 &&
      hipFuncSetAttribute((const void*)k_chain<RPL, NSEG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return TCI_EHIP;
  hipLaunchKernelGGL((k_chain<RPL, NSEG>), dim3((unsigned)st.n_chains), dim3(kThreads), lds, stream, st, p, kp,
                     s_begin, s_end);
  return hipGetLastError() == hipSuccess ? TCI_OK : TCI_EHIP;
}

template <int RPL>
int launch_chain_r(const DramState& st, const DramParams& p, const KParams& kp, int64_t a, int64_t b, hipStream_t s) {
  switch (kp.n_seg) {
    case 1: return launch_chain_t<RPL, 1>(st, p, kp, a, b, s);
    case 2: return launch_chain_t<RPL, 2>(st, p, kp, a, b, s);
    case 3: return launch_chain_t<RPL, 3>(st, p, kp, a, b, s);
    case 4: return launch_chain_t<RPL, 4>(st, p, kp, a, b, s);
    default: return TCI_EINVAL;
  }
}


// Adaptation for chains whose packed covariance fits in LDS (P(P+1)/2 doubles; P <= 139 keeps
// two workgroups per CU). Thread t owns the packed upper-triangle entries e = t + 256 k of cov:
// covupd runs on them in registers (no index arithmetic, one barrier pair per window row), then
// an LDL'-form right-looking Cholesky on the packed triangle (one barrier per pivot; R rows are
// scaled by 1/sqrt(pivot) at the end) and the row-by-row triangular inverse.
template <int KMAX>
__global__ __launch_bounds__(kThreads) void k_adapt_packed(DramState st, DramParams p) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ int fail;
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t step = *st.step;
  if (c >= st.n_chains || p.adaptint <= 0 || step % p.adaptint != 0) return;  // uniform exit
  const int64_t ld = st.ld;
  const int P = st.npar[c];
  const int T = P * (P + 1) / 2;
  double* A = dyn;       // packed upper triangle, row i at off(i) = i*P - i*(i-1)/2
  double* dm = A + T;    // P
  double* dsq = dm + P;  // P
  double* xs = dsq + P;  // P
  double* cvg = st.cov + c * ld * ld;
  double* mu = st.cmean + c * ld;
  double* R = st.R + c * ld * ld;
  double* iR = st.iR + c * ld * ld;
  auto off = [P](int i) { return i * P - (i * (i - 1)) / 2; };
  // ---- the owned entries (i, j), walking the packed order from e = t in strides of 256
  int own[KMAX];
  double a[KMAX];
  {
    int i = 0, j = t;
    while (i < P && j >= P) {
      j = j - P + i + 1;
      ++i;
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const bool v = i < P;
      own[k] = v ? (i << 16) | j : -1;
      a[k] = v ? cvg[(int64_t)i * ld + j] : 0.0;
      j += kThreads;
      while (i < P && j >= P) {
        j = j - P + i + 1;
        ++i;
      }
    }
  }
  // ---- covupd over the window rows (chain rows step-adaptint+1 .. step), mcmcstat's recurrence
  double ws = st.wsum[c];
  double mu0 = t < P ? mu[t] : 0.0, mu1 = t + kThreads < P ? mu[t + kThreads] : 0.0;
  for (int64_t r = 0; r < p.adaptint; ++r) {
    const double* x = st.window + (c * p.adaptint + r) * ld;
    if (ws == 0.0) {  // first row: mean = x, cov = 0
      if (t < P) mu0 = x[t];
      if (t + kThreads < P) mu1 = x[t + kThreads];
      ws = 1.0;
      continue;
    }
    const double d0 = t < P ? x[t] - mu0 : 0.0, d1 = t + kThreads < P ? x[t + kThreads] - mu1 : 0.0;
    if (t < P) dm[t] = d0;
    if (t + kThreads < P) dm[t + kThreads] = d1;
    __syncthreads();
    // xcov = oldcov + w/(w+oldwsum-1) * (oldwsum/(w+oldwsum) * d'd - oldcov), w = 1
    const double f1 = 1.0 / ws, f2 = ws / (ws + 1.0);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (own[k] >= 0) {
        const int i = own[k] >> 16, j = own[k] & 0xFFFF;
        a[k] = a[k] + f1 * (f2 * dm[i] * dm[j] - a[k]);
      }
    }
    mu0 = mu0 + d0 / (ws + 1.0);
    mu1 = mu1 + d1 / (ws + 1.0);
    ws += 1.0;
    __syncthreads();  // dm is rewritten by the next row
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (own[k] >= 0) cvg[(int64_t)(own[k] >> 16) * ld + (own[k] & 0xFFFF)] = a[k];
  }
  if (t < P) mu[t] = mu0;
  if (t + kThreads < P) mu[t + kThreads] = mu1;
  if (t == 0) st.wsum[c] = ws;
  if (step < p.burnintime) {
    // burn-in: no covariance adaptation, only scaling by the window's rejection rate
    const double rate = (double)st.nrej_win[c] / (double)p.adaptint;
    double s = 1.0;
    if (rate > 0.95) s = 1.0 / p.burnin_scale;
    else if (rate < 0.05) s = p.burnin_scale;
    if (s != 1.0) {
      for (int64_t e = t; e < (int64_t)P * P; e += kThreads) {
        const int i = (int)(e / P), j = (int)(e % P);
        R[(int64_t)i * ld + j] *= s;
        iR[(int64_t)i * ld + j] /= s;
      }
    }
    __syncthreads();
    if (t == 0) st.nrej_win[c] = 0;
    return;
  }
  // ---- Cholesky of cov + qcovadj*I: eliminate with unscaled pivot rows, A = U' D^-1 U
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (own[k] >= 0) {
      const int i = own[k] >> 16, j = own[k] & 0xFFFF;
      A[t + kThreads * k] = a[k] + (i == j ? p.qcovadj : 0.0);
    }
  }
  if (t == 0) fail = 0;
  __syncthreads();
  for (int k = 0; k < P; ++k) {
    const int ok = off(k);
    const double d = A[ok];
    if (!(d > 0.0) || !isfinite(d)) {  // uniform: every thread reads the same pivot
      if (t == 0) fail = 1;
      break;
    }
    const double inv = 1.0 / d;
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
      if (own[q] >= 0) {
        const int i = own[q] >> 16, j = own[q] & 0xFFFF;
        if (i > k) A[t + kThreads * q] -= A[ok + i - k] * A[ok + j - k] * inv;
      }
    }
    __syncthreads();
  }
  __syncthreads();
  if (!fail) {  // singular: keep the previous R (mcmcstat: "cmat singular, not adapting")
    const double sc = p.adascale > 0.0 ? p.adascale : 2.4 / sqrt((double)P);
    for (int i = t; i < P; i += kThreads) dsq[i] = sqrt(A[off(i)]);
    __syncthreads();
    // C = D^-1/2 U (upper, C'C = cov + qcovadj*I); R = C * adascale
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
      if (own[q] >= 0) {
        const int i = own[q] >> 16, j = own[q] & 0xFFFF;
        const double cij = A[t + kThreads * q] / dsq[i];
        A[t + kThreads * q] = cij;
        R[(int64_t)i * ld + j] = cij * sc;
      }
    }
    __syncthreads();
    // iR = C^-1 / adascale, in place, row by row from the bottom:
    // X(i,j) = (d_ij - sum_{k=i+1..j} C(i,k) X(k,j)) / C(i,i)
    for (int i = P - 1; i >= 0; --i) {
      const int oi = off(i);
      for (int k = i + t; k < P; k += kThreads) xs[k] = A[oi + k - i];
      __syncthreads();
      for (int j = i + t; j < P; j += kThreads) {
        double s = (i == j) ? 1.0 : 0.0;
        for (int k = i + 1; k <= j; ++k) s -= xs[k] * A[off(k) + j - k];
        A[oi + j - i] = s / xs[i];
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
      if (own[q] >= 0) {
        const int i = own[q] >> 16, j = own[q] & 0xFFFF;
        iR[(int64_t)i * ld + j] = A[t + kThreads * q] / sc;
      }
    }
  }
  __syncthreads();
  if (t == 0) st.nrej_win[c] = 0;
}

// Packed-adaptation bound: KMAX entries per thread and the LDS triangle + 3 vectors.
constexpr int kAdaptKmax = 40;
__host__ __device__ inline int64_t adapt_packed_lds_bytes(int64_t P) { return (P * (P + 1) / 2 + 3 * P) * 8; }

inline int finish() { return hipGetLastError() == hipSuccess ? TCI_OK : TCI_EHIP; }
inline dim3 chain_grid(int64_t n) { return dim3((unsigned)n); }

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
  hipLaunchKernelGGL(k_propose1, chain_grid(st.n_chains), dim3(kThreads), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_accept1(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_accept1, chain_grid(st.n_chains), dim3(kThreads), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_accept2(const DramState& st, const DramParams& p, void* stream) {
  hipLaunchKernelGGL(k_accept2, chain_grid(st.n_chains), dim3(kThreads), 0, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_adapt(const DramState& st, const DramParams& p, void* stream) {
  if (p.pmax * (p.pmax + 1) / 2 <= (int64_t)kAdaptKmax * kThreads && adapt_packed_lds_bytes(p.pmax) <= 78 * 1024) {
    const size_t bytes = (size_t)adapt_packed_lds_bytes(p.pmax);
    if (bytes > 48 * 1024 &&
        hipFuncSetAttribute((const void*)k_adapt_packed<kAdaptKmax>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes) != hipSuccess)
      return TCI_EHIP;
    hipLaunchKernelGGL(k_adapt_packed<kAdaptKmax>, chain_grid(st.n_chains), dim3(kThreads), bytes,
                       (hipStream_t)stream, st, p);
    return finish();
  }
  const size_t lds = p.lds_matrix ? (size_t)p.lds_matrix : 0;
  if (lds > 0 && hipFuncSetAttribute((const void*)k_adapt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
                     hipSuccess)
    return TCI_EHIP;
  hipLaunchKernelGGL(k_adapt, chain_grid(st.n_chains), dim3(kThreads), lds, (hipStream_t)stream, st, p);
  return finish();
}
int dram_launch_chain(const DramState& st, const DramParams& p, const KParams& kp, int rpl, int64_t s_begin,
                      int64_t s_end, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (rpl) {
    case 1: return launch_chain_r<1>(st, p, kp, s_begin, s_end, s);
    case 2: return launch_chain_r<2>(st, p, kp, s_begin, s_end, s);
    case 4: return launch_chain_r<4>(st, p, kp, s_begin, s_end, s);
    case 8: return launch_chain_r<8>(st, p, kp, s_begin, s_end, s);
    default: return TCI_EINVAL;
  }
}
int64_t dram_chain_lds_bytes(int64_t ld, int rpl) {
  return chain_lds_doubles(ld) * 8 + 2 * (4 * 64 * rpl + 4 * rpl) * 8 + 64;
}
int dram_launch_step_incr(const DramState& st, void* stream) {
  hipLaunchKernelGGL(k_step_incr, dim3(1), dim3(64), 0, (hipStream_t)stream, st.step);
  return finish();
}

}  // namespace tci
