/*
 * tci_dram_oracle.c -- CPU restatement of the reference's sampler call (TEST INFRASTRUCTURE ONLY:
 * loaded by tests/ and bench.py's cpu_baseline legs, never by the product).
 *
 * mcmcrun(model, data, params, options) as TranscriptionCycleMCMC.m:263-273 calls it -- one chain,
 * step by step, with the C oracle (tci_oracle.c) as model.ssfun -- restating mcmcstat's published
 * DRAM (Haario, Laine, Mira & Saksman 2006; github.com/mjlaine/mcmcstat mcmcrun.m / covupd.m,
 * version unpinned, not vendored: README.md:5) in its own MATLAB form:
 *   stage 1   newpar = oldpar + randn(1,npar)*R; out of bounds -> rejected without ssfun;
 *             alpha12 = min(1, exp(-0.5*(newss-oldss)/sigma2 - 0.5*(newprior-oldprior)))
 *   stage 2   newpar2 = oldpar + randn(1,npar)*(R./drscale)
 *             alpha32 = min(1, exp(-0.5*(newss-newss2)/sigma2 - 0.5*(newprior-newprior2)))
 *             l2 = exp(-0.5*(newss2-oldss)/sigma2 - 0.5*(newprior2-oldprior))
 *             q1 = exp(-0.5*(|(newpar2-newpar) iR|^2 - |(oldpar-newpar) iR|^2))
 *                = exp(-0.5*(|z2/drscale - z1|^2 - |z1|^2))     (exact algebra, no iR)
 *             alpha13 = l2*q1*(1-alpha32)/(1-alpha12)
 *   sigma2    1/sigma2 ~ Gamma(N/2, 2/oldss)  (N0 = 0, N = length(ydata) = 2 N_c, :260)
 *   adapt     every adaptint rows: before burnintime R./burnin_scale (rejection rate > 0.95) or
 *             R.*burnin_scale (< 0.05); afterwards covupd over the rows since the last update (all
 *             rows at the first one: the batch covariance, then covupd's row recurrence
 *             C = C + 1/(n-1) ((n-1)/n d d' - C), d = x - mean) and R = chol(C + qcovadj I) *
 *             2.4/sqrt(npar); a matrix that is not positive definite keeps R
 *   prior     sum(((theta - mu)./sig).^2) over finite sig (dR: N(0, 50), :254)
 *   summaries mean / std(., 1) of rows stats_from..end (:284-301), sqrt(mean(s2chain)) and
 *             std(sqrt(s2chain), 1) over every row (:302-303)
 * The random numbers are the GPU sampler's streams (Philox4x32-10 keyed by (seed), counter (chain
 * key, step, purpose, index); FP64 Box-Muller normals in the GPU's own arithmetic (bm_*), bit for
 * bit; Marsaglia-Tsang Gamma), so for the same
 * inputs this chain and the GPU's agree up to the rounding of the continuous arithmetic (the
 * GPU's SS summation order, its pairwise covariance merge, its Cholesky order): a GPU test checks
 * that (tests/test_dram_gpu.py), and bench.py times this restatement as config 1's CPU fit.
 *
 * Build: oracle/Makefile (-ffp-contract=off, as tci_oracle.c).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "tci_oracle.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

typedef struct {
  int64_t n_steps, burnintime, adaptint;
  int32_t ntry, updatesigma;
  double drscale, adascale, qcovadj, burnin_scale;
  int64_t stats_from;
  uint64_t seed;
} or_dram_opts;

typedef struct {
  double *mean, *std, *final_theta;               /* [n_chains][ld] */
  double *sigma_mean, *sigma_std, *accept_rate;   /* [n_chains] */
  int64_t *n_evals;                               /* [n_chains] */
  double *chain;                                  /* [n_steps][n_chains][ld] or NULL */
  double *s2chain;                                /* [n_steps][n_chains] or NULL */
  double *R;                                      /* [n_chains][ld][ld] final proposal factor or NULL */
} or_dram_out;

enum { P_NORM1 = 1, P_U1 = 2, P_NORM2 = 3, P_U2 = 4, P_GAMMA = 5 };

/* ---- Philox4x32-10 (Salmon, Moraes, Dror & Shaw 2011), the GPU sampler's generator */
typedef struct { uint32_t x, y, z, w; } u32x4;

u32x4 oracle_philox(u32x4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u32x4 n = {hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

static u32x4 rng(uint64_t seed, int64_t chain, int64_t step, uint32_t purpose, uint32_t idx) {
  u32x4 c = {(uint32_t)chain, (uint32_t)step, ((uint32_t)(step >> 32) & 0x00FFFFFFu) | (purpose << 24), idx};
  return oracle_philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

/* uniform in (0,1) from 64 bits: 53-bit mantissa, never 0 or 1 */
static double u01(uint32_t a, uint32_t b) {
  const uint64_t x = (((uint64_t)a << 32) | b) >> 11;
  return ((double)x + 0.5) * 0x1p-53;
}

/* Box-Muller's transcendental pair as the GPU computes it (csrc/tci_dram.hip bm_neg2log,
 * bm_sincospi): correctly rounded +, *, /, sqrt and fma only, operation for operation, so the
 * normals are the GPU's bits. -2 log(u): u = m 2^e, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s),
 * s = (m - 1)/(m + 1), the odd series to s^19; e ln 2 as fdlibm's ln2_hi + ln2_lo. */
double bm_neg2log(double u) {
  int e;
  double m = frexp(u, &e); /* [1/2, 1) */
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
  const double lm = fma(sv * z, q, sv);
  const double de = (double)e;
  return -2.0 * (de * 6.93147180369123816490e-01 + (2.0 * lm + de * 1.90821492927058770002e-10));
}

/* sin(pi x), cos(pi x), x in (0, 2): t = 2x quarter turns, r = t - rint(t) (exact), the Taylor
 * series of sin / cos((pi/2) r) to r^17 / r^16, then the quadrant */
void bm_sincospi(double x, double *sn, double *cs) {
  const double t = 2.0 * x;
  const double n = rint(t);
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
  const double a = (k & 1) ? cp : sp, b = (k & 1) ? sp : cp;
  *sn = (k & 2) ? -a : a;
  *cs = ((k + 1) & 2) ? -b : b;
}

/* z[0..P) of stream (chain, step, purpose): Box-Muller, 2 normals per Philox call */
static void normals(uint64_t seed, int64_t key, int64_t step, uint32_t purpose, int P, double *z) {
  for (int q = 0; 2 * q < P; ++q) {
    const u32x4 r = rng(seed, key, step, purpose, (uint32_t)q);
    const double rad = sqrt(bm_neg2log(u01(r.x, r.y)));
    double sn, cs;
    bm_sincospi(2.0 * u01(r.z, r.w), &sn, &cs);
    z[2 * q] = rad * cs;
    if (2 * q + 1 < P) z[2 * q + 1] = rad * sn;
  }
}

static double uniform(uint64_t seed, int64_t key, int64_t step, uint32_t purpose) {
  const u32x4 r = rng(seed, key, step, purpose, 0);
  return u01(r.x, r.y);
}

/* Gamma(a, 1), a >= 1: Marsaglia & Tsang (2000) */
static double gamma_unit(uint64_t seed, int64_t key, int64_t step, double a) {
  const double d = a - 1.0 / 3.0, cc = 1.0 / sqrt(9.0 * d);
  for (uint32_t it = 0; it < 1024; ++it) {
    const u32x4 r = rng(seed, key, step, P_GAMMA, it);
    const double x = sqrt(-2.0 * log(u01(r.x, r.y))) * cos(2.0 * M_PI * u01(r.z, r.w));
    const u32x4 r2 = rng(seed, key, step, P_GAMMA, it | 0x80000000u);
    const double u = u01(r2.x, r2.y);
    double v = 1.0 + cc * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double x2 = x * x;
    if (u < 1.0 - 0.0331 * x2 * x2) return d * v;
    if (log(u) < 0.5 * x2 + d - d * v + d * log(v)) return d * v;
  }
  return a;
}

/* sum(((th - mu)./sig).^2) over finite sig (mcmcstat's default priorfun) */
static double prior(const double *th, const double *mu, const double *sig, int P) {
  double s = 0.0;
  for (int j = 0; j < P; ++j)
    if (isfinite(sig[j])) {
      const double z = (th[j] - mu[j]) / sig[j];
      s = s + z * z;
    }
  return s;
}

/* upper Cholesky A = U'U (MATLAB chol), row-major P x P; returns 0, or 1 if A is not positive
 * definite (U untouched then) */
static int chol_upper(const double *A, int P, int ld, double *U, double *work) {
  for (int i = 0; i < P * P; ++i) work[i] = 0.0;
  for (int j = 0; j < P; ++j) {
    double s = A[j * ld + j];
    for (int k = 0; k < j; ++k) s = s - work[k * P + j] * work[k * P + j];
    if (!(s > 0.0) || !isfinite(s)) return 1;
    const double rjj = sqrt(s);
    work[j * P + j] = rjj;
    for (int i = j + 1; i < P; ++i) {
      double t = A[j * ld + i];
      for (int k = 0; k < j; ++k) t = t - work[k * P + j] * work[k * P + i];
      work[j * P + i] = t / rjj;
    }
  }
  for (int i = 0; i < P; ++i)
    for (int j = 0; j < P; ++j) U[i * ld + j] = work[i * P + j];
  return 0;
}

typedef struct {
  double *th, *y1, *y2, *z1, *z2, *R, *R2, *cov, *cmean, *A, *work, *rows, *smean, *sm2, *d;
} chain_ws;

static void ws_free(chain_ws *w) {
  free(w->th); free(w->y1); free(w->y2); free(w->z1); free(w->z2); free(w->R); free(w->R2); free(w->cov);
  free(w->cmean); free(w->A); free(w->work); free(w->rows); free(w->smean); free(w->sm2); free(w->d);
}

static int run_chain(const int64_t *offsets, const double *t, const double *ms2, const double *pp7,
                     const or_construct *cs, int64_t c, int64_t n_chains, int32_t cell, int64_t key,
                     const double *x0, const double *lo, const double *hi, const double *mu, const double *sig,
                     const double *qd, double s2, int64_t ld, const or_dram_opts *o, or_dram_out *out) {
  const int64_t off = offsets[cell], N = offsets[cell + 1] - off;
  const int P = (int)(7 + N);
  const double *tc = t + off, *y1c = ms2 + off, *y2c = pp7 + off;
  /* rows kept for covupd: every row up to the first adaptation at or after burnintime, adaptint after */
  const int64_t rows_cap = o->adaptint > 0 ? (o->burnintime > 0 ? o->burnintime : 0) + o->adaptint + 1 : 1;
  chain_ws w;
  memset(&w, 0, sizeof(w));
  const size_t PV = (size_t)P * sizeof(double), PP = (size_t)P * (size_t)P * sizeof(double);
  w.th = malloc(PV); w.y1 = malloc(PV); w.y2 = malloc(PV); w.z1 = malloc(PV); w.z2 = malloc(PV);
  w.R = calloc(1, PP); w.R2 = malloc(PP); w.cov = calloc(1, PP); w.cmean = calloc(1, PV); w.A = malloc(PP);
  w.work = malloc(PP); w.rows = malloc((size_t)rows_cap * PV); w.smean = calloc(1, PV); w.sm2 = calloc(1, PV);
  w.d = malloc(PV);
  void *sw = oracle_scratch_new(N + 8);
  if (!w.th || !w.y1 || !w.y2 || !w.z1 || !w.z2 || !w.R || !w.R2 || !w.cov || !w.cmean || !w.A || !w.work ||
      !w.rows || !w.smean || !w.sm2 || !w.d || !sw) {
    ws_free(&w);
    oracle_scratch_free(sw);
    return -4;
  }
  double *th = w.th, *R = w.R;
  memcpy(th, x0, PV);
  for (int j = 0; j < P; ++j) R[j * P + j] = sqrt(qd[j]);          /* R = chol(qcov), qcov = J0 (:230) */
  const double nobs = 2.0 * (double)N;                              /* model.N (:260), NaNs included */
  double ss, pr = prior(th, mu, sig, P);
  int rc = oracle_ss_one(cs, tc, y1c, y2c, N, th, sw, &ss);         /* the initial ssfun call */
  if (rc != 0) { ws_free(&w); oracle_scratch_free(sw); return rc; }
  int64_t nev = 1, nacc = 0, rej = 0, lasti = 0, nrows = 0;         /* rows: chain rows lasti+1 .. */
  double cw = 0.0;                                                  /* covupd's wsum (0: empty) */
  int64_t ns = 0;                                                   /* statistics rows so far */
  double s2n = 0.0, s2sum = 0.0, qmean = 0.0, qm2 = 0.0;
  const double inv_ds = 1.0 / o->drscale;
  /* row 1: the initial state */
  for (int64_t row = 1; row <= o->n_steps; ++row) {
    if (row >= 2) {
      const int64_t step = row;
      /* ---- stage 1 */
      normals(o->seed, key, step, P_NORM1, P, w.z1);
      int inb = 1;
      for (int j = 0; j < P; ++j) {
        double u = 0.0;
        for (int i = 0; i <= j; ++i) u = u + w.z1[i] * R[i * P + j];
        w.y1[j] = th[j] + u;
        inb &= (w.y1[j] >= lo[j] && w.y1[j] <= hi[j]);
      }
      double ss1 = INFINITY, pr1 = 0.0, a12 = 0.0;
      int acc = 0, moved = 0;
      if (inb) {
        if ((rc = oracle_ss_one(cs, tc, y1c, y2c, N, w.y1, sw, &ss1)) != 0) break;
        ++nev;
        pr1 = prior(w.y1, mu, sig, P);
        a12 = fmin(1.0, exp(-0.5 * (ss1 - ss) / s2 - 0.5 * (pr1 - pr)));
        acc = uniform(o->seed, key, step, P_U1) < a12;
      }
      if (acc) {
        memcpy(th, w.y1, PV);
        ss = ss1;
        pr = pr1;
        moved = 1;
      } else if (o->ntry >= 2) {
        /* ---- stage 2 (delayed rejection) with R2 = R ./ drscale */
        normals(o->seed, key, step, P_NORM2, P, w.z2);
        int inb2 = 1;
        for (int j = 0; j < P; ++j) {
          double u = 0.0;
          for (int i = 0; i <= j; ++i) u = u + w.z2[i] * (R[i * P + j] / o->drscale);
          w.y2[j] = th[j] + u;
          inb2 &= (w.y2[j] >= lo[j] && w.y2[j] <= hi[j]);
        }
        if (inb2) {
          double ss2;
          if ((rc = oracle_ss_one(cs, tc, y1c, y2c, N, w.y2, sw, &ss2)) != 0) break;
          ++nev;
          const double pr2 = prior(w.y2, mu, sig, P);
          const double a32 = fmin(1.0, exp(-0.5 * (ss1 - ss2) / s2 - 0.5 * (pr1 - pr2)));
          const double l2 = exp(-0.5 * (ss2 - ss) / s2 - 0.5 * (pr2 - pr));
          double q21 = 0.0, q01 = 0.0;
          for (int j = 0; j < P; ++j) {
            const double dz = w.z2[j] * inv_ds - w.z1[j];
            q21 = q21 + dz * dz;
            q01 = q01 + w.z1[j] * w.z1[j];
          }
          const double q1 = exp(-0.5 * (q21 - q01));
          const double a13 = l2 * q1 * (1.0 - a32) / (1.0 - a12);
          if (uniform(o->seed, key, step, P_U2) < a13) {
            memcpy(th, w.y2, PV);
            ss = ss2;
            pr = pr2;
            moved = 1;
          }
        }
      }
      if (moved) ++nacc;
      else ++rej;
      /* ---- sigma2 Gibbs update */
      if (o->updatesigma) s2 = 1.0 / (gamma_unit(o->seed, key, step, 0.5 * nobs) * (2.0 / ss));
    }
    /* ---- the row's records */
    if (out->chain) memcpy(out->chain + ((size_t)(row - 1) * (size_t)n_chains + (size_t)c) * (size_t)ld, th, PV);
    if (out->s2chain) out->s2chain[(size_t)(row - 1) * (size_t)n_chains + (size_t)c] = s2;
    if (row >= o->stats_from) {  /* Welford over rows stats_from..end */
      ++ns;
      for (int j = 0; j < P; ++j) {
        const double dm = th[j] - w.smean[j];
        w.smean[j] = w.smean[j] + dm / (double)ns;
        w.sm2[j] = w.sm2[j] + dm * (th[j] - w.smean[j]);
      }
    }
    s2n += 1.0;
    s2sum = s2sum + s2;
    {
      const double q = sqrt(s2), dq = q - qmean;
      qmean = qmean + dq / s2n;
      qm2 = qm2 + dq * (q - qmean);
    }
    if (o->adaptint > 0) {
      if (nrows < rows_cap) memcpy(w.rows + (size_t)nrows * (size_t)P, th, PV);
      ++nrows;
    }
    /* ---- adaptation after rows that are multiples of adaptint */
    if (row >= 2 && o->adaptint > 0 && row % o->adaptint == 0) {
      if (row < o->burnintime) {
        const double rate = (double)rej / (double)o->adaptint;
        if (rate > 0.95)
          for (int i = 0; i < P * P; ++i) R[i] = R[i] / o->burnin_scale;
        else if (rate < 0.05)
          for (int i = 0; i < P * P; ++i) R[i] = R[i] * o->burnin_scale;
      } else {
        /* covupd(chain((lasti+1):row, :), 1, cov, mean, wsum) */
        const int64_t n = row - lasti;
        if (n > rows_cap || nrows != n) { rc = -5; break; }
        const double *X = w.rows;
        if (cw == 0.0) {  /* first call: the batch's mean and covariance */
          for (int j = 0; j < P; ++j) {
            double s = 0.0;
            for (int64_t r = 0; r < n; ++r) s = s + X[r * P + j];
            w.cmean[j] = s / (double)n;
          }
          for (int i = 0; i < P; ++i)
            for (int j = i; j < P; ++j) {
              double s = 0.0;
              for (int64_t r = 0; r < n; ++r) s = s + (X[r * P + i] - w.cmean[i]) * (X[r * P + j] - w.cmean[j]);
              w.cov[i * P + j] = w.cov[j * P + i] = n > 1 ? s / (double)(n - 1) : 0.0;
            }
          cw = (double)n;
        } else {  /* the row recurrence */
          for (int64_t r = 0; r < n; ++r) {
            const double *x = X + r * P;
            const double nn = cw + 1.0;
            for (int j = 0; j < P; ++j) w.d[j] = x[j] - w.cmean[j];
            for (int i = 0; i < P; ++i)
              for (int j = i; j < P; ++j) {
                const double v = w.cov[i * P + j] + (1.0 / (nn - 1.0)) * ((cw / nn) * (w.d[i] * w.d[j]) - w.cov[i * P + j]);
                w.cov[i * P + j] = w.cov[j * P + i] = v;
              }
            for (int j = 0; j < P; ++j) w.cmean[j] = w.cmean[j] + (1.0 / nn) * w.d[j];
            cw = nn;
          }
        }
        lasti = row;
        nrows = 0;
        for (int i = 0; i < P; ++i)
          for (int j = 0; j < P; ++j) w.A[i * P + j] = w.cov[i * P + j] + (i == j ? o->qcovadj : 0.0);
        if (chol_upper(w.A, P, P, w.R2, w.work) == 0) {  /* singular: "cmat singular, not adapting" */
          const double sc = o->adascale > 0.0 ? o->adascale : 2.4 / sqrt((double)P);
          for (int i = 0; i < P * P; ++i) R[i] = w.R2[i] * sc;
        }
      }
      rej = 0;
    }
  }
  if (rc == 0) {
    for (int j = 0; j < P; ++j) {
      out->mean[c * ld + j] = ns > 0 ? w.smean[j] : NAN;
      out->std[c * ld + j] = ns > 0 ? sqrt(w.sm2[j] / (double)ns) : NAN;
      out->final_theta[c * ld + j] = th[j];
    }
    /* padding past the chain's P (include/tci.h, tci_dram_outputs): mean/std NaN, final_theta
     * the caller's theta0 padding, unchanged */
    for (int j = P; j < ld; ++j) {
      out->mean[c * ld + j] = out->std[c * ld + j] = NAN;
      out->final_theta[c * ld + j] = x0[j];
    }
    out->sigma_mean[c] = sqrt(s2sum / s2n);
    out->sigma_std[c] = sqrt(qm2 / s2n);
    out->accept_rate[c] = o->n_steps > 1 ? (double)nacc / (double)(o->n_steps - 1) : 0.0;
    out->n_evals[c] = nev;
    if (out->R) {
      double *Ro = out->R + (size_t)c * (size_t)ld * (size_t)ld;
      for (int64_t i = 0; i < ld * ld; ++i) Ro[i] = 0.0;
      for (int i = 0; i < P; ++i)
        for (int j = 0; j < P; ++j) Ro[i * ld + j] = R[i * P + j];
    }
  }
  ws_free(&w);
  oracle_scratch_free(sw);
  return rc;
}

/* One chain per row, chains in parallel (OpenMP over chains: the parfor, :161). Inputs as
 * tci_dram_run (include/tci.h): rows of ld doubles. keys: RNG stream key per chain (NULL: the
 * row index). Returns 0 or the first error (< 0). */
int oracle_dram_run(const int64_t *offsets, const double *t, const double *ms2, const double *pp7, int64_t n_cells,
                    const or_construct *cs, int64_t n_chains, const int32_t *cell_id, const int64_t *keys,
                    const double *theta0, const double *lower, const double *upper, const double *pmu,
                    const double *psig, const double *qcov_diag, const double *sigma2_0, int64_t ld,
                    const or_dram_opts *o, or_dram_out *out, int nthreads) {
  if (!offsets || !t || !ms2 || !pp7 || !cs || !cell_id || !theta0 || !lower || !upper || !pmu || !psig ||
      !qcov_diag || !sigma2_0 || !o || !out || !out->mean || !out->std || !out->final_theta || !out->sigma_mean ||
      !out->sigma_std || !out->accept_rate || !out->n_evals || o->n_steps < 1 || o->ntry < 1 || o->ntry > 2)
    return -3;
  for (int64_t c = 0; c < n_chains; ++c)
    if (cell_id[c] < 0 || cell_id[c] >= n_cells || 7 + offsets[cell_id[c] + 1] - offsets[cell_id[c]] > ld) return -3;
  int err = 0;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1) reduction(min : err)
#endif
  for (int64_t c = 0; c < n_chains; ++c) {
    const size_t r = (size_t)c * (size_t)ld;
    const int rc = run_chain(offsets, t, ms2, pp7, cs, c, n_chains, cell_id[c], keys ? keys[c] : c, theta0 + r,
                             lower + r, upper + r, pmu + r, psig + r, qcov_diag + r, sigma2_0[c], ld, o, out);
    if (rc < err) err = rc;
  }
  return err;
}
