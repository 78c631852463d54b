/*
 * tci_oracle.c -- CPU oracle (C restatement) of the reference likelihood hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Restates, in the reference's matrix form (the full time x polymerase
 * position matrix is materialised, as MATLAB does):
 *   SumofSquaresFunction_TranscriptionCycleMCMC.m:1-64   (grid, unpack, SS)
 *   dependencies/ConstantElongationSim.m:1-67             (Pol II positions)
 *   GetFluorFromPolPos.m:1-71                             (MS2/PP7 maps)
 * and the MATLAB builtins colon / mean / interp1(linear) / nansum.
 *
 * Build with -ffp-contract=off (oracle/Makefile): MATLAB never fuses a
 * multiply into an add, and floor(counter) plus the strict position masks are
 * discontinuous, so the operation order must be MATLAB's.
 *
 * Parallelism: OpenMP over evaluations -- the analogue of the reference's
 * parfor over cells (TranscriptionCycleMCMC.m:161).
 *
 * Pinned by the reference's own known-answer vectors (MCMCplot.simMS2/simPP7
 * at MCMCresults.mean_*, see tests/test_oracle_golden.py) -- bit-exact.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_OK 0
#define OR_EDIM -1   /* "Matrix dimensions must agree" (ConstantElongationSim.m:47) */
#define OR_EIDX -2   /* "Index exceeds matrix dimensions" (ConstantElongationSim.m:64) */
#define OR_EARG -3
#define OR_ENOMEM -4

#include "tci_oracle.h"

static double round_half_away(double x) { return x >= 0 ? floor(x + 0.5) : -floor(-x + 0.5); }

/* MATLAB colon a:d:b (colonop). Writes at most cap points; returns count or -1. */
static int64_t matlab_colon(double a, double d, double b, double *v, int64_t cap) {
  if (!isfinite(a) || !isfinite(d) || !isfinite(b)) {
    if (cap < 1) return -1;
    v[0] = NAN;
    return 1;
  }
  if (d == 0 || (a < b && d < 0) || (b < a && d > 0)) return 0;
  double tol = 2.0 * 2.220446049250313e-16 * fmax(fabs(a), fabs(b));
  double sig = d > 0 ? 1.0 : -1.0;
  double n;
  if (a == floor(a) && d == 1) {
    n = floor(b) - a;
  } else if (a == floor(a) && d == floor(d)) {
    double q = floor(a / d);
    double r = a - q * d;
    n = floor((b - r) / d) - q;
  } else {
    n = round_half_away((b - a) / d);
    if (sig * (a + n * d - b) > tol) n = n - 1;
  }
  int64_t ni = (int64_t)n;
  if (ni + 1 > cap) return -1;
  double c = a + n * d;
  if (sig * (c - b) > -tol) c = b;
  for (int64_t k = 0; k <= ni / 2; ++k) {
    double kd = (double)k;
    v[k] = a + kd * d;
    v[ni - k] = c - kd * d;
  }
  if (ni % 2 == 0) v[ni / 2] = (a + c) / 2;
  return ni + 1;
}

/* SumofSquares...m:29-30 : dt = mean(diff(t)); t_interp = t(1):dt:t(end). */
static int64_t interp_grid(const double *t, int64_t N, double *ti, int64_t cap) {
  double s = 0.0;
  for (int64_t i = 0; i + 1 < N; ++i) s = s + (t[i + 1] - t[i]);
  double dt = s / (double)(N - 1);
  return matlab_colon(t[0], dt, t[N - 1], ti, cap);
}

/* ConstantElongationSim(v,ton,R,t) into a row-major m x ncol matrix x.
 * R has m entries (R_full); R(1:end-1) is used. Returns ncol (>=0) or error. */
static int64_t elongation_sim(double v, double ton, const double *R, const double *t, int64_t m,
                              double **xbuf, int64_t *xcap) {
  if (m < 1) return OR_EARG;
  double *Rc = (double *)malloc(sizeof(double) * (size_t)(m > 1 ? m - 1 : 1));
  double *dt = (double *)malloc(sizeof(double) * (size_t)(m > 1 ? m - 1 : 1));
  if (!Rc || !dt) { free(Rc); free(dt); return OR_ENOMEM; }
  for (int64_t i = 0; i + 1 < m; ++i) {
    Rc[i] = R[i];                     /* :33 */
    if (Rc[i] < 0) Rc[i] = 0;         /* :36 */
    dt[i] = t[i + 1] - t[i];          /* :42-45 */
  }
  double s = 0.0;
  for (int64_t i = 0; i + 1 < m; ++i) s = s + Rc[i] * dt[i];
  int64_t n = isfinite(s) && s > 0 ? (int64_t)floor(s) : 0;   /* :47 */
  size_t need = (size_t)m * (size_t)(n > 0 ? n : 1);
  if ((int64_t)need > *xcap) {
    free(*xbuf);
    *xbuf = (double *)malloc(sizeof(double) * need);
    if (!*xbuf) { *xcap = 0; free(Rc); free(dt); return OR_ENOMEM; }
    *xcap = (int64_t)need;
  }
  double *x = *xbuf;
  memset(x, 0, sizeof(double) * (size_t)m * (size_t)n);        /* :50 */
  double counter = 0.0;                                        /* :53 */
  int64_t rc = n;
  for (int64_t i = 0; i + 1 < m; ++i) {                        /* :56 */
    if (t[i] < ton) continue;                                  /* :57 */
    double inc = Rc[i] * dt[i];
    counter = counter + inc;                                   /* :60 */
    double fk = floor(counter);                                /* :61 */
    if (!(fk >= 1)) continue;                                  /* 1:0 or 1:NaN is empty */
    int64_t K = (int64_t)fk;
    if (K > n) { rc = OR_EIDX; break; }                        /* x(i,k) reads past column n */
    double vd = v * dt[i];
    double *xi = x + (size_t)i * (size_t)n, *xo = x + (size_t)(i + 1) * (size_t)n;
    int any_neg = 0;
    for (int64_t k = 0; k < K; ++k) {                          /* :64 */
      xo[k] = xi[k] + vd;
      any_neg |= xo[k] < 0;
    }
    if (any_neg) {
      /* :65  x(x(i+1,k)<0)=0 -- the length-K row mask is a LINEAR (column-major)
       * index into x: element q -> row q % m, column q / m. Mask first, then assign. */
      char *mask = (char *)malloc((size_t)K);
      for (int64_t k = 0; k < K; ++k) mask[k] = xo[k] < 0;
      for (int64_t q = 0; q < K; ++q)
        if (mask[q]) x[(size_t)(q % m) * (size_t)n + (size_t)(q / m)] = 0;
      free(mask);
    }
  }
  free(Rc);
  free(dt);
  return rc;
}

/* GetFluorFromPolPos(construct,PolPos,v,tau,MS2_basal,PP7_basal) -> MS2[m], PP7[m]. */
static void fluor_from_polpos(const or_construct *cs, const double *x, int64_t m, int64_t n, double v,
                              double tau, double b1, double b2, double *MS2, double *PP7) {
  double L = cs->L0 + tau * v;                                  /* :19-20 */
  for (int64_t r = 0; r < m; ++r) { MS2[r] = 0; PP7[r] = 0; }   /* :29-30 */
  for (int32_t s = 0; s < cs->n_seg; ++s) {                     /* :47 */
    for (int dye = 0; dye < 2; ++dye) {
      double a = dye ? cs->pp7_start[s] : cs->ms2_start[s];
      double e = dye ? cs->pp7_end[s] : cs->ms2_end[s];
      double fv = (dye ? cs->pp7_loopn[s] : cs->ms2_loopn[s]) / 24;   /* :48 / :60 */
      double basal = dye ? b2 : b1;
      double *out = dye ? PP7 : MS2;
      for (int64_t r = 0; r < m; ++r) {
        const double *row = x + (size_t)r * (size_t)n;
        double acc = 0.0;
        for (int64_t k = 0; k < n; ++k) {                       /* sum(map,2), column order */
          double p = row[k], val = 0.0;
          if (p > e && p < L) val = fv;                         /* :50 / :62 */
          if (p > a && p < e) val = (p - a) * fv / (e - a);     /* :51-52 / :63-64 */
          acc = acc + val;
        }
        out[r] = out[r] + acc;                                  /* :54 / :66 */
        if (out[r] < basal) out[r] = basal;                     /* :57 / :69 */
      }
    }
  }
}

/* interp1(x, y, xq) linear; NaN outside [x(1), x(end)]. */
static double interp1_linear(const double *x, const double *y, int64_t M, double q) {
  if (!(q >= x[0] && q <= x[M - 1])) return NAN;
  int64_t lo = 0, hi = M;                                       /* last k with x[k] <= q */
  while (hi - lo > 1) {
    int64_t mid = (lo + hi) / 2;
    if (x[mid] <= q) lo = mid; else hi = mid;
  }
  int64_t k = lo;
  if (k > M - 2) k = M - 2;
  if (k < 0) k = 0;
  double s = (q - x[k]) / (x[k + 1] - x[k]);
  return y[k] + s * (y[k + 1] - y[k]);
}

typedef struct {
  double *x; int64_t xcap;
  double *ti, *ms2, *pp7;
  int64_t cap;
} scratch;

static int scratch_init(scratch *w, int64_t cap) {
  memset(w, 0, sizeof(*w));
  w->cap = cap;
  w->ti = (double *)malloc(sizeof(double) * (size_t)cap);
  w->ms2 = (double *)malloc(sizeof(double) * (size_t)cap);
  w->pp7 = (double *)malloc(sizeof(double) * (size_t)cap);
  return (w->ti && w->ms2 && w->pp7) ? OR_OK : OR_ENOMEM;
}
static void scratch_free(scratch *w) { free(w->x); free(w->ti); free(w->ms2); free(w->pp7); }

/* One SS evaluation: SumofSquaresFunction_TranscriptionCycleMCMC(construct,data,x). */
static int ss_one(const or_construct *cs, const double *t, const double *y1, const double *y2, int64_t N,
                  const double *th, scratch *w, double *ss_out) {
  if (N < 2) return OR_EARG;
  int64_t M = interp_grid(t, N, w->ti, w->cap);                 /* :28-30 */
  if (M < 0) return OR_EARG;
  if (M != N) return OR_EDIM;       /* R.*dt would not conform (ConstantElongationSim.m:47) */
  double v = th[0], tau = th[1], ton = th[2], b1 = th[3], b2 = th[4], A = th[5], R = th[6];
  double *Rf = w->pp7;              /* reuse as R_full scratch before PP7 is produced */
  for (int64_t i = 0; i < N; ++i) Rf[i] = R + th[7 + i];         /* :45 */
  int64_t n = elongation_sim(v, ton, Rf, w->ti, M, &w->x, &w->xcap);   /* :49 */
  if (n < 0) return (int)n;
  fluor_from_polpos(cs, w->x, M, n, v, tau, b1, b2, w->ms2, w->pp7);   /* :50 */
  for (int64_t r = 0; r < M; ++r) w->ms2[r] = A * w->ms2[r];          /* :51 */
  double ss = 0.0;
  for (int dye = 0; dye < 2; ++dye) {                                   /* :55-64 */
    const double *ys = dye ? w->pp7 : w->ms2;
    const double *ye = dye ? y2 : y1;
    for (int64_t j = 0; j < N; ++j) {
      double r = ye[j] - interp1_linear(w->ti, ys, M, t[j]);
      double r2 = r * r;
      if (r2 == r2) ss = ss + r2;                                       /* nansum */
    }
  }
  *ss_out = ss;
  return OR_OK;
}

/* One SS evaluation with caller-held scratch (the DRAM restatement's ssfun, oracle/tci_dram_oracle.c). */
void *oracle_scratch_new(int64_t cap) {
  scratch *w = (scratch *)malloc(sizeof(scratch));
  if (!w) return NULL;
  if (scratch_init(w, cap) != OR_OK) { scratch_free(w); free(w); return NULL; }
  return w;
}
void oracle_scratch_free(void *w) {
  if (w) { scratch_free((scratch *)w); free(w); }
}
int oracle_ss_one(const or_construct *cs, const double *t, const double *y1, const double *y2, int64_t N,
                  const double *th, void *w, double *ss_out) {
  return ss_one(cs, t, y1, y2, N, th, (scratch *)w, ss_out);
}

/* Batched SS: ss_out[b] = ssfun(theta[b,:], cell[cell_id[b]]); inactive rows get +Inf.
 * status_out[b] (optional) receives the per-row status (0 ok, <0 reference error). */
int oracle_ss_batch(const int64_t *offsets, const double *t, const double *ms2, const double *pp7,
                    int64_t n_cells, const or_construct *cs, const double *theta, int64_t ld_theta,
                    const int32_t *cell_id, const uint8_t *active, int64_t B, double *ss_out,
                    int32_t *status_out, int nthreads) {
  if (!offsets || !t || !theta || !cell_id || !ss_out || !cs || B < 0) return OR_EARG;
  int64_t nmax = 0;
  for (int64_t c = 0; c < n_cells; ++c) {
    int64_t N = offsets[c + 1] - offsets[c];
    if (N > nmax) nmax = N;
  }
  int err = OR_OK;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(min : err)
#endif
  {
    scratch w;
    int ok = scratch_init(&w, nmax + 8);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
    for (int64_t b = 0; b < B; ++b) {
      int32_t st = OR_OK;
      double ss = INFINITY;
      int32_t c = cell_id[b];
      if (ok != OR_OK) st = OR_ENOMEM;
      else if (c < 0 || c >= n_cells) st = OR_EARG;
      else if (!active || active[b]) {
        int64_t o = offsets[c], N = offsets[c + 1] - o;
        if (ld_theta < 7 + N) st = OR_EARG;
        else st = ss_one(cs, t + o, ms2 + o, pp7 + o, N, theta + (size_t)b * (size_t)ld_theta, &w, &ss);
        if (st != OR_OK) ss = NAN;
      }
      ss_out[b] = ss;
      if (status_out) status_out[b] = st;
      if (st < err) err = st;
    }
    scratch_free(&w);
  }
  return err;
}

/* Forward model for one theta on the raw times (mode 0, TranscriptionCycleMCMC.m:307-309)
 * or through the uniform grid + interp1 (mode 1, SumofSquares...m:28-56). */
int oracle_forward(const double *t, int64_t N, const or_construct *cs, const double *th, int mode,
                   double *ms2_out, double *pp7_out) {
  if (N < 2) return OR_EARG;
  scratch w;
  if (scratch_init(&w, N + 8) != OR_OK) { scratch_free(&w); return OR_ENOMEM; }
  const double *grid = t;
  int64_t M = N;
  if (mode == 1) {
    M = interp_grid(t, N, w.ti, w.cap);
    if (M != N) { scratch_free(&w); return OR_EDIM; }
    grid = w.ti;
  }
  double *Rf = (double *)malloc(sizeof(double) * (size_t)N);
  for (int64_t i = 0; i < N; ++i) Rf[i] = th[6] + th[7 + i];
  int64_t n = elongation_sim(th[0], th[2], Rf, grid, M, &w.x, &w.xcap);
  free(Rf);
  if (n < 0) { scratch_free(&w); return (int)n; }
  fluor_from_polpos(cs, w.x, M, n, th[0], th[1], th[3], th[4], w.ms2, w.pp7);
  for (int64_t r = 0; r < M; ++r) w.ms2[r] = th[5] * w.ms2[r];
  for (int64_t j = 0; j < N; ++j) {
    if (mode == 1) {
      ms2_out[j] = interp1_linear(w.ti, w.ms2, M, t[j]);
      pp7_out[j] = interp1_linear(w.ti, w.pp7, M, t[j]);
    } else {
      ms2_out[j] = w.ms2[j];
      pp7_out[j] = w.pp7[j];
    }
  }
  scratch_free(&w);
  return OR_OK;
}

/* Interpolation grid as the reference builds it (for grid tests). Returns M or <0. */
int64_t oracle_interp_grid(const double *t, int64_t N, double *ti_out, int64_t cap) {
  if (N < 2) return OR_EARG;
  return interp_grid(t, N, ti_out, cap);
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
