// tci_api.cpp -- C ABI (include/tci.h): context, resident cell table, validation, launches.
//
// The context replaces the per-call work the reference repeats inside every ssfun call
// (SumofSquaresFunction_TranscriptionCycleMCMC.m:28-30: the grid, which is theta-independent)
// with a one-time build at tci_create, and keeps the cell table resident in HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <utility>
#include <string>
#include <vector>

#include "tci_diag.h"
#include "tci_dram_internal.h"
#include "tci_internal.h"

using tci::CellMeta;
using tci::KParams;

struct tci_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int rpl = 1;
  int64_t stride = 0;               // records per cell in the resident tables
  int64_t n_cells = 0;
  int64_t max_points = 0;
  int64_t device_bytes = 0;
  std::vector<CellMeta> meta;       // host copy
  std::vector<double> grid;         // host copy of t_interp (cell c at c * stride)
  KParams kp{};
  void* dbuf = nullptr;             // one allocation for the whole resident cell table
  // staging buffers for the host-pointer entry points
  double* d_theta = nullptr;
  int32_t* d_cell = nullptr;
  uint8_t* d_active = nullptr;
  double* d_out0 = nullptr;
  double* d_out1 = nullptr;
  size_t cap_theta = 0, cap_cell = 0, cap_active = 0, cap_out0 = 0, cap_out1 = 0;
  // small batches of the host-pointer entry points: one pinned, device-mapped buffer the kernel
  // reads and writes in place (no copy launches; tci_ss_batch)
  char* h_io = nullptr;
  char* d_io = nullptr;
  size_t cap_io = 0;
  std::string err;
};

namespace {

const char kVersion[] = "tci-mi355x 0.1.0 (gfx950)";

int fail(tci_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int hip_fail(tci_ctx* ctx, hipError_t e, const char* what) {
  return fail(ctx, TCI_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define TCI_HIP(ctx, call)                                  \
  do {                                                      \
    hipError_t e_ = (call);                                 \
    if (e_ != hipSuccess) return hip_fail((ctx), e_, #call); \
  } while (0)

double round_half_away(double x) { return x >= 0 ? std::floor(x + 0.5) : -std::floor(-x + 0.5); }

// MATLAB a:d:b by the documented colon algorithm (colonop): n from round((b-a)/d) with a
// 2*eps*max(|a|,|b|) tolerance, right end snapped to b, and the vector built symmetrically
// from both ends. Used for t_interp = t(1):dt:t(end) (SumofSquares...m:30).
std::vector<double> colon(double a, double d, double b) {
  if (!std::isfinite(a) || !std::isfinite(d) || !std::isfinite(b)) return {NAN};
  if (d == 0 || (a < b && d < 0) || (b < a && d > 0)) return {};
  const double tol = 2.0 * 2.220446049250313e-16 * std::max(std::fabs(a), std::fabs(b));
  const double sig = d > 0 ? 1.0 : -1.0;
  double n;
  if (a == std::floor(a) && d == 1) {
    n = std::floor(b) - a;
  } else if (a == std::floor(a) && d == std::floor(d)) {
    const double q = std::floor(a / d);
    const double r = a - q * d;
    n = std::floor((b - r) / d) - q;
  } else {
    n = round_half_away((b - a) / d);
    if (sig * (a + n * d - b) > tol) n = n - 1;
  }
  if (!(n >= 0) || n > 1e7) return {};
  const int64_t ni = (int64_t)n;
  double c = a + n * d;
  if (sig * (c - b) > -tol) c = b;
  std::vector<double> v((size_t)ni + 1);
  for (int64_t k = 0; k <= ni / 2; ++k) {
    const double kd = (double)k;
    v[(size_t)k] = a + kd * d;
    v[(size_t)(ni - k)] = c - kd * d;
  }
  if (ni % 2 == 0) v[(size_t)(ni / 2)] = (a + c) / 2;
  return v;
}

// dt = mean(t(2:end)-t(1:end-1)) (sequential sum / count), then the colon grid.
std::vector<double> interp_grid(const double* t, int64_t n, double* d_out) {
  double s = 0.0;
  for (int64_t i = 0; i + 1 < n; ++i) s = s + (t[i + 1] - t[i]);
  const double d = s / (double)(n - 1);
  if (d_out) *d_out = d;
  return colon(t[0], d, t[n - 1]);
}

template <typename T>
int ensure(tci_ctx* ctx, T** p, size_t* cap, size_t need) {
  if (need <= *cap) return TCI_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  size_t n = std::max(need, (size_t)1024);
  TCI_HIP(ctx, hipMalloc((void**)p, n * sizeof(T)));
  *cap = n;
  return TCI_OK;
}

// Bytes of theta + ids + flags + SS per call up to which tci_ss_batch works in place in pinned host
// memory (TCI_ZERO_COPY_MAX overrides; 0 disables).
size_t zero_copy_max() {
  static const size_t v = [] {
    const char* e = std::getenv("TCI_ZERO_COPY_MAX");
    return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)1024 * 1024;
  }();
  return v;
}

int ensure_io(tci_ctx* ctx, size_t need) {
  if (need <= ctx->cap_io) return TCI_OK;
  if (ctx->h_io) (void)hipHostFree(ctx->h_io);
  ctx->h_io = ctx->d_io = nullptr;
  ctx->cap_io = 0;
  const size_t n = std::max(need, (size_t)64 * 1024);
  TCI_HIP(ctx, hipHostMalloc((void**)&ctx->h_io, n, hipHostMallocMapped | hipHostMallocCoherent));
  TCI_HIP(ctx, hipHostGetDevicePointer((void**)&ctx->d_io, ctx->h_io, 0));
  ctx->cap_io = n;
  return TCI_OK;
}

int check_construct(tci_ctx* ctx, const tci_construct* cs) {
  if (!cs) return fail(ctx, TCI_EINVAL, "construct is NULL");
  if (cs->n_seg < 1 || cs->n_seg > TCI_MAX_SEG)
    return fail(ctx, TCI_EINVAL, "construct n_seg must be in [1, " + std::to_string(TCI_MAX_SEG) + "]");
  if (!cs->ms2_start || !cs->ms2_end || !cs->ms2_loopn || !cs->pp7_start || !cs->pp7_end || !cs->pp7_loopn)
    return fail(ctx, TCI_EINVAL, "construct segment arrays must not be NULL");
  if (!std::isfinite(cs->L0)) return fail(ctx, TCI_EINVAL, "construct L0 must be finite");
  for (int s = 0; s < cs->n_seg; ++s) {
    const double vals[6] = {cs->ms2_start[s], cs->ms2_end[s], cs->ms2_loopn[s],
                            cs->pp7_start[s], cs->pp7_end[s], cs->pp7_loopn[s]};
    for (double x : vals)
      if (!std::isfinite(x)) return fail(ctx, TCI_EINVAL, "construct values must be finite");
    if (!(cs->ms2_start[s] >= 0 && cs->ms2_start[s] < cs->ms2_end[s] && cs->pp7_start[s] >= 0 &&
          cs->pp7_start[s] < cs->pp7_end[s]))
      return fail(ctx, TCI_EINVAL, "construct segment " + std::to_string(s) + " needs 0 <= start < end");
  }
  return TCI_OK;
}

void fill_segments(KParams* kp, const tci_construct* cs) {
  kp->L0 = cs->L0;
  kp->n_seg = cs->n_seg;
  double emax = 0.0;
  for (int s = 0; s < cs->n_seg; ++s) {
    tci::SegParams m, p;
    m.a = cs->ms2_start[s];
    m.e = cs->ms2_end[s];
    m.phi = cs->ms2_loopn[s] / 24;  // GetFluorFromPolPos.m:48
    m.k = m.phi / (m.e - m.a);
    m.ka = m.k * m.a;
    p.a = cs->pp7_start[s];
    p.e = cs->pp7_end[s];
    p.phi = cs->pp7_loopn[s] / 24;  // GetFluorFromPolPos.m:60
    p.k = p.phi / (p.e - p.a);
    p.ka = p.k * p.a;
    kp->ms2[s] = m;
    kp->pp7[s] = p;
    emax = std::max(emax, std::max(m.e, p.e));
  }
  kp->emax = emax;
}

// Rows per lane of the register-resident kernel, or 0 for the long-cell kernel (N > 513).
int pick_rpl(int64_t max_points) {
  const int64_t steps = max_points - 1;
  for (int r : {1, 2, 4, 8})
    if (64 * r >= steps) return r;
  return 0;
}

int run(tci_ctx* ctx, int mode, const double* theta, int64_t ld, const int32_t* cell, const uint8_t* active,
        int64_t B, double* out0, double* out1, int64_t ld_out, void* stream) {
  TCI_HIP(ctx, hipSetDevice(ctx->device));
  // every cell has >= 2 points, so a row needs >= 9 entries; the kernels read theta[0..6] of a row
  // before they know its cell (tci_kernels.hip)
  if (B > 0 && ld < 9) return fail(ctx, TCI_ERANGE, "ld_theta=" + std::to_string(ld) + " < 9 (7 + at least 2 rates)");
  const int rc = tci::launch(ctx->kp, ctx->rpl, mode, theta, ld, cell, active, B, out0, out1, ld_out, stream);
  if (rc != TCI_OK) {
    if (rc == TCI_EHIP) return hip_fail(ctx, hipGetLastError(), "kernel launch");
    return fail(ctx, rc, "kernel launch rejected");
  }
  return TCI_OK;
}

// Host-side validation of a host-pointer batch (cell ids and row lengths).
int check_rows(tci_ctx* ctx, int64_t ld, const int32_t* cell, int64_t B) {
  for (int64_t b = 0; b < B; ++b) {
    const int32_t c = cell[b];
    if (c < 0 || c >= ctx->n_cells)
      return fail(ctx, TCI_ERANGE, "row " + std::to_string(b) + ": cell id " + std::to_string(c) + " out of range");
    if (ld < 7 + ctx->meta[(size_t)c].n)
      return fail(ctx, TCI_ERANGE, "row " + std::to_string(b) + ": theta needs " +
                                       std::to_string(7 + ctx->meta[(size_t)c].n) + " entries (ld_theta=" +
                                       std::to_string(ld) + ")");
  }
  return TCI_OK;
}

const double kP2P_ms2_start[1] = {0.024};
const double kP2P_ms2_end[1] = {1.299};
const double kP2P_ms2_loopn[1] = {24};
const double kP2P_pp7_start[1] = {4.292};
const double kP2P_pp7_end[1] = {5.758};
const double kP2P_pp7_loopn[1] = {24};

}  // namespace

namespace tci {

int ensure_dyn_lds(const void* func, size_t bytes) {
  if (bytes <= 48 * 1024) return TCI_OK;  // within the default limit
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TCI_EHIP;
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, size_t> set;  // per device and kernel
  std::lock_guard<std::mutex> lock(mu);
  size_t& have = set[{dev, func}];
  if (bytes <= have) return TCI_OK;
  if (hipFuncSetAttribute(func, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) return TCI_EHIP;
  have = bytes;
  return TCI_OK;
}

}  // namespace tci

extern "C" {

const char* tci_version(void) { return kVersion; }

int tci_construct_by_name(const char* name, tci_construct* out) {
  if (!name || !out) return TCI_EINVAL;
  // GetFluorFromPolPos.m:18-28
  if (std::strcmp(name, "P2P-MS2v5-LacZ-PP7v4") == 0) {
    out->L0 = 6.626;
    out->n_seg = 1;
    out->ms2_start = kP2P_ms2_start;
    out->ms2_end = kP2P_ms2_end;
    out->ms2_loopn = kP2P_ms2_loopn;
    out->pp7_start = kP2P_pp7_start;
    out->pp7_end = kP2P_pp7_end;
    out->pp7_loopn = kP2P_pp7_loopn;
    return TCI_OK;
  }
  return TCI_EINVAL;
}

const char* tci_last_error(const tci_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int tci_create(const tci_cells* cells, const tci_construct* construct, int device, tci_ctx** out) {
  if (!out) return TCI_EINVAL;
  *out = nullptr;
  tci_ctx* ctx = new (std::nothrow) tci_ctx();
  if (!ctx) return TCI_ENOMEM;
  auto bail = [&](int rc) {
    *out = ctx;  // hand back the context so the caller can read tci_last_error, then destroy it
    return rc;
  };
  if (!cells || !cells->offsets || !cells->t || !cells->ms2 || !cells->pp7 || cells->n_cells <= 0)
    return bail(fail(ctx, TCI_EINVAL, "cells table is empty or has NULL arrays"));
  int rc = check_construct(ctx, construct);
  if (rc != TCI_OK) return bail(rc);
  ctx->device = device;
  ctx->n_cells = cells->n_cells;

  // ---- host precompute of the theta-independent per-cell tables
  const int64_t C = cells->n_cells;
  ctx->meta.resize((size_t)C);
  for (int64_t c = 0; c < C; ++c) {
    const int64_t n = cells->offsets[c + 1] - cells->offsets[c];
    if (n < 2) return bail(fail(ctx, TCI_EINVAL, "cell " + std::to_string(c) + " has fewer than 2 points"));
    if (n > TCI_MAX_POINTS)
      return bail(fail(ctx, TCI_EINVAL, "cell " + std::to_string(c) + " has " + std::to_string(n) +
                                            " points (max " + std::to_string(TCI_MAX_POINTS) + ")"));
    ctx->meta[(size_t)c] = CellMeta{(int32_t)n, 0, 0.0, 0.0, 0.0};
    ctx->max_points = std::max(ctx->max_points, n);
  }
  ctx->rpl = pick_rpl(ctx->max_points);
  // records per cell: every slot/point index a wave touches (the long-cell kernel reads < N)
  const int64_t stride = ctx->rpl > 0 ? 64 * (ctx->rpl + 1) : (ctx->max_points + 63) / 64 * 64;
  ctx->stride = stride;
  const size_t total = (size_t)C * (size_t)stride;
  // slots past a cell's last step: dt = 0 and t = -Inf, so every kernel skips them as steps before ton
  // (ConstantElongationSim.m:57-60) without a bounds test
  std::vector<tci::StepRec> steps(total, tci::StepRec{0.0, -INFINITY}), steps_raw(total, tci::StepRec{0.0, -INFINITY});
  std::vector<tci::PointRec> points(total, tci::PointRec{NAN, NAN, NAN, 0, 0});
  ctx->grid.assign(total, 0.0);
  for (int64_t c = 0; c < C; ++c) {
    const int64_t o = cells->offsets[c], n = ctx->meta[(size_t)c].n, base = c * stride;
    const double* t = cells->t + o;
    for (int64_t j = 0; j < n; ++j) {
      if (!std::isfinite(t[j]))
        return bail(fail(ctx, TCI_EINVAL, "cell " + std::to_string(c) + ": non-finite time"));
      if (j > 0 && !(t[j] > t[j - 1]))
        return bail(fail(ctx, TCI_EINVAL, "cell " + std::to_string(c) + ": times must be strictly increasing"));
    }
    double dgrid = 0.0;
    std::vector<double> g = interp_grid(t, n, &dgrid);  // SumofSquares...m:29-30
    if ((int64_t)g.size() != n)
      return bail(fail(ctx, TCI_EDIM, "cell " + std::to_string(c) + ": grid t(1):mean(diff(t)):t(end) has " +
                                          std::to_string(g.size()) + " points, data has " + std::to_string(n) +
                                          " (the reference errors: ConstantElongationSim.m:47)"));
    double delta = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      ctx->grid[(size_t)(base + i)] = g[(size_t)i];
      if (i + 1 < n) {
        const double dti = g[(size_t)i + 1] - g[(size_t)i];  // ConstantElongationSim.m:43-45
        steps[(size_t)(base + i)] = tci::StepRec{dti, g[(size_t)i]};
        steps_raw[(size_t)(base + i)] = tci::StepRec{t[i + 1] - t[i], t[i]};
        delta = std::max(delta, std::fabs(dti - dgrid));
      }
    }
    ctx->meta[(size_t)c].d = dgrid;
    ctx->meta[(size_t)c].delta = delta;
    // |p(r, r-m) - m*(v*d)| <= v * (m*delta + (m+4)*u*m*(d+delta)) for every distance m <= n-1
    // (tci_kernels.hip, fast path); doubled, plus 2^-40 relative for the rounding of v * eps_v.
    const double mx = (double)(n - 1);
    ctx->meta[(size_t)c].eps_v =
        2.0 * (mx * delta + (mx + 4.0) * 0x1p-53 * mx * (dgrid + delta)) * (1.0 + 0x1p-40);
    // interp1(t_interp, y, t): interval k = last grid point <= t_j (clamped to n-2);
    // outside [t_interp(1), t_interp(end)] -> NaN (w = NaN, k = 0).
    for (int64_t j = 0; j < n; ++j) {
      tci::PointRec& pr = points[(size_t)(base + j)];
      pr.y1 = cells->ms2[o + j];
      pr.y2 = cells->pp7[o + j];
      const double q = t[j];
      if (!(q >= g[0] && q <= g[(size_t)n - 1])) continue;
      int64_t k = (int64_t)(std::upper_bound(g.begin(), g.end(), q) - g.begin()) - 1;
      k = std::min(std::max(k, (int64_t)0), n - 2);
      pr.k = (int32_t)k;
      pr.w = (q - g[(size_t)k]) / (g[(size_t)k + 1] - g[(size_t)k]);
    }
  }

  // ---- upload: one resident allocation, 256-byte aligned sub-arrays
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t szM = al((size_t)C * sizeof(CellMeta)), szS = al(total * sizeof(tci::StepRec)),
               szP = al(total * sizeof(tci::PointRec));
  const size_t szT = al(64 * sizeof(double));
  const size_t bytes = szM + 2 * szS + szP + szT;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return bail(hip_fail(ctx, e, "hipSetDevice"));
  e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e != hipSuccess) return bail(hip_fail(ctx, e, "hipStreamCreate"));
  e = hipMalloc(&ctx->dbuf, bytes);
  if (e != hipSuccess) return bail(hip_fail(ctx, e, "hipMalloc(cell table)"));
  ctx->device_bytes = (int64_t)bytes;
  char* p = (char*)ctx->dbuf;
  auto put = [&](const void* src, size_t n, size_t span) -> void* {
    void* dst = p;
    p += span;
    if (hipMemcpy(dst, src, n, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return dst;
  };
  KParams& kp = ctx->kp;
  kp.cells = (const CellMeta*)put(ctx->meta.data(), (size_t)C * sizeof(CellMeta), szM);
  kp.steps = (const tci::StepRec*)put(steps.data(), total * sizeof(tci::StepRec), szS);
  kp.steps_raw = (const tci::StepRec*)put(steps_raw.data(), total * sizeof(tci::StepRec), szS);
  kp.points = (const tci::PointRec*)put(points.data(), total * sizeof(tci::PointRec), szP);
  double thr[64] = {0.0};
  for (int k = 0; k < construct->n_seg; ++k) {
    thr[1 + 4 * k] = construct->ms2_start[k];
    thr[2 + 4 * k] = construct->ms2_end[k];
    thr[3 + 4 * k] = construct->pp7_start[k];
    thr[4 + 4 * k] = construct->pp7_end[k];
  }
  kp.thr = (const double*)put(thr, sizeof(thr), szT);
  if (!kp.cells || !kp.steps || !kp.steps_raw || !kp.points || !kp.thr)
    return bail(fail(ctx, TCI_EHIP, "hipMemcpy(cell table) failed"));
  kp.cell_stride = stride;
  kp.max_n = ctx->max_points;
  kp.n_cells = C;
  kp.force_exact = 0;
  fill_segments(&kp, construct);
  *out = ctx;
  return TCI_OK;
}

int tci_destroy(tci_ctx* ctx) {
  if (!ctx) return TCI_EINVAL;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (void* q : {(void*)ctx->dbuf, (void*)ctx->d_theta, (void*)ctx->d_cell, (void*)ctx->d_active,
                  (void*)ctx->d_out0, (void*)ctx->d_out1})
    if (q) (void)hipFree(q);
  if (ctx->h_io) (void)hipHostFree(ctx->h_io);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return TCI_OK;
}

int tci_get_info(const tci_ctx* ctx, tci_info* out) {
  if (!ctx || !out) return TCI_EINVAL;
  out->device = ctx->device;
  out->rows_per_lane = ctx->rpl;
  out->n_cells = ctx->n_cells;
  out->max_points = ctx->max_points;
  out->device_bytes = ctx->device_bytes;
  return TCI_OK;
}

int tci_set_force_exact_scan(tci_ctx* ctx, int flags) {
  if (!ctx || flags < 0 || flags > 3) return TCI_EINVAL;
  ctx->kp.force_exact = flags;
  return TCI_OK;
}

int tci_ss_batch_async(tci_ctx* ctx, const double* d_theta, int64_t ld_theta, const int32_t* d_cell_id,
                       const uint8_t* d_active, int64_t B, double* d_ss_out, void* stream) {
  if (!ctx) return TCI_EINVAL;
  if (B < 0 || (B > 0 && (!d_theta || !d_cell_id || !d_ss_out)))
    return fail(ctx, TCI_EINVAL, "null device pointer or negative batch");
  return run(ctx, tci::MODE_SS, d_theta, ld_theta, d_cell_id, d_active, B, d_ss_out, nullptr, 0, stream);
}

int tci_ss_batch(tci_ctx* ctx, const double* theta, int64_t ld_theta, const int32_t* cell_id,
                 const uint8_t* active, int64_t B, double* ss_out) {
  if (!ctx) return TCI_EINVAL;
  if (B < 0 || (B > 0 && (!theta || !cell_id || !ss_out)))
    return fail(ctx, TCI_EINVAL, "null pointer or negative batch");
  if (B == 0) return TCI_OK;
  int rc = check_rows(ctx, ld_theta, cell_id, B);
  if (rc != TCI_OK) return rc;
  TCI_HIP(ctx, hipSetDevice(ctx->device));
  const size_t nth = (size_t)B * (size_t)ld_theta;
  // layout of the zero-copy buffer: theta | SS | cell ids | active flags (8-byte aligned blocks)
  const size_t o_ss = nth * 8, o_cell = o_ss + (size_t)B * 8, o_act = o_cell + ((size_t)B * 4 + 7) / 8 * 8;
  if (o_act + (size_t)B <= zero_copy_max()) {
    // a small batch (the drop-in tci_ssfun is B = 1): the kernel reads theta/ids/flags from pinned
    // host memory and writes the SS there; one launch and one synchronisation per call
    if ((rc = ensure_io(ctx, o_act + (size_t)B)) != TCI_OK) return rc;
    std::memcpy(ctx->h_io, theta, nth * 8);
    std::memcpy(ctx->h_io + o_cell, cell_id, (size_t)B * 4);
    if (active) std::memcpy(ctx->h_io + o_act, active, (size_t)B);
    rc = run(ctx, tci::MODE_SS, (const double*)ctx->d_io, ld_theta, (const int32_t*)(ctx->d_io + o_cell),
             active ? (const uint8_t*)(ctx->d_io + o_act) : nullptr, B, (double*)(ctx->d_io + o_ss), nullptr, 0,
             (void*)ctx->stream);
    if (rc != TCI_OK) return rc;
    TCI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::memcpy(ss_out, ctx->h_io + o_ss, (size_t)B * 8);
    return TCI_OK;
  }
  if ((rc = ensure(ctx, &ctx->d_theta, &ctx->cap_theta, nth)) != TCI_OK) return rc;
  if ((rc = ensure(ctx, &ctx->d_cell, &ctx->cap_cell, (size_t)B)) != TCI_OK) return rc;
  if ((rc = ensure(ctx, &ctx->d_active, &ctx->cap_active, (size_t)B)) != TCI_OK) return rc;
  if ((rc = ensure(ctx, &ctx->d_out0, &ctx->cap_out0, (size_t)B)) != TCI_OK) return rc;
  hipStream_t st = ctx->stream;
  TCI_HIP(ctx, hipMemcpyAsync(ctx->d_theta, theta, nth * sizeof(double), hipMemcpyHostToDevice, st));
  TCI_HIP(ctx, hipMemcpyAsync(ctx->d_cell, cell_id, (size_t)B * sizeof(int32_t), hipMemcpyHostToDevice, st));
  if (active)
    TCI_HIP(ctx, hipMemcpyAsync(ctx->d_active, active, (size_t)B, hipMemcpyHostToDevice, st));
  rc = run(ctx, tci::MODE_SS, ctx->d_theta, ld_theta, ctx->d_cell, active ? ctx->d_active : nullptr, B, ctx->d_out0,
           nullptr, 0, (void*)st);
  if (rc != TCI_OK) return rc;
  TCI_HIP(ctx, hipMemcpyAsync(ss_out, ctx->d_out0, (size_t)B * sizeof(double), hipMemcpyDeviceToHost, st));
  TCI_HIP(ctx, hipStreamSynchronize(st));
  return TCI_OK;
}

int tci_ssfun(tci_ctx* ctx, int32_t cell, const double* theta, int64_t P, double* ss_out) {
  if (!ctx) return TCI_EINVAL;
  return tci_ss_batch(ctx, theta, P, &cell, nullptr, 1, ss_out);
}

int tci_forward(tci_ctx* ctx, const double* theta, int64_t ld_theta, const int32_t* cell_id, int64_t B,
                int grid_mode, double* ms2_out, double* pp7_out, int64_t ld_out) {
  if (!ctx) return TCI_EINVAL;
  if (grid_mode != TCI_GRID_INTERP && grid_mode != TCI_GRID_RAW)
    return fail(ctx, TCI_EINVAL, "grid_mode must be TCI_GRID_INTERP or TCI_GRID_RAW");
  if (B < 0 || (B > 0 && (!theta || !cell_id || !ms2_out || !pp7_out)))
    return fail(ctx, TCI_EINVAL, "null pointer or negative batch");
  if (B == 0) return TCI_OK;
  int rc = check_rows(ctx, ld_theta, cell_id, B);
  if (rc != TCI_OK) return rc;
  for (int64_t b = 0; b < B; ++b)
    if (ld_out < ctx->meta[(size_t)cell_id[b]].n) return fail(ctx, TCI_ERANGE, "ld_out shorter than a cell");
  TCI_HIP(ctx, hipSetDevice(ctx->device));
  const size_t nth = (size_t)B * (size_t)ld_theta, nout = (size_t)B * (size_t)ld_out;
  if ((rc = ensure(ctx, &ctx->d_theta, &ctx->cap_theta, nth)) != TCI_OK) return rc;
  if ((rc = ensure(ctx, &ctx->d_cell, &ctx->cap_cell, (size_t)B)) != TCI_OK) return rc;
  if ((rc = ensure(ctx, &ctx->d_out0, &ctx->cap_out0, nout)) != TCI_OK) return rc;
  if ((rc = ensure(ctx, &ctx->d_out1, &ctx->cap_out1, nout)) != TCI_OK) return rc;
  hipStream_t st = ctx->stream;
  TCI_HIP(ctx, hipMemcpyAsync(ctx->d_theta, theta, nth * sizeof(double), hipMemcpyHostToDevice, st));
  TCI_HIP(ctx, hipMemcpyAsync(ctx->d_cell, cell_id, (size_t)B * sizeof(int32_t), hipMemcpyHostToDevice, st));
  rc = run(ctx, grid_mode == TCI_GRID_RAW ? tci::MODE_FWD_RAW : tci::MODE_FWD_INTERP, ctx->d_theta, ld_theta,
           ctx->d_cell, nullptr, B, ctx->d_out0, ctx->d_out1, ld_out, (void*)st);
  if (rc != TCI_OK) return rc;
  TCI_HIP(ctx, hipMemcpyAsync(ms2_out, ctx->d_out0, nout * sizeof(double), hipMemcpyDeviceToHost, st));
  TCI_HIP(ctx, hipMemcpyAsync(pp7_out, ctx->d_out1, nout * sizeof(double), hipMemcpyDeviceToHost, st));
  TCI_HIP(ctx, hipStreamSynchronize(st));
  return TCI_OK;
}

int tci_device_count(int* n_out) {
  if (!n_out) return TCI_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;  // hipErrorNoDevice: none visible
  *n_out = n;
  return TCI_OK;
}

int tci_cell_points(const tci_ctx* ctx, int32_t cell, int64_t* n_out) {
  if (!ctx || !n_out || cell < 0 || cell >= ctx->n_cells) return TCI_EINVAL;
  *n_out = ctx->meta[(size_t)cell].n;
  return TCI_OK;
}

int tci_cell_grid(const tci_ctx* ctx, int32_t cell, double* t_interp_out, int64_t cap, int64_t* m_out) {
  if (!ctx || cell < 0 || cell >= ctx->n_cells) return TCI_EINVAL;
  const CellMeta& m = ctx->meta[(size_t)cell];
  if (m_out) *m_out = m.n;
  if (!t_interp_out) return TCI_OK;
  if (cap < m.n) return TCI_ERANGE;
  std::memcpy(t_interp_out, ctx->grid.data() + (size_t)cell * (size_t)ctx->stride, (size_t)m.n * sizeof(double));
  return TCI_OK;
}

}  // extern "C"

namespace {

// Device allocations of one DRAM run, freed together.
struct DevAllocs {
  std::vector<void*> ptrs;
  ~DevAllocs() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <typename T>
  T* alloc(size_t n, hipError_t* err) {
    void* p = nullptr;
    *err = hipMalloc(&p, std::max(n, (size_t)1) * sizeof(T));
    if (*err == hipSuccess) ptrs.push_back(p);
    return (T*)p;
  }
};

// One DRAM step: propose -> ssfun -> accept/propose stage 2 -> ssfun -> accept, sigma2, log the row
// -> [window records] -> [adapt] -> step + 1.
int enqueue_step(tci_ctx* ctx, const tci::DramState& st, const tci::DramParams& p, hipStream_t s, bool with_stats,
                 bool with_adapt) {
  int rc;
  if ((rc = tci::dram_launch_propose1(st, p, s)) != TCI_OK) return rc;
  if ((rc = tci::launch(ctx->kp, ctx->rpl, tci::MODE_SS, st.prop1, st.ld, st.cell, st.act1, st.n_chains, st.ss1,
                        nullptr, 0, s)) != TCI_OK)
    return rc;
  if ((rc = tci::dram_launch_accept1(st, p, s)) != TCI_OK) return rc;
  if (p.ntry >= 2 && (rc = tci::launch(ctx->kp, ctx->rpl, tci::MODE_SS, st.prop2, st.ld, st.cell, st.act2,
                                       st.n_chains, st.ss2, nullptr, 0, s)) != TCI_OK)
    return rc;
  if ((rc = tci::dram_launch_accept2(st, p, s)) != TCI_OK) return rc;
  if (with_stats && (rc = tci::dram_launch_stats(st, p, s)) != TCI_OK) return rc;
  if (with_adapt && (rc = tci::dram_launch_adapt(st, p, s)) != TCI_OK) return rc;  // no-op unless step % adaptint == 0
  return tci::dram_launch_step_incr(st, s);
}

}  // namespace

extern "C" {

int tci_dram_defaults(tci_dram_options* o) {
  if (!o) return TCI_EINVAL;
  o->n_steps = 20000;     // TranscriptionCycleMCMC.m:40
  o->burnintime = 10000;  // :39, :267
  o->adaptint = 100;      // :268
  o->ntry = 2;            // 'dram' (:269)
  o->updatesigma = 1;     // :265
  o->drscale = 5.0;
  o->adascale = 0.0;
  o->qcovadj = 1e-5;
  o->burnin_scale = 10.0;
  o->stats_from = 10000;  // chain(n_burn:end, :) (:276)
  o->thin = 0;
  o->seed = 20201028;
  o->engine = TCI_DRAM_AUTO;
  o->max_chunk = 0;
  o->chain_keys = nullptr;
  o->adapt_pmax = 0;
  o->kernel_times = 0;
  return TCI_OK;
}

int tci_dram_run(tci_ctx* ctx, const tci_dram_options* opt, int64_t n_chains, const int32_t* cell_id,
                 const double* theta0, const double* lower, const double* upper, const double* prior_mu,
                 const double* prior_sig, const double* qcov_diag, const double* sigma2_0, int64_t ld,
                 tci_dram_outputs* out) {
  if (!ctx) return TCI_EINVAL;
  if (!opt || !out || n_chains <= 0 || !cell_id || !theta0 || !lower || !upper || !prior_mu || !prior_sig ||
      !qcov_diag || !sigma2_0)
    return fail(ctx, TCI_EINVAL, "tci_dram_run: null argument or no chains");
  if (opt->n_steps < 1 || opt->ntry < 1 || opt->ntry > 2 || opt->adaptint < 0 || !(opt->drscale > 0) ||
      opt->engine < TCI_DRAM_AUTO || opt->engine > TCI_DRAM_WALK || opt->max_chunk < 0 || opt->adapt_pmax < 0 ||
      opt->adapt_pmax > TCI_MAX_POINTS + 7)
    return fail(ctx, TCI_EINVAL,
                "tci_dram_run: bad options (n_steps >= 1, ntry in {1,2}, adaptint >= 0, engine in {0,1,2,3}, "
                "max_chunk >= 0, 0 <= adapt_pmax <= 2055)");
  int rc = check_rows(ctx, ld, cell_id, n_chains);
  if (rc != TCI_OK) return rc;
  if (ld > TCI_MAX_POINTS + 7) return fail(ctx, TCI_ERANGE, "tci_dram_run: ld too large");
  const size_t n = (size_t)n_chains, L = (size_t)ld, L2 = L * L;
  std::vector<int32_t> npar(n), nobs(n);
  for (size_t c = 0; c < n; ++c) {
    const int32_t N = ctx->meta[(size_t)cell_id[c]].n;
    npar[c] = 7 + N;
    nobs[c] = 2 * N;  // model.N = length(data.ydata) (:260), NaNs included
    for (int32_t j = 0; j < npar[c]; ++j) {
      const double x = theta0[c * L + j];
      if (!(x >= lower[c * L + j] && x <= upper[c * L + j]))
        return fail(ctx, TCI_EINVAL, "tci_dram_run: chain " + std::to_string(c) + " starts outside its bounds");
      if (!(qcov_diag[c * L + j] > 0)) return fail(ctx, TCI_EINVAL, "tci_dram_run: qcov_diag must be > 0");
    }
  }
  // the P the adaptation kernel is picked for (> 208: k_adapt_gt and its tile grid): this run's largest,
  // or the whole fit's when this run is a shard of it (adapt_pmax)
  const int64_t p_max_all = std::max<int64_t>(*std::max_element(npar.begin(), npar.end()), opt->adapt_pmax);
  // limits of the adaptation window, checked before anything is allocated or launched: the
  // adaptation kernel's LDS (the window's run table grows with adaptint) and the chain kernels'
  // 32-bit window-log offsets (adaptint * ld)
  if (opt->adaptint > 0 && tci::dram_adapt_lds_bytes(p_max_all, opt->adaptint) > 160 * 1024)
    return fail(ctx, TCI_ERANGE, "tci_dram_run: adaptint " + std::to_string(opt->adaptint) +
                                     " needs more LDS than a CU has for the adaptation at P = " +
                                     std::to_string(p_max_all));
  if ((opt->adaptint > 0 ? opt->adaptint : 100) * ld >= (int64_t)INT32_MAX)
    return fail(ctx, TCI_ERANGE, "tci_dram_run: adaptint * ld must be < 2^31");
  TCI_HIP(ctx, hipSetDevice(ctx->device));
  DevAllocs A;
  hipError_t e = hipSuccess;
  tci::DramState st{};
  tci::DramParams p{};
  // Chunk of chain rows per fused-engine pass (its draws buffer holds one chunk; at most the next
  // adaptation row) and the window slots per chain: the covupd window (adaptint rows), which is also
  // every engine's per-row log.
  const int64_t ai = opt->adaptint;
  const int64_t DW = tci::draw_stride(ld);
  const int64_t chunk_cap =
      std::max<int64_t>(32, (int64_t)(((size_t)tci::kDrawsGiB << 30) / (n * (size_t)DW * sizeof(double))));
  // Without adaptation the window is 100 rows: the records' merge partition (the same for every engine)
  // and the batched engine's graph block stay small (a 1,000-row window made the batched engine run up
  // to 1,000 steps as plain launches before its first graph replay).
  const int64_t win = ai > 0 ? ai : 100;
  int64_t chunk = std::min<int64_t>(win, chunk_cap);
  if (opt->max_chunk > 0) chunk = std::min<int64_t>(chunk, opt->max_chunk);
  const int64_t n_keep = opt->thin > 0 ? (opt->n_steps + opt->thin - 1) / opt->thin : 0;
  st.n_chains = n_chains;
  st.ld = ld;
#define TCI_ALLOC(field, T, count)                                  \
  do {                                                              \
    st.field = A.alloc<T>((count), &e);                             \
    if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(dram " #field ")"); \
  } while (0)
  int32_t *d_cell, *d_npar, *d_nobs;
  double *d_lower, *d_upper, *d_pmu, *d_psig, *d_qdiag, *d_s20;
  d_cell = A.alloc<int32_t>(n, &e);
  int64_t* d_key = A.alloc<int64_t>(n, &e);
  d_npar = A.alloc<int32_t>(n, &e);
  d_nobs = A.alloc<int32_t>(n, &e);
  d_lower = A.alloc<double>(n * L, &e);
  d_upper = A.alloc<double>(n * L, &e);
  d_pmu = A.alloc<double>(n * L, &e);
  d_psig = A.alloc<double>(n * L, &e);
  d_qdiag = A.alloc<double>(n * L, &e);
  d_s20 = A.alloc<double>(n, &e);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(dram inputs)");
  st.cell = d_cell;
  st.key = d_key;
  st.npar = d_npar;
  st.nobs = d_nobs;
  st.lower = d_lower;
  st.upper = d_upper;
  st.pmu = d_pmu;
  st.psig = d_psig;
  TCI_ALLOC(theta, double, n * L);
  TCI_ALLOC(ss, double, n);
  TCI_ALLOC(prior, double, n);
  TCI_ALLOC(sigma2, double, n);
  TCI_ALLOC(Rd, double, n * tci::dram_tri_stride(L));
  TCI_ALLOC(cov, double, n * tci::dram_cov_stride(L));
  TCI_ALLOC(work, double, p_max_all > tci::kAdaptGtFrom ? n * (size_t)((L + 15) / 16 * 16) * ((L + 15) / 16 * 16) : 1);
  TCI_ALLOC(cmean, double, n * L);
  TCI_ALLOC(wsum, double, n);
  TCI_ALLOC(window, double, n * (size_t)win * L);
  TCI_ALLOC(wsumv, double, n * L);
  TCI_ALLOC(wacc1, double, n * L);
  TCI_ALLOC(wacc2, double, n * L);
  TCI_ALLOC(s2acc, double, n * 3);
  TCI_ALLOC(s2log, double, n * (size_t)win);
  TCI_ALLOC(runf, uint8_t, n * (size_t)win);
  TCI_ALLOC(prop1, double, n * L);
  TCI_ALLOC(prop2, double, n * L);
  TCI_ALLOC(act1, uint8_t, n);
  TCI_ALLOC(act2, uint8_t, n);
  TCI_ALLOC(acc1, uint8_t, n);
  TCI_ALLOC(ss1, double, n);
  TCI_ALLOC(ss2, double, n);
  TCI_ALLOC(prior1, double, n);
  TCI_ALLOC(a12, double, n);
  TCI_ALLOC(naccept, int32_t, n);
  TCI_ALLOC(nrej_win, int32_t, n);
  TCI_ALLOC(nevals, int64_t, n);
  TCI_ALLOC(smean, double, n * L);
  TCI_ALLOC(sm2, double, n * L);
  TCI_ALLOC(s2sum, double, n);
  TCI_ALLOC(sq_mean, double, n);
  TCI_ALLOC(sq_m2, double, n);
  TCI_ALLOC(step, int64_t, 1);
#if TCI_CHAIN_PROFILE || TCI_ADAPT_PROFILE
  TCI_ALLOC(prof, int64_t, 32);
  TCI_HIP(ctx, hipMemsetAsync(st.prof, 0, 32 * sizeof(int64_t), ctx->stream));
#endif
  if (n_keep > 0 && (out->chain || out->s2chain)) {
    TCI_ALLOC(chain_out, double, (size_t)n_keep * n * L);
    TCI_ALLOC(s2_out, double, (size_t)n_keep * n);
    // entries past a chain's P are never written: zero them so outputs are deterministic
    TCI_HIP(ctx, hipMemsetAsync(st.chain_out, 0, (size_t)n_keep * n * L * sizeof(double), ctx->stream));
  }
#undef TCI_ALLOC
  hipStream_t s = ctx->stream;
  TCI_HIP(ctx, hipMemcpyAsync(d_cell, cell_id, n * sizeof(int32_t), hipMemcpyHostToDevice, s));
  std::vector<int64_t> keys(n);
  for (size_t c = 0; c < n; ++c) keys[c] = opt->chain_keys ? opt->chain_keys[c] : (int64_t)c;
  TCI_HIP(ctx, hipMemcpyAsync(d_key, keys.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(d_npar, npar.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(d_nobs, nobs.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(d_lower, lower, n * L * sizeof(double), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(d_upper, upper, n * L * sizeof(double), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(d_pmu, prior_mu, n * L * sizeof(double), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(d_psig, prior_sig, n * L * sizeof(double), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(d_qdiag, qcov_diag, n * L * sizeof(double), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(d_s20, sigma2_0, n * sizeof(double), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemcpyAsync(st.theta, theta0, n * L * sizeof(double), hipMemcpyHostToDevice, s));
  TCI_HIP(ctx, hipMemsetAsync(st.wsum, 0, n * sizeof(double), s));
  TCI_HIP(ctx, hipMemsetAsync(st.act2, 0, n, s));
  p.seed = opt->seed;
  p.ntry = opt->ntry;
  p.updatesigma = opt->updatesigma;
  p.drscale = opt->drscale;
  p.adascale = opt->adascale;
  p.qcovadj = opt->qcovadj;
  p.burnin_scale = opt->burnin_scale;
  p.adaptint = opt->adaptint;
  p.burnintime = opt->burnintime;
  p.stats_from = std::max<int64_t>(opt->stats_from, 1);
  p.thin = opt->thin;
  p.n_keep = n_keep;
  p.win = win;
  // initial state: R = chol(J0), prior, sigma2, the initial ssfun call, chain row 1
  if ((rc = tci::dram_launch_init(st, d_qdiag, d_s20, s)) != TCI_OK) return fail(ctx, rc, "dram init launch");
  if ((rc = tci::launch(ctx->kp, ctx->rpl, tci::MODE_SS, st.theta, ld, d_cell, nullptr, n_chains, st.ss, nullptr, 0,
                        s)) != TCI_OK)
    return fail(ctx, rc, "initial ssfun launch");
  if ((rc = tci::dram_launch_init_stats(st, p, s)) != TCI_OK) return fail(ctx, rc, "dram stats launch");
  if (win == 1) {  // one-row windows: row 1 is a window of its own
    const int64_t one = 1;
    TCI_HIP(ctx, hipMemcpyAsync(st.step, &one, sizeof(int64_t), hipMemcpyHostToDevice, s));
    if ((rc = tci::dram_launch_stats(st, p, s)) != TCI_OK) return fail(ctx, rc, "dram stats launch");
  }
  const int64_t two = 2;
  TCI_HIP(ctx, hipMemcpyAsync(st.step, &two, sizeof(int64_t), hipMemcpyHostToDevice, s));
  hipEvent_t ev0, ev1;
  TCI_HIP(ctx, hipEventCreate(&ev0));
  TCI_HIP(ctx, hipEventCreate(&ev1));
  TCI_HIP(ctx, hipEventRecord(ev0, s));
  p.pmax = p_max_all;
  // the fused engine's draws pass keeps a chain's R (packed fp32) and a tile of normals and products
  // in LDS: it must fit a CU (160 KB). AUTO picks it whenever it fits: measured on config 4 (10,000
  // chains x 200 points, 39 per CU) its chain walk + draws pass take 209 us per step against 1950 us
  // for the batched engine's per-step kernels, which stage every chain's R once per stage.
  const int64_t fused_lds = tci::dram_chain_lds_bytes(ld, ctx->rpl);
  const bool fused_fits = ctx->rpl > 0 && fused_lds <= 160 * 1024;  // long cells: the batched engine
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  // WALK (one wavefront per chain) once k_chain's one-workgroup-per-chain layout would need more
  // than one round of resident workgroups (two chains per CU).
  int n_cu = 0;
  TCI_HIP(ctx, hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, ctx->device));
  bool fused = opt->engine == TCI_DRAM_FUSED || opt->engine == TCI_DRAM_WALK;
  p.walk = opt->engine == TCI_DRAM_WALK ? 1 : 0;
  if (opt->engine == TCI_DRAM_AUTO) {
    fused = fused_fits;
    p.walk = n_chains > 2 * (int64_t)std::max(n_cu, 1) ? 1 : 0;
  }
  if (fused && !fused_fits) return fail(ctx, TCI_ERANGE, "tci_dram_run: rows too long for the fused engine");
  for (int k = 0; k < 4; ++k) {
    out->kernel_ms[k] = 0.0;
    out->kernel_launches[k] = 0;
  }
  tci::LaunchTimer timer;
  tci::LaunchTimer* tm = opt->kernel_times && fused ? &timer : nullptr;
  if (fused) {
    // Chunks of chain rows up to the next adaptation row (and at most p.chunk rows: the draws
    // buffer holds one chunk); k_chain leaves *st.step at the chunk end. Per chunk: the draws pass
    // and the walk (dram_launch_chain, which also keeps a completed window's records), and at an
    // adaptation row the adaptation.
    p.chunk = chunk;
    st.draws = A.alloc<double>(n * (size_t)p.chunk * DW, &e);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(dram draws)");
    std::vector<std::pair<int64_t, int64_t>> chunks;
    for (int64_t next = 2; next <= opt->n_steps;) {
      int64_t end = std::min<int64_t>(opt->n_steps, next + p.chunk - 1);
      end = std::min<int64_t>(end, ((next + win - 1) / win) * win);  // chunks never cross a window
      chunks.emplace_back(next, end);
      next = end + 1;
    }
    // k_chain's engine splits the draws (DramParams::split; TCI_DRAWS_SPLIT=0 keeps them in one
    // launch): chunk i + 1's normals and scalar draws go into the other of two draws buffers, drawn by
    // extra workgroups of chunk i's k_chain launch in the CU slots its chains leave free; k_draws then
    // only multiplies by the adapted R. The first chunk's: one k_draws_rng launch.
    // Only while the chains leave slots free (at most two chain workgroups per CU, AUTO's FUSED range):
    // past that the extra workgroups would wait behind the chains.
    const char* split_env = getenv("TCI_DRAWS_SPLIT");
    p.split = !p.walk && n_chains < 2 * (int64_t)std::max(n_cu, 1) && !(split_env && split_env[0] == '0') ? 1 : 0;
    double* dbuf[2] = {st.draws, st.draws};
    int rng_wgs = 0;
    if (p.split && !chunks.empty()) {
      dbuf[1] = A.alloc<double>(n * (size_t)p.chunk * DW, &e);
      if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(dram draws, second buffer)");
      // the workgroup slots the chains leave (two per CU), at least a quarter of the CUs
      const char* w_env = getenv("TCI_RNG_WGS");
      rng_wgs = w_env && atoi(w_env) > 0 ? atoi(w_env)
                                         : (int)std::max<int64_t>(2 * (int64_t)n_cu - n_chains, n_cu / 4);
      if ((rc = tci::dram_launch_draws_rng(st, p, chunks[0].first, chunks[0].second, 4 * std::max(n_cu, 1), s, tm)) !=
          TCI_OK)
        return fail(ctx, rc, "dram draws launch");
    }
    for (size_t i = 0; i < chunks.size() && rc == TCI_OK; ++i) {
      const int64_t next = chunks[i].first, end = chunks[i].second;
      const int rec = end % win == 0 || end == opt->n_steps;  // the records kept in the chain kernel
      tci::DramState sc = st;
      sc.draws = dbuf[i & 1];
      // the next chunk's buffer was last read by chunk i - 1's walk, which ended before this launch
      tci::ChainNext nx{dbuf[(i + 1) & 1], 0, -1, rng_wgs};
      if (i + 1 < chunks.size()) {
        nx.s_begin = chunks[i + 1].first;
        nx.s_end = chunks[i + 1].second;
      }
      rc = tci::dram_launch_chain(sc, p, ctx->kp, ctx->rpl, next, end, rec, s, tm,
                                  p.split && i + 1 < chunks.size() ? &nx : nullptr);
      if (rc == TCI_OK && ai > 0 && end % ai == 0) rc = tci::dram_launch_adapt(sc, p, s, tm);
    }
    e = hipSuccess;
  } else {
  // The step loop. Steps 2 .. n_steps; adaptation after steps that are multiples of adaptint.
  // Blocks of adaptint steps (aligned so that each ends on an adaptation step) are captured once
  // as a hipGraph and replayed; the head (steps 2..adaptint) and the tail run as plain launches.
  int64_t next = 2;  // next step number to enqueue
  auto plain = [&](int64_t upto) {  // steps next .. upto
    for (; next <= upto && rc == TCI_OK; ++next)
      rc = enqueue_step(ctx, st, p, s, next % win == 0, ai > 0 && next % ai == 0);
  };
  const int64_t G = win;  // graph blocks of one window (win = adaptint when adapting)
  plain(std::min<int64_t>(win, opt->n_steps));  // head: up to the first window's end
  const int64_t blocks = (opt->n_steps - next + 1) / G;
  if (rc == TCI_OK && blocks > 0) {
    TCI_HIP(ctx, hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int crc = TCI_OK;
    for (int64_t k = 0; k < G && crc == TCI_OK; ++k) crc = enqueue_step(ctx, st, p, s, k == G - 1, ai > 0 && k == G - 1);
    hipError_t ce = hipStreamEndCapture(s, &graph);
    if (crc != TCI_OK || ce != hipSuccess) {
      if (graph) (void)hipGraphDestroy(graph);
      return fail(ctx, TCI_EHIP, "DRAM step graph capture failed");
    }
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    if (e != hipSuccess) {
      (void)hipGraphDestroy(graph);
      return hip_fail(ctx, e, "hipGraphInstantiate");
    }
    for (int64_t b = 0; b < blocks && e == hipSuccess; ++b) e = hipGraphLaunch(exec, s);
    next += blocks * G;
  }
  if (e == hipSuccess) plain(opt->n_steps);  // tail
  }
  // the last, partial window's records (the fused engines: kept by the last chunk's kernel)
  if (e == hipSuccess && rc == TCI_OK && opt->n_steps % win != 0 && !(fused && opt->n_steps >= 2)) {
    const int64_t last = opt->n_steps;
    rc = hipMemcpyAsync(st.step, &last, sizeof(int64_t), hipMemcpyHostToDevice, s) == hipSuccess ? TCI_OK : TCI_EHIP;
    if (rc == TCI_OK) rc = tci::dram_launch_stats(st, p, s);
  }
  const hipError_t ge = e;
  TCI_HIP(ctx, hipEventRecord(ev1, s));
  TCI_HIP(ctx, hipStreamSynchronize(s));
  if (exec) (void)hipGraphExecDestroy(exec);
  if (graph) (void)hipGraphDestroy(graph);
#if TCI_CHAIN_PROFILE || TCI_ADAPT_PROFILE
  {
    int64_t ph[32];
    TCI_HIP(ctx, hipMemcpy(ph, st.prof, sizeof(ph), hipMemcpyDeviceToHost));
    // TCI_CHAIN_PROFILE=1: slots 0-6 are wave 0's cycles per phase; slot 5 also counts the rounds
    // in its bits 40+ (decoded here). =2: per-wave barrier waits (0-3) and pre-barrier work (4-7).
    // TCI_ADAPT_PROFILE: thread 0's cycles per adaptation phase. All summed over the chains.
    double rounds = 0.0;
    int nslots = 8;
#if TCI_CHAIN_PROFILE == 1 || TCI_CHAIN_PROFILE == 3
    // =3: slots 8 w + k, wave w's cycles per phase (slot 8 w + 5 also counts the rounds)
    nslots = TCI_CHAIN_PROFILE == 3 ? 32 : 8;
    rounds = (double)((uint64_t)ph[5] >> 40) / (double)n;
    for (int w = 0; w < nslots / 8; ++w) ph[8 * w + 5] = (int64_t)((uint64_t)ph[8 * w + 5] & ((1ull << 40) - 1));
#endif
    std::fprintf(stderr, "{\"cycles_per_chain\": [");
    for (int k = 0; k < nslots; ++k) std::fprintf(stderr, "%s%.1f", k ? ", " : "", (double)ph[k] / (double)n);
    std::fprintf(stderr, "], \"rounds_per_chain\": %.1f}\n", rounds);
  }
#endif
  if (ge != hipSuccess) return hip_fail(ctx, ge, "DRAM step replay");
  if (rc != TCI_OK) return fail(ctx, rc, "DRAM step launch");
  if (tm) tm->collect(out->kernel_ms, out->kernel_launches);
  float ms = 0.f;
  TCI_HIP(ctx, hipEventElapsedTime(&ms, ev0, ev1));
  (void)hipEventDestroy(ev0);
  (void)hipEventDestroy(ev1);
  out->elapsed_ms = ms;
  // ---- outputs
  std::vector<double> smean(n * L), sm2(n * L), s2sum(n), sqm(n), sqm2(n);
  std::vector<int32_t> nacc(n);
  std::vector<int64_t> nev(n);
  TCI_HIP(ctx, hipMemcpy(smean.data(), st.smean, n * L * sizeof(double), hipMemcpyDeviceToHost));
  TCI_HIP(ctx, hipMemcpy(sm2.data(), st.sm2, n * L * sizeof(double), hipMemcpyDeviceToHost));
  TCI_HIP(ctx, hipMemcpy(s2sum.data(), st.s2sum, n * sizeof(double), hipMemcpyDeviceToHost));
  TCI_HIP(ctx, hipMemcpy(sqm.data(), st.sq_mean, n * sizeof(double), hipMemcpyDeviceToHost));
  TCI_HIP(ctx, hipMemcpy(sqm2.data(), st.sq_m2, n * sizeof(double), hipMemcpyDeviceToHost));
  TCI_HIP(ctx, hipMemcpy(nacc.data(), st.naccept, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  TCI_HIP(ctx, hipMemcpy(nev.data(), st.nevals, n * sizeof(int64_t), hipMemcpyDeviceToHost));
  const double nrow_stats = (double)std::max<int64_t>(opt->n_steps - p.stats_from + 1, 0);
  for (size_t c = 0; c < n; ++c) {
    for (size_t j = 0; j < L; ++j) {
      if (out->mean) out->mean[c * L + j] = (int64_t)j < npar[c] && nrow_stats > 0 ? smean[c * L + j] : NAN;
      if (out->std)
        out->std[c * L + j] = (int64_t)j < npar[c] && nrow_stats > 0 ? std::sqrt(sm2[c * L + j] / nrow_stats) : NAN;
    }
    if (out->sigma_mean) out->sigma_mean[c] = std::sqrt(s2sum[c] / (double)opt->n_steps);
    if (out->sigma_std) out->sigma_std[c] = std::sqrt(sqm2[c] / (double)opt->n_steps);
    if (out->accept_rate) out->accept_rate[c] = opt->n_steps > 1 ? nacc[c] / (double)(opt->n_steps - 1) : 0.0;
    if (out->n_evals) out->n_evals[c] = nev[c];
  }
  if (out->final_theta) TCI_HIP(ctx, hipMemcpy(out->final_theta, st.theta, n * L * sizeof(double), hipMemcpyDeviceToHost));
  if (st.chain_out && out->chain)
    TCI_HIP(ctx, hipMemcpy(out->chain, st.chain_out, (size_t)n_keep * n * L * sizeof(double), hipMemcpyDeviceToHost));
  if (out->qcov_R) {  // the device keeps R as packed FP64 upper triangles
    const int64_t ts = tci::dram_tri_stride((int64_t)L);
    std::vector<double> rd((size_t)n * ts);
    TCI_HIP(ctx, hipMemcpy(rd.data(), st.Rd, rd.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (size_t c = 0; c < n; ++c) {
      double* R = out->qcov_R + c * L2;
      std::fill(R, R + L2, 0.0);
      const int64_t P = npar[c];
      const double* src = rd.data() + c * ts;
      for (int64_t i = 0, e = 0; i < P; ++i)
        for (int64_t j = i; j < P; ++j, ++e) R[i * L + j] = src[e];
    }
  }
  if (st.s2_out && out->s2chain)
    TCI_HIP(ctx, hipMemcpy(out->s2chain, st.s2_out, (size_t)n_keep * n * sizeof(double), hipMemcpyDeviceToHost));
  return TCI_OK;
}

}  // extern "C"
