// tci_mex.cpp -- MATLAB MEX gateway over the C ABI in include/tci.h.
//
// The reference's host code is MATLAB; its likelihood hook is mcmcstat's model.ssfun
// (/root/reference/src/TranscriptionCycleMCMC.m:186,258). This gateway is the FFI a MATLAB
// user binds to reach the MI355X kernels. Build (where MATLAB and ROCm are installed):
//
//   mex -R2018a -I../include matlab/tci_mex.cpp -L../transcriptioncycleinference_amd -ltci
//
// Here (no MATLAB) it is compiled against the builder-written stand-in API in matlab/mexstub/ and
// executed by tests/test_mex_gateway.py (transcriptioncycleinference_amd/build.py:build_mex_stub).
//
// Commands (handles are uint64 scalars; cells are 1-based as in MATLAB):
//   h  = tci_mex('create', data, construct, device)
//          data: struct array with fields time, MS2, PP7 (README.md:11-16), already truncated
//          construct: a name ('P2P-MS2v5-LacZ-PP7v4') or a struct with fields
//                     L0, MS2_start, MS2_end, MS2_loopn, PP7_start, PP7_end, PP7_loopn
//   ss = tci_mex('ss', h, cell, x)            one ssfun(x, data) call (x: 1 x P row)
//   ss = tci_mex('ss_batch', h, cells, X)      X: P x B (one theta per COLUMN, no transpose),
//                                               cells: 1 x B; returns B x 1
//   ss = tci_mex('ss_batch', h, cells, X, active)   active: 1 x B logical (false -> +Inf)
//   [ms2, pp7] = tci_mex('forward', h, cell, x, 'raw' | 'interp')
//   tci_mex('destroy', h)
//   n = tci_mex('device_count')                 HIP devices visible to this MATLAB process
//   [results, chain, s2chain, R] = tci_mex('dram', h, cells, X0, LB, UB, MU, SIG, J0, sigma2[, options])
//          mcmcrun (TranscriptionCycleMCMC.m:273) for every chain at once on the GPU (tci_dram_run):
//          one chain per COLUMN. cells: 1 x n; X0 / LB / UB (params, :242-255), MU / SIG (Gaussian
//          priors, SIG = Inf: none, :254) and J0 (the diagonal of options.qcov, :230) are P x n with
//          P >= 7 + N of every chain's cell (rows past a chain's 7 + N are ignored); sigma2: model.sigma2
//          (:259), a scalar or 1 x n. options: mcmcstat's names -- nsimu, burnintime, adaptint, method
//          ('dram' | 'am' | 'dr' | 'mh'), updatesigma, drscale, adascale, qcovadj, burnin_scale -- plus
//          stats_from (first row of the summaries; default burnintime, the reference's n_burn, :276),
//          thin (chain rows kept: 1, 1+thin, ...; default 1 when chain or s2chain is asked for), seed,
//          engine ('auto' | 'fused' | 'walk' | 'batched'), max_chunk, chain_keys (1 x n RNG stream keys)
//          and adapt_pmax; verbosity / waitbar / printint are accepted and ignored.
//          results: struct with mean, std (std(...,1)), final_theta (P x n), sigma_mean, sigma_std
//          (:302-303), accept_rate, n_evals (1 x n) and elapsed_ms; chain: P x n x ceil(nsimu/thin);
//          s2chain: n x ceil(nsimu/thin); R: P x P x n upper factors with R(:,:,k)'*R(:,:,k) the final
//          proposal covariance of chain k (mcmcstat results.qcov).
// Errors are raised with mexErrMsgIdAndTxt('tci:...'), carrying tci_last_error().
// Every argument's class and size is checked before a pointer reaches the C ABI. Live contexts
// are tracked; a handle that this MEX file did not create (or already destroyed) is rejected,
// and `clear tci_mex` (mexAtExit) destroys the ones still alive.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <set>
#include <string>
#include <vector>

#include "mex.h"
#include "tci.h"

namespace {

std::set<tci_ctx*>& live() {
  static std::set<tci_ctx*> s;
  return s;
}

void destroy_all() {
  for (tci_ctx* c : live()) tci_destroy(c);
  live().clear();
}

tci_ctx* handle_of(const mxArray* a) {
  if (!mxIsUint64(a) || mxGetNumberOfElements(a) != 1) mexErrMsgIdAndTxt("tci:handle", "expected a uint64 handle");
  tci_ctx* c = reinterpret_cast<tci_ctx*>(static_cast<uintptr_t>(*static_cast<uint64_t*>(mxGetData(a))));
  if (!live().count(c)) mexErrMsgIdAndTxt("tci:handle", "not a live tci_mex handle");
  return c;
}

// A real double vector of exactly n elements (n < 0: any length).
const double* doubles(const mxArray* a, long long n, const char* what) {
  if (!mxIsDouble(a) || mxIsComplex(a) || mxIsSparse(a)) mexErrMsgIdAndTxt("tci:arg", "%s must be real double", what);
  if (n >= 0 && (long long)mxGetNumberOfElements(a) != n)
    mexErrMsgIdAndTxt("tci:arg", "%s must have %lld elements", what, n);
  return mxGetPr(a);
}

int32_t cell_of(const mxArray* a) {
  const double c = *doubles(a, 1, "cell");
  if (!(c >= 1 && c <= 2147483647.0) || c != (double)(int64_t)c) mexErrMsgIdAndTxt("tci:arg", "cell must be a positive integer");
  return (int32_t)c - 1;
}

void check(tci_ctx* ctx, int rc, const char* what) {
  if (rc != TCI_OK) mexErrMsgIdAndTxt("tci:call", "%s failed (%d): %s", what, rc, tci_last_error(ctx));
}

std::string str_of(const mxArray* a) {
  char* s = mxArrayToString(a);
  if (!s) mexErrMsgIdAndTxt("tci:arg", "expected a character vector");
  std::string r(s);
  mxFree(s);
  return r;
}

std::vector<double> field_vec(const mxArray* s, mwIndex i, const char* name) {
  const mxArray* f = mxGetField(s, i, name);
  if (!f || !mxIsDouble(f)) mexErrMsgIdAndTxt("tci:data", "field %s missing or not double", name);
  const double* p = mxGetPr(f);
  return std::vector<double>(p, p + mxGetNumberOfElements(f));
}

void cmd_create(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs < 3) mexErrMsgIdAndTxt("tci:arg", "tci_mex('create', data, construct[, device])");
  const mxArray* data = prhs[1];
  if (!mxIsStruct(data)) mexErrMsgIdAndTxt("tci:data", "data must be a struct array (README.md:11-16)");
  const mwSize C = mxGetNumberOfElements(data);
  std::vector<int64_t> off(1, 0);
  std::vector<double> t, m, p;
  for (mwIndex i = 0; i < C; ++i) {
    std::vector<double> ti = field_vec(data, i, "time"), mi = field_vec(data, i, "MS2"), pi = field_vec(data, i, "PP7");
    if (mi.size() != ti.size() || pi.size() != ti.size())
      mexErrMsgIdAndTxt("tci:data", "cell %d: time, MS2, PP7 lengths differ", (int)i + 1);
    t.insert(t.end(), ti.begin(), ti.end());
    m.insert(m.end(), mi.begin(), mi.end());
    p.insert(p.end(), pi.begin(), pi.end());
    off.push_back((int64_t)t.size());
  }
  tci_construct cs;
  std::vector<double> seg[6];
  if (mxIsChar(prhs[2])) {
    if (tci_construct_by_name(str_of(prhs[2]).c_str(), &cs) != TCI_OK)
      mexErrMsgIdAndTxt("tci:construct", "construct is not defined (GetFluorFromPolPos.m:18)");
  } else if (mxIsStruct(prhs[2])) {
    const char* names[6] = {"MS2_start", "MS2_end", "MS2_loopn", "PP7_start", "PP7_end", "PP7_loopn"};
    if (mxGetNumberOfElements(prhs[2]) != 1) mexErrMsgIdAndTxt("tci:construct", "construct must be a 1x1 struct");
    for (int k = 0; k < 6; ++k) seg[k] = field_vec(prhs[2], 0, names[k]);
    for (int k = 1; k < 6; ++k)
      if (seg[k].size() != seg[0].size())
        mexErrMsgIdAndTxt("tci:construct", "%s and %s must have the same number of segments", names[k], names[0]);
    const std::vector<double> L0 = field_vec(prhs[2], 0, "L0");
    if (L0.size() != 1) mexErrMsgIdAndTxt("tci:construct", "L0 must be a scalar");
    cs.L0 = L0[0];
    cs.n_seg = (int32_t)seg[0].size();
    cs.ms2_start = seg[0].data();
    cs.ms2_end = seg[1].data();
    cs.ms2_loopn = seg[2].data();
    cs.pp7_start = seg[3].data();
    cs.pp7_end = seg[4].data();
    cs.pp7_loopn = seg[5].data();
  } else {
    mexErrMsgIdAndTxt("tci:construct", "construct must be a name or a struct");
  }
  const int device = nrhs > 3 ? (int)*doubles(prhs[3], 1, "device") : 0;
  tci_cells cells{(int64_t)C, off.data(), t.data(), m.data(), p.data()};
  tci_ctx* ctx = nullptr;
  const int rc = tci_create(&cells, &cs, device, &ctx);
  if (rc != TCI_OK) {
    std::string msg = ctx ? tci_last_error(ctx) : "tci_create failed";
    if (ctx) tci_destroy(ctx);
    mexErrMsgIdAndTxt("tci:create", "%s", msg.c_str());
  }
  live().insert(ctx);
  plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
  *static_cast<uint64_t*>(mxGetData(plhs[0])) = static_cast<uint64_t>(reinterpret_cast<uintptr_t>(ctx));
  (void)nlhs;
}

void cmd_ss(mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs != 4) mexErrMsgIdAndTxt("tci:arg", "tci_mex('ss', h, cell, x)");
  tci_ctx* ctx = handle_of(prhs[1]);
  const int32_t cell = cell_of(prhs[2]);
  const double* x = doubles(prhs[3], -1, "x");
  double ss = 0;
  check(ctx, tci_ssfun(ctx, cell, x, (int64_t)mxGetNumberOfElements(prhs[3]), &ss), "tci_ssfun");
  plhs[0] = mxCreateDoubleScalar(ss);
}

void cmd_ss_batch(mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs < 4) mexErrMsgIdAndTxt("tci:arg", "tci_mex('ss_batch', h, cells, X[, active])");
  tci_ctx* ctx = handle_of(prhs[1]);
  const mwSize B = mxGetNumberOfElements(prhs[2]);
  const double* c = doubles(prhs[2], -1, "cells");
  doubles(prhs[3], -1, "X");
  if (mxGetNumberOfDimensions(prhs[3]) != 2 || mxGetN(prhs[3]) != B)
    mexErrMsgIdAndTxt("tci:arg", "X must be P x B (one theta per column)");
  const int64_t P = (int64_t)mxGetM(prhs[3]);  // column-major P x B == row-major B x P
  std::vector<int32_t> cid(B);
  for (mwSize b = 0; b < B; ++b) {
    if (!(c[b] >= 1 && c[b] <= 2147483647.0) || c[b] != (double)(int64_t)c[b])
      mexErrMsgIdAndTxt("tci:arg", "cells(%d) must be a positive integer", (int)b + 1);
    cid[b] = (int32_t)c[b] - 1;
  }
  std::vector<uint8_t> act;
  if (nrhs > 4) {  // logical mask, or a double 0/1 vector (nonzero = active)
    if (mxGetNumberOfElements(prhs[4]) != B) mexErrMsgIdAndTxt("tci:arg", "active must have B elements");
    if (mxIsLogical(prhs[4])) {
      const mxLogical* a = mxGetLogicals(prhs[4]);
      act.resize(B);
      for (mwSize b = 0; b < B; ++b) act[b] = a[b] ? 1 : 0;
    } else {
      const double* a = doubles(prhs[4], (long long)B, "active");
      act.resize(B);
      for (mwSize b = 0; b < B; ++b) act[b] = a[b] != 0.0 ? 1 : 0;
    }
  }
  plhs[0] = mxCreateDoubleMatrix(B, 1, mxREAL);
  check(ctx, tci_ss_batch(ctx, mxGetPr(prhs[3]), P, cid.data(), act.empty() ? nullptr : act.data(), (int64_t)B,
                          mxGetPr(plhs[0])), "tci_ss_batch");
}

void cmd_forward(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs < 4) mexErrMsgIdAndTxt("tci:arg", "tci_mex('forward', h, cell, x[, 'raw'|'interp'])");
  tci_ctx* ctx = handle_of(prhs[1]);
  const int32_t cell = cell_of(prhs[2]);
  const double* x = doubles(prhs[3], -1, "x");
  const int mode = (nrhs > 4 && str_of(prhs[4]) == "interp") ? TCI_GRID_INTERP : TCI_GRID_RAW;
  int64_t n = 0;
  check(ctx, tci_cell_points(ctx, cell, &n), "tci_cell_points");
  plhs[0] = mxCreateDoubleMatrix(1, (mwSize)n, mxREAL);
  mxArray* pp7 = mxCreateDoubleMatrix(1, (mwSize)n, mxREAL);
  check(ctx, tci_forward(ctx, x, (int64_t)mxGetNumberOfElements(prhs[3]), &cell, 1, mode,
                         mxGetPr(plhs[0]), mxGetPr(pp7), n), "tci_forward");
  if (nlhs > 1) plhs[1] = pp7; else mxDestroyArray(pp7);
}

// ---- 'dram': the GPU-resident sampler -------------------------------------------------------

double opt_num(const mxArray* o, const char* name, double def) {
  const mxArray* f = o ? mxGetField(o, 0, name) : nullptr;
  if (!f) return def;
  if (!mxIsDouble(f) && !mxIsLogical(f)) mexErrMsgIdAndTxt("tci:opts", "options.%s must be numeric", name);
  if (mxGetNumberOfElements(f) != 1) mexErrMsgIdAndTxt("tci:opts", "options.%s must be a scalar", name);
  return mxIsLogical(f) ? (mxGetLogicals(f)[0] ? 1.0 : 0.0) : mxGetPr(f)[0];
}

int64_t opt_int(const mxArray* o, const char* name, int64_t def, int64_t lo) {
  const double v = opt_num(o, name, (double)def);
  if (!(v >= (double)lo && v <= 9.0e15) || v != (double)(int64_t)v)
    mexErrMsgIdAndTxt("tci:opts", "options.%s must be an integer >= %lld", name, (long long)lo);
  return (int64_t)v;
}

std::string opt_str(const mxArray* o, const char* name, const char* def) {
  const mxArray* f = o ? mxGetField(o, 0, name) : nullptr;
  if (!f) return def;
  if (!mxIsChar(f)) mexErrMsgIdAndTxt("tci:opts", "options.%s must be a character vector", name);
  std::string r = str_of(f);
  for (char& ch : r) ch = (char)((ch >= 'A' && ch <= 'Z') ? ch - 'A' + 'a' : ch);
  return r;
}

// A P x n real double matrix (one chain per column).
const double* chain_matrix(const mxArray* a, const char* what, size_t P, size_t n) {
  if (!mxIsDouble(a) || mxIsComplex(a) || mxIsSparse(a)) mexErrMsgIdAndTxt("tci:arg", "%s must be real double", what);
  if (mxGetNumberOfDimensions(a) != 2 || mxGetM(a) != P || mxGetN(a) != n)
    mexErrMsgIdAndTxt("tci:arg", "%s must be %d x %d (one chain per column, as X0)", what, (int)P, (int)n);
  return mxGetPr(a);
}

void cmd_dram(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs < 10 || nrhs > 11)
    mexErrMsgIdAndTxt("tci:arg", "tci_mex('dram', h, cells, X0, LB, UB, MU, SIG, J0, sigma2[, options])");
  // every argument and option is checked before the handle (and before anything reaches the GPU)
  const size_t n = mxGetNumberOfElements(prhs[2]);
  const double* c = doubles(prhs[2], -1, "cells");
  if (n == 0) mexErrMsgIdAndTxt("tci:arg", "cells must name at least one chain's cell");
  if (!mxIsDouble(prhs[3]) || mxGetNumberOfDimensions(prhs[3]) != 2 || mxGetN(prhs[3]) != n)
    mexErrMsgIdAndTxt("tci:arg", "X0 must be P x n: one chain per column, n = numel(cells)");
  const size_t P = mxGetM(prhs[3]);
  if (P < 7) mexErrMsgIdAndTxt("tci:arg", "X0 must have at least 7 rows ([v, tau, ton, MS2_basal, PP7_basal, A, R, dR])");
  const char* names[6] = {"X0", "LB", "UB", "MU", "SIG", "J0"};
  const double* in[6];
  for (int k = 0; k < 6; ++k) in[k] = chain_matrix(prhs[3 + k], names[k], P, n);
  const size_t ns2 = mxGetNumberOfElements(prhs[9]);
  const double* s2 = doubles(prhs[9], -1, "sigma2");
  if (ns2 != 1 && ns2 != n) mexErrMsgIdAndTxt("tci:arg", "sigma2 must be a scalar or have one entry per chain");
  std::vector<int32_t> cid(n);
  for (size_t b = 0; b < n; ++b) {
    if (!(c[b] >= 1 && c[b] <= 2147483647.0) || c[b] != (double)(int64_t)c[b])
      mexErrMsgIdAndTxt("tci:arg", "cells(%d) must be a positive integer", (int)b + 1);
    cid[b] = (int32_t)c[b] - 1;
  }
  std::vector<double> s2v(n);
  for (size_t b = 0; b < n; ++b) s2v[b] = s2[ns2 == 1 ? 0 : b];

  // options: mcmcstat's names (TranscriptionCycleMCMC.m:263-270), unknown fields refused
  const mxArray* o = nullptr;
  if (nrhs > 10 && !(mxIsDouble(prhs[10]) && mxGetNumberOfElements(prhs[10]) == 0)) {  // [] = defaults
    if (!mxIsStruct(prhs[10]) || mxGetNumberOfElements(prhs[10]) != 1)
      mexErrMsgIdAndTxt("tci:opts", "options must be a 1x1 struct");
    o = prhs[10];
    static const char* known[] = {"nsimu", "burnintime", "adaptint", "method", "updatesigma", "drscale", "adascale",
                                  "qcovadj", "burnin_scale", "stats_from", "thin", "seed", "engine", "max_chunk",
                                  "chain_keys", "adapt_pmax", "verbosity", "waitbar", "printint"};
    for (int f = 0; f < mxGetNumberOfFields(o); ++f) {
      const char* fn = mxGetFieldNameByNumber(o, f);
      bool ok = false;
      for (const char* k : known) ok = ok || strcmp(fn, k) == 0;
      if (!ok && strcmp(fn, "qcov") == 0)
        mexErrMsgIdAndTxt("tci:opts", "options.qcov: pass the initial proposal variances as J0 (P x n)");
      if (!ok) mexErrMsgIdAndTxt("tci:opts", "options.%s is not an option of tci_mex('dram')", fn);
    }
  }
  tci_dram_options opt;
  tci_dram_defaults(&opt);
  opt.n_steps = opt_int(o, "nsimu", opt.n_steps, 1);
  opt.burnintime = opt_int(o, "burnintime", opt.burnintime, 0);
  opt.adaptint = opt_int(o, "adaptint", opt.adaptint, 0);
  const std::string method = opt_str(o, "method", "dram");  // mcmcstat: mh, am, dr, dram
  if (method == "dram" || method == "am") {
    opt.ntry = method == "dram" ? 2 : 1;
  } else if (method == "dr" || method == "mh") {
    opt.ntry = method == "dr" ? 2 : 1;
    opt.adaptint = 0;
  } else {
    mexErrMsgIdAndTxt("tci:opts", "options.method must be 'dram', 'am', 'dr' or 'mh'");
  }
  opt.updatesigma = opt_num(o, "updatesigma", opt.updatesigma) != 0.0 ? 1 : 0;
  opt.drscale = opt_num(o, "drscale", opt.drscale);
  opt.adascale = opt_num(o, "adascale", opt.adascale);
  opt.qcovadj = opt_num(o, "qcovadj", opt.qcovadj);
  opt.burnin_scale = opt_num(o, "burnin_scale", opt.burnin_scale);
  opt.stats_from = opt_int(o, "stats_from", std::max<int64_t>(opt.burnintime, 1), 1);
  const bool want_chain = nlhs >= 2;
  const int64_t thin = opt_int(o, "thin", 1, 0);
  opt.thin = want_chain ? thin : 0;
  opt.seed = (uint64_t)opt_int(o, "seed", (int64_t)opt.seed, 0);
  const std::string engine = opt_str(o, "engine", "auto");
  if (engine == "auto") opt.engine = TCI_DRAM_AUTO;
  else if (engine == "fused") opt.engine = TCI_DRAM_FUSED;
  else if (engine == "batched") opt.engine = TCI_DRAM_BATCHED;
  else if (engine == "walk") opt.engine = TCI_DRAM_WALK;
  else mexErrMsgIdAndTxt("tci:opts", "options.engine must be 'auto', 'fused', 'walk' or 'batched'");
  opt.max_chunk = (int32_t)opt_int(o, "max_chunk", 0, 0);
  opt.adapt_pmax = opt_int(o, "adapt_pmax", 0, 0);
  std::vector<int64_t> keys;
  if (const mxArray* k = o ? mxGetField(o, 0, "chain_keys") : nullptr) {
    const double* kv = doubles(k, (long long)n, "options.chain_keys");
    keys.resize(n);
    for (size_t b = 0; b < n; ++b) {
      if (!(kv[b] >= 0 && kv[b] <= 9.0e15) || kv[b] != (double)(int64_t)kv[b])
        mexErrMsgIdAndTxt("tci:opts", "options.chain_keys(%d) must be a non-negative integer", (int)b + 1);
      keys[b] = (int64_t)kv[b];
    }
    opt.chain_keys = keys.data();
  }

  tci_ctx* ctx = handle_of(prhs[1]);
  // outputs, written in place: the ABI's row-major [chain][P] is MATLAB's column-major P x n
  static const char* fields[] = {"mean", "std", "final_theta", "sigma_mean", "sigma_std", "accept_rate", "n_evals",
                                 "elapsed_ms"};
  mxArray* res = mxCreateStructMatrix(1, 1, 8, fields);
  mxArray* pn[6];
  for (int k = 0; k < 3; ++k) pn[k] = mxCreateDoubleMatrix(P, n, mxREAL);
  for (int k = 3; k < 6; ++k) pn[k] = mxCreateDoubleMatrix(1, n, mxREAL);
  for (int k = 0; k < 6; ++k) mxSetField(res, 0, fields[k], pn[k]);
  std::vector<int64_t> nev(n);
  tci_dram_outputs out;
  memset(&out, 0, sizeof out);
  out.mean = mxGetPr(pn[0]);
  out.std = mxGetPr(pn[1]);
  out.final_theta = mxGetPr(pn[2]);
  out.sigma_mean = mxGetPr(pn[3]);
  out.sigma_std = mxGetPr(pn[4]);
  out.accept_rate = mxGetPr(pn[5]);
  out.n_evals = nev.data();
  const size_t n_keep = opt.thin > 0 ? (size_t)((opt.n_steps + opt.thin - 1) / opt.thin) : 0;
  mxArray* ch = nullptr;
  mxArray* s2c = nullptr;
  if (want_chain) {
    const mwSize d3[3] = {P, n, n_keep};
    ch = mxCreateNumericArray(3, d3, mxDOUBLE_CLASS, mxREAL);  // P x n x n_keep == [row][chain][P]
    s2c = mxCreateDoubleMatrix(n, n_keep, mxREAL);            // n x n_keep == [row][chain]
    if (n_keep) {
      out.chain = mxGetPr(ch);
      out.s2chain = mxGetPr(s2c);
    }
  }
  std::vector<double> rbuf;
  if (nlhs >= 4) {
    rbuf.resize(n * P * P);
    out.qcov_R = rbuf.data();
  }
  const int rc = tci_dram_run(ctx, &opt, (int64_t)n, cid.data(), in[0], in[1], in[2], in[3], in[4], in[5], s2v.data(),
                              (int64_t)P, &out);
  if (rc != TCI_OK) {
    mxDestroyArray(res);
    if (ch) mxDestroyArray(ch);
    if (s2c) mxDestroyArray(s2c);
    check(ctx, rc, "tci_dram_run");
  }
  mxArray* ne = mxCreateDoubleMatrix(1, n, mxREAL);
  for (size_t b = 0; b < n; ++b) mxGetPr(ne)[b] = (double)nev[b];
  mxSetField(res, 0, "n_evals", ne);
  mxSetField(res, 0, "elapsed_ms", mxCreateDoubleScalar(out.elapsed_ms));
  plhs[0] = res;
  if (nlhs >= 2) plhs[1] = ch;
  if (nlhs >= 3) plhs[2] = s2c;
  else if (s2c) mxDestroyArray(s2c);
  if (nlhs >= 4) {  // [chain][i][j] (upper) -> R(i, j, chain): MATLAB's column-major
    const mwSize d3[3] = {P, P, n};
    mxArray* R = mxCreateNumericArray(3, d3, mxDOUBLE_CLASS, mxREAL);
    double* r = mxGetPr(R);
    for (size_t k = 0; k < n; ++k)
      for (size_t i = 0; i < P; ++i)
        for (size_t j = 0; j < P; ++j) r[k * P * P + j * P + i] = rbuf[k * P * P + i * P + j];
    plhs[3] = R;
  }
}

}  // namespace

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  static bool at_exit = false;
  if (!at_exit) {
    mexAtExit(destroy_all);
    at_exit = true;
  }
  if (nrhs < 1 || !mxIsChar(prhs[0])) mexErrMsgIdAndTxt("tci:arg", "first argument must be a command");
  const std::string cmd = str_of(prhs[0]);
  if (cmd == "create") cmd_create(nlhs, plhs, nrhs, prhs);
  else if (cmd == "ss") cmd_ss(plhs, nrhs, prhs);
  else if (cmd == "ss_batch") cmd_ss_batch(plhs, nrhs, prhs);
  else if (cmd == "forward") cmd_forward(nlhs, plhs, nrhs, prhs);
  else if (cmd == "dram") cmd_dram(nlhs, plhs, nrhs, prhs);
  else if (cmd == "device_count") {
    int n = 0;
    tci_device_count(&n);
    plhs[0] = mxCreateDoubleScalar((double)n);
  }
  else if (cmd == "destroy") {
    if (nrhs > 1) {
      tci_ctx* c = handle_of(prhs[1]);
      live().erase(c);
      tci_destroy(c);
    }
  }
  else mexErrMsgIdAndTxt("tci:arg", "unknown command '%s'", cmd.c_str());
}
