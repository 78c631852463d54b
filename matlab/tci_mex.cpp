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
// Errors are raised with mexErrMsgIdAndTxt('tci:...'), carrying tci_last_error().
// Every argument's class and size is checked before a pointer reaches the C ABI. Live contexts
// are tracked; a handle that this MEX file did not create (or already destroyed) is rejected,
// and `clear tci_mex` (mexAtExit) destroys the ones still alive.
#include <stdint.h>
#include <string.h>

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
