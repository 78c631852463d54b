// mexstub.cpp -- the stand-in MATLAB C/MEX API of mex.h / matrix.h, plus a small harness API
// (mexstub_*) through which tests/test_mex_gateway.py builds MATLAB values, calls the gateway's
// mexFunction and reads the results. Test infrastructure only (see matrix.h).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "mex.h"

struct mxArray_tag {
  mxClassID cls = mxUNKNOWN_CLASS;
  size_t m = 0, n = 0;                // rows, and the product of the dimensions past the first
  std::vector<size_t> dims;           // every dimension (at least two)
  bool complex = false;
  std::vector<unsigned char> data;    // numeric / logical / char payload, column-major
  std::vector<std::string> fields;    // struct field names
  std::vector<mxArray*> elems;        // struct values: element-major, elems[i * nfields + f]
};

namespace {

size_t elem_size(mxClassID c) {
  switch (c) {
    case mxDOUBLE_CLASS: case mxINT64_CLASS: case mxUINT64_CLASS: return 8;
    case mxSINGLE_CLASS: case mxINT32_CLASS: case mxUINT32_CLASS: return 4;
    case mxINT16_CLASS: case mxUINT16_CLASS: return 2;
    case mxLOGICAL_CLASS: case mxCHAR_CLASS: case mxINT8_CLASS: case mxUINT8_CLASS: return 1;
    default: return 0;
  }
}

mxArray* make(mxClassID c, size_t m, size_t n) {
  mxArray* a = new mxArray_tag();
  a->cls = c;
  a->m = m;
  a->n = n;
  a->dims = {m, n};
  a->data.assign(m * n * elem_size(c), 0);
  return a;
}

struct MexError : std::runtime_error {
  std::string id;
  MexError(const std::string& i, const std::string& msg) : std::runtime_error(msg), id(i) {}
};

std::string g_err_id, g_err_msg;
std::vector<void (*)(void)> g_at_exit;

}  // namespace

extern "C" {

mwSize mxGetNumberOfElements(const mxArray* a) { return a->m * a->n; }
mwSize mxGetNumberOfDimensions(const mxArray* a) { return a->dims.size(); }
const mwSize* mxGetDimensions(const mxArray* a) { return a->dims.data(); }
size_t mxGetM(const mxArray* a) { return a->m; }
size_t mxGetN(const mxArray* a) { return a->n; }
bool mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
bool mxIsComplex(const mxArray* a) { return a->complex; }
bool mxIsSparse(const mxArray*) { return false; }
bool mxIsUint64(const mxArray* a) { return a->cls == mxUINT64_CLASS; }
bool mxIsLogical(const mxArray* a) { return a->cls == mxLOGICAL_CLASS; }
bool mxIsChar(const mxArray* a) { return a->cls == mxCHAR_CLASS; }
bool mxIsStruct(const mxArray* a) { return a->cls == mxSTRUCT_CLASS; }
mxClassID mxGetClassID(const mxArray* a) { return a->cls; }

void* mxGetData(const mxArray* a) { return a->data.empty() ? nullptr : (void*)a->data.data(); }
double* mxGetPr(const mxArray* a) { return a->cls == mxDOUBLE_CLASS ? (double*)mxGetData(a) : nullptr; }
mxLogical* mxGetLogicals(const mxArray* a) { return a->cls == mxLOGICAL_CLASS ? (mxLogical*)mxGetData(a) : nullptr; }

mxArray* mxGetField(const mxArray* s, mwIndex i, const char* name) {
  if (s->cls != mxSTRUCT_CLASS || i >= s->m * s->n) return nullptr;
  for (size_t f = 0; f < s->fields.size(); ++f)
    if (s->fields[f] == name) return s->elems[i * s->fields.size() + f];
  return nullptr;
}

int mxGetNumberOfFields(const mxArray* s) { return s->cls == mxSTRUCT_CLASS ? (int)s->fields.size() : 0; }
const char* mxGetFieldNameByNumber(const mxArray* s, int n) {
  return s->cls == mxSTRUCT_CLASS && n >= 0 && n < (int)s->fields.size() ? s->fields[n].c_str() : nullptr;
}

char* mxArrayToString(const mxArray* a) {
  if (a->cls != mxCHAR_CLASS) return nullptr;
  char* s = (char*)malloc(a->data.size() + 1);
  memcpy(s, a->data.data(), a->data.size());
  s[a->data.size()] = 0;
  return s;
}
void mxFree(void* p) { free(p); }

mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity) { return make(mxDOUBLE_CLASS, m, n); }
mxArray* mxCreateDoubleScalar(double v) {
  mxArray* a = make(mxDOUBLE_CLASS, 1, 1);
  memcpy(a->data.data(), &v, 8);
  return a;
}
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity) { return make(cls, m, n); }
mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID cls, mxComplexity) {
  // trailing singleton dimensions are dropped down to two, as MATLAB does
  std::vector<size_t> d(dims, dims + ndim);
  while (d.size() > 2 && d.back() == 1) d.pop_back();
  while (d.size() < 2) d.push_back(d.empty() ? 0 : 1);
  size_t rest = 1;
  for (size_t k = 1; k < d.size(); ++k) rest *= d[k];
  mxArray* a = make(cls, d[0], rest);
  a->dims = d;
  return a;
}
mxArray* mxCreateLogicalMatrix(size_t m, size_t n) { return make(mxLOGICAL_CLASS, m, n); }
mxArray* mxCreateString(const char* s) {
  const size_t k = strlen(s);
  mxArray* a = make(mxCHAR_CLASS, k ? 1 : 0, k);
  memcpy(a->data.data(), s, k);
  return a;
}
mxArray* mxCreateStructMatrix(size_t m, size_t n, int nfields, const char** names) {
  mxArray* a = make(mxSTRUCT_CLASS, m, n);
  for (int f = 0; f < nfields; ++f) a->fields.push_back(names[f]);
  a->elems.assign(m * n * (size_t)nfields, nullptr);
  return a;
}
void mxSetField(mxArray* s, mwIndex i, const char* name, mxArray* value) {
  for (size_t f = 0; f < s->fields.size(); ++f)
    if (s->fields[f] == name) {
      mxArray*& slot = s->elems[i * s->fields.size() + f];
      if (slot) mxDestroyArray(slot);
      slot = value;
      return;
    }
}
void mxDestroyArray(mxArray* a) {
  if (!a) return;
  for (mxArray* e : a->elems) mxDestroyArray(e);
  delete a;
}

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  throw MexError(id, buf);
}
int mexAtExit(void (*fn)(void)) {
  for (auto f : g_at_exit)
    if (f == fn) return 0;
  g_at_exit.push_back(fn);
  return 0;
}

// ---- harness API (tests/test_mex_gateway.py) ------------------------------------------------

// One MATLAB call [plhs{1:nlhs}] = tci_mex(prhs{:}). Returns 0, or 1 after mexErrMsgIdAndTxt
// (id / message in mexstub_error_id / mexstub_error_msg), or 2 after any other C++ exception.
int mexstub_call(int nlhs, mxArray** plhs, int nrhs, const mxArray** prhs) {
  g_err_id.clear();
  g_err_msg.clear();
  for (int i = 0; i < nlhs; ++i) plhs[i] = nullptr;
  try {
    mexFunction(nlhs, plhs, nrhs, prhs);
  } catch (const MexError& e) {
    g_err_id = e.id;
    g_err_msg = e.what();
    return 1;
  } catch (const std::exception& e) {
    g_err_id = "mexstub:exception";
    g_err_msg = e.what();
    return 2;
  }
  return 0;
}
const char* mexstub_error_id(void) { return g_err_id.c_str(); }
const char* mexstub_error_msg(void) { return g_err_msg.c_str(); }
// `clear tci_mex`: the functions registered with mexAtExit, then forget them
void mexstub_clear(void) {
  for (auto f : g_at_exit) f();
  g_at_exit.clear();
}
// uint64 scalar (a handle) of an mxArray
uint64_t mexstub_uint64(const mxArray* a) { return a->cls == mxUINT64_CLASS ? *(const uint64_t*)a->data.data() : 0; }
mxArray* mexstub_make_uint64(uint64_t v) {
  mxArray* a = make(mxUINT64_CLASS, 1, 1);
  memcpy(a->data.data(), &v, 8);
  return a;
}

}  // extern "C"
