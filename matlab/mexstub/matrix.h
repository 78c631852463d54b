/*
 * matrix.h -- a minimal, builder-written stand-in for MATLAB's C Matrix API, just the part
 * matlab/tci_mex.cpp uses. MATLAB and its headers are absent from this build image; this stand-in
 * lets the MEX gateway be compiled and EXECUTED here (tests/test_mex_gateway.py) against the real
 * libtci.so. It is test infrastructure: a MATLAB install builds tci_mex.cpp against its own headers
 * (INTEGRATION.md §2), and nothing here is linked into the product library.
 *
 * Semantics follow the documented MATLAB C API (R2018a interleaved-complex form is irrelevant:
 * only real doubles are used): arrays are column-major, mxGetM/mxGetN are rows/columns of a 2-D
 * array, struct arrays hold one mxArray* per (element, field), mxArrayToString returns storage
 * released with mxFree.
 */
#ifndef TCI_MEXSTUB_MATRIX_H_
#define TCI_MEXSTUB_MATRIX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef size_t mwSize;
typedef size_t mwIndex;
typedef bool mxLogical;

typedef enum {
  mxUNKNOWN_CLASS = 0,
  mxCELL_CLASS,
  mxSTRUCT_CLASS,
  mxLOGICAL_CLASS,
  mxCHAR_CLASS,
  mxVOID_CLASS,
  mxDOUBLE_CLASS,
  mxSINGLE_CLASS,
  mxINT8_CLASS,
  mxUINT8_CLASS,
  mxINT16_CLASS,
  mxUINT16_CLASS,
  mxINT32_CLASS,
  mxUINT32_CLASS,
  mxINT64_CLASS,
  mxUINT64_CLASS
} mxClassID;

typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;

typedef struct mxArray_tag mxArray;

/* queries (mxGetN of an N-D array is the product of its dimensions past the first, as in MATLAB) */
mwSize mxGetNumberOfElements(const mxArray* a);
mwSize mxGetNumberOfDimensions(const mxArray* a);
const mwSize* mxGetDimensions(const mxArray* a);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
bool mxIsDouble(const mxArray* a);
bool mxIsComplex(const mxArray* a);
bool mxIsSparse(const mxArray* a);
bool mxIsUint64(const mxArray* a);
bool mxIsLogical(const mxArray* a);
bool mxIsChar(const mxArray* a);
bool mxIsStruct(const mxArray* a);
mxClassID mxGetClassID(const mxArray* a);

/* data */
void* mxGetData(const mxArray* a);
double* mxGetPr(const mxArray* a);
mxLogical* mxGetLogicals(const mxArray* a);
mxArray* mxGetField(const mxArray* s, mwIndex i, const char* name);
int mxGetNumberOfFields(const mxArray* s);
const char* mxGetFieldNameByNumber(const mxArray* s, int n);
char* mxArrayToString(const mxArray* a);
void mxFree(void* p);

/* creation / destruction */
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity c);
mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID cls, mxComplexity c);
mxArray* mxCreateLogicalMatrix(size_t m, size_t n);
mxArray* mxCreateString(const char* s);
mxArray* mxCreateStructMatrix(size_t m, size_t n, int nfields, const char** names);
void mxSetField(mxArray* s, mwIndex i, const char* name, mxArray* value);
void mxDestroyArray(mxArray* a);

#ifdef __cplusplus
}
#endif

#endif /* TCI_MEXSTUB_MATRIX_H_ */
