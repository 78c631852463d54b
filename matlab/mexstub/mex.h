/*
 * mex.h -- builder-written stand-in for MATLAB's MEX API (see matrix.h): the gateway entry point
 * and the three mex* calls matlab/tci_mex.cpp makes. mexErrMsgIdAndTxt ends the MEX call as
 * MATLAB does (here by a C++ exception that mexstub_call catches), so the caller sees the error
 * identifier and message and no output.
 */
#ifndef TCI_MEXSTUB_MEX_H_
#define TCI_MEXSTUB_MEX_H_

#include "matrix.h"

#ifdef __cplusplus
extern "C" {
#endif

/* the gateway every MEX file defines */
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

#ifdef __cplusplus
[[noreturn]]
#endif
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));

#ifdef __cplusplus
}
#endif

#endif /* TCI_MEXSTUB_MEX_H_ */
