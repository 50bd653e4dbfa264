/* mex.h -- TEST STAND-IN for MATLAB's MEX API (see matrix.h). */
#ifndef CPK_TEST_MEX_H
#define CPK_TEST_MEX_H
#include "matrix.h"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]);
/* does not return: unwinds to the caller of the MEX function (longjmp in the stand-in) */
void mexErrMsgIdAndTxt(const char *id, const char *fmt, ...) __attribute__((noreturn));
int mexAtExit(void (*fn)(void));
/* the stand-in knows one MATLAB function: func2str of a function handle */
int mexCallMATLAB(int nlhs, mxArray *plhs[], int nrhs, mxArray *prhs[], const char *name);
#endif
