/* matrix.h -- TEST STAND-IN for MATLAB's mx API (tests/test_mex_shim.py).  Only what
 * matlab/cpk_mex.c uses, with MATLAB's documented semantics: -largeArrayDims index types
 * (mwSize / mwIndex = size_t), column-major real doubles, 0-based CSC for sparse arrays
 * (jc[ncols + 1], ir[nnz]), 1x1 structs, mxSetField taking ownership of the value, mxCalloc'd
 * memory and unreturned arrays freed by the runtime when the MEX call ends (error or not). */
#ifndef CPK_TEST_MATRIX_H
#define CPK_TEST_MATRIX_H
#include <stddef.h>

typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct mxArray_tag mxArray;
typedef enum { mxUNKNOWN_CLASS = 0, mxSTRUCT_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxDOUBLE_CLASS,
               mxUINT64_CLASS, mxFUNCTION_CLASS } mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef unsigned char mxLogical;

int mxIsSparse(const mxArray *a);
int mxIsComplex(const mxArray *a);
int mxIsChar(const mxArray *a);
int mxIsStruct(const mxArray *a);
int mxIsUint64(const mxArray *a);
int mxIsEmpty(const mxArray *a);
int mxIsClass(const mxArray *a, const char *name);
size_t mxGetM(const mxArray *a);
size_t mxGetN(const mxArray *a);
size_t mxGetNumberOfElements(const mxArray *a);
mwIndex *mxGetJc(const mxArray *a);
mwIndex *mxGetIr(const mxArray *a);
double *mxGetPr(const mxArray *a);
void *mxGetData(const mxArray *a);
double mxGetScalar(const mxArray *a);
int mxGetString(const mxArray *a, char *buf, mwSize len);
mxArray *mxGetField(const mxArray *s, mwIndex i, const char *name);
void mxSetField(mxArray *s, mwIndex i, const char *name, mxArray *v);
mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray *mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c);
mxArray *mxCreateDoubleScalar(double v);
mxArray *mxCreateLogicalScalar(mxLogical v);
mxArray *mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char **names);
void mxDestroyArray(mxArray *a);
void *mxCalloc(size_t n, size_t size);
void mxFree(void *p);
#endif
