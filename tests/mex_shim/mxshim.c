/* mxshim.c -- TEST STAND-IN for the MATLAB runtime around a MEX function (matrix.h, mex.h), so
 * that matlab/cpk_mex.c -- the drop-in boundary's MATLAB side -- can be
 * compiled and driven from tests/test_mex_shim.py without MATLAB.
 *
 * What it emulates:
 *   - mxArrays: real double dense / sparse (CSC, 0-based), char, uint64 and logical scalars,
 *     1x1 structs (mxSetField owns its value), function handles (func2str gives their text);
 *   - a MEX call (shim_call): mexErrMsgIdAndTxt longjmps back to it; when the call ends, error or
 *     not, the runtime destroys every array the call made and did not return in plhs, and frees
 *     its mxCalloc blocks -- MATLAB's rules;
 *   - counters of what stays alive: mxArrays, mxCalloc blocks, and the libcpk matrices and
 *     preconditioners the gateway made (cpk_mex.c is compiled with its cpk_mat_create_csc /
 *     cpk_mat_destroy / cpk_pc_create / cpk_pc_destroy calls renamed to the shim_* wrappers
 *     below, which count and forward).  After an error only the preconditioner handles the test
 *     still owns may remain.
 */
#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cpk.h"
#include "mex.h"

struct mxArray_tag {
    mxClassID cls;
    int sparse;
    size_t m, n, nzmax;
    double *pr;
    uint64_t u64;
    mxLogical lg;
    size_t *ir, *jc;
    char *str;
    int nf;
    char **fnames;
    mxArray **fvals;
    int owned;       /* a struct field (destroyed with its struct) */
    int call_temp;   /* made during the current call */
    mxArray *next_live, *prev_live;
};

static mxArray *g_live = NULL;
static long g_live_arrays = 0, g_live_calloc = 0, g_live_mats = 0, g_live_pcs = 0;
static int g_in_call = 0;
static jmp_buf g_jmp;
static char g_err_id[128], g_err_msg[1024];
static void (*g_atexit)(void) = NULL;
enum { kMaxCalloc = 4096 };
static void *g_calloc[kMaxCalloc];
static int g_ncalloc = 0;

static mxArray *new_array(mxClassID cls, size_t m, size_t n) {
    mxArray *a = calloc(1, sizeof *a);
    a->cls = cls, a->m = m, a->n = n;
    a->call_temp = g_in_call;
    a->next_live = g_live;
    if (g_live) g_live->prev_live = a;
    g_live = a;
    g_live_arrays++;
    return a;
}

void mxDestroyArray(mxArray *a) {
    if (!a) return;
    for (int i = 0; i < a->nf; i++) {
        free(a->fnames[i]);
        if (a->fvals[i]) a->fvals[i]->owned = 0, mxDestroyArray(a->fvals[i]);
    }
    free(a->fnames), free(a->fvals), free(a->pr), free(a->ir), free(a->jc), free(a->str);
    if (a->prev_live) a->prev_live->next_live = a->next_live;
    else g_live = a->next_live;
    if (a->next_live) a->next_live->prev_live = a->prev_live;
    g_live_arrays--;
    free(a);
}

int mxIsSparse(const mxArray *a) { return a && a->sparse; }
int mxIsComplex(const mxArray *a) { (void)a; return 0; }
int mxIsChar(const mxArray *a) { return a && a->cls == mxCHAR_CLASS; }
int mxIsStruct(const mxArray *a) { return a && a->cls == mxSTRUCT_CLASS; }
int mxIsUint64(const mxArray *a) { return a && a->cls == mxUINT64_CLASS; }
int mxIsEmpty(const mxArray *a) { return !a || a->m == 0 || a->n == 0; }
int mxIsClass(const mxArray *a, const char *name) {
    return a && !strcmp(name, "function_handle") && a->cls == mxFUNCTION_CLASS;
}
size_t mxGetM(const mxArray *a) { return a ? a->m : 0; }
size_t mxGetN(const mxArray *a) { return a ? a->n : 0; }
size_t mxGetNumberOfElements(const mxArray *a) { return a ? a->m * a->n : 0; }
mwIndex *mxGetJc(const mxArray *a) { return a->jc; }
mwIndex *mxGetIr(const mxArray *a) { return a->ir; }
double *mxGetPr(const mxArray *a) { return a->pr; }
void *mxGetData(const mxArray *a) {
    if (a->cls == mxUINT64_CLASS) return (void *)&a->u64;
    if (a->cls == mxLOGICAL_CLASS) return (void *)&a->lg;
    return a->pr;
}
double mxGetScalar(const mxArray *a) {
    if (!a) return 0;
    if (a->cls == mxUINT64_CLASS) return (double)a->u64;
    if (a->cls == mxLOGICAL_CLASS) return a->lg;
    return a->pr && (a->m * a->n) != 0 ? a->pr[0] : 0.0;
}
int mxGetString(const mxArray *a, char *buf, mwSize len) {
    if (!a || !a->str || !len) return 1;
    snprintf(buf, len, "%s", a->str);
    return strlen(a->str) + 1 > len;
}
mxArray *mxGetField(const mxArray *s, mwIndex i, const char *name) {
    if (!s || s->cls != mxSTRUCT_CLASS || i != 0) return NULL;
    for (int k = 0; k < s->nf; k++)
        if (!strcmp(s->fnames[k], name)) return s->fvals[k];
    return NULL;
}
void mxSetField(mxArray *s, mwIndex i, const char *name, mxArray *v) {
    if (!s || s->cls != mxSTRUCT_CLASS || i != 0) return;
    for (int k = 0; k < s->nf; k++)
        if (!strcmp(s->fnames[k], name)) {
            if (s->fvals[k]) s->fvals[k]->owned = 0, mxDestroyArray(s->fvals[k]);
            s->fvals[k] = v;
            if (v) v->owned = 1;
            return;
        }
}
mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
    (void)c;
    mxArray *a = new_array(mxDOUBLE_CLASS, m, n);
    a->pr = calloc((m * n) != 0 ? m * n : 1, sizeof(double));
    return a;
}
mxArray *mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c) {
    if (cls == mxDOUBLE_CLASS) return mxCreateDoubleMatrix(m, n, c);
    return new_array(cls, m, n); /* uint64: 1x1 only (the gateway's handles) */
}
mxArray *mxCreateDoubleScalar(double v) {
    mxArray *a = mxCreateDoubleMatrix(1, 1, mxREAL);
    a->pr[0] = v;
    return a;
}
mxArray *mxCreateLogicalScalar(mxLogical v) {
    mxArray *a = new_array(mxLOGICAL_CLASS, 1, 1);
    a->lg = v;
    return a;
}
mxArray *mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char **names) {
    mxArray *a = new_array(mxSTRUCT_CLASS, m, n);
    a->nf = nfields;
    a->fnames = calloc(nfields ? nfields : 1, sizeof(char *));
    a->fvals = calloc(nfields ? nfields : 1, sizeof(mxArray *));
    for (int k = 0; k < nfields; k++) a->fnames[k] = strdup(names[k]);
    return a;
}
void *mxCalloc(size_t n, size_t size) {
    void *p = calloc(n ? n : 1, size ? size : 1);
    if (g_ncalloc < kMaxCalloc) g_calloc[g_ncalloc++] = p;
    g_live_calloc++;
    return p;
}
void mxFree(void *p) {
    if (!p) return;
    for (int i = 0; i < g_ncalloc; i++)
        if (g_calloc[i] == p) {
            g_calloc[i] = g_calloc[--g_ncalloc];
            g_live_calloc--;
            free(p);
            return;
        }
}

void mexErrMsgIdAndTxt(const char *id, const char *fmt, ...) {
    va_list ap;
    snprintf(g_err_id, sizeof g_err_id, "%s", id);
    va_start(ap, fmt);
    vsnprintf(g_err_msg, sizeof g_err_msg, fmt, ap);
    va_end(ap);
    longjmp(g_jmp, 1);
}
int mexAtExit(void (*fn)(void)) {
    g_atexit = fn;
    return 0;
}
int mexCallMATLAB(int nlhs, mxArray *plhs[], int nrhs, mxArray *prhs[], const char *name) {
    if (strcmp(name, "func2str") || nlhs != 1 || nrhs != 1 || !prhs[0] || prhs[0]->cls != mxFUNCTION_CLASS) return 1;
    mxArray *a = new_array(mxCHAR_CLASS, 1, strlen(prhs[0]->str));
    a->str = strdup(prhs[0]->str);
    plhs[0] = a;
    return 0;
}

/* ---- libcpk calls of the gateway, counted (cpk_mex.c is compiled with -D renames) ---------- */
int shim_cpk_mat_create_csc(cpk_ctx ctx, int64_t nrows, int64_t ncols, const size_t *jc, const size_t *ir,
                            const double *pr, cpk_mat *out) {
    const int st = cpk_mat_create_csc(ctx, nrows, ncols, jc, ir, pr, out);
    if (st == CPK_OK) g_live_mats++;
    return st;
}
int shim_cpk_mat_destroy(cpk_mat A) {
    if (A) g_live_mats--;
    return cpk_mat_destroy(A);
}
int shim_cpk_pc_create(cpk_ctx ctx, cpk_mat A11, cpk_mat B, cpk_mat C22, double *ptime, cpk_pc *out) {
    const int st = cpk_pc_create(ctx, A11, B, C22, ptime, out);
    if (st == CPK_OK) g_live_pcs++;
    return st;
}
int shim_cpk_pc_destroy(cpk_pc M) {
    if (M) g_live_pcs--;
    return cpk_pc_destroy(M);
}

/* ---- the test's side --------------------------------------------------------------------- */
mxArray *shim_dense(size_t m, size_t n, const double *pr) {
    mxArray *a = mxCreateDoubleMatrix(m, n, mxREAL);
    if ((m * n) != 0) memcpy(a->pr, pr, m * n * sizeof(double));
    return a;
}
mxArray *shim_sparse(size_t m, size_t n, const size_t *jc, const size_t *ir, const double *pr) {
    mxArray *a = new_array(mxDOUBLE_CLASS, m, n);
    const size_t nnz = jc[n];
    a->sparse = 1, a->nzmax = nnz;
    a->jc = malloc((n + 1) * sizeof(size_t));
    a->ir = malloc((nnz ? nnz : 1) * sizeof(size_t));
    a->pr = malloc((nnz ? nnz : 1) * sizeof(double));
    memcpy(a->jc, jc, (n + 1) * sizeof(size_t));
    if (nnz) memcpy(a->ir, ir, nnz * sizeof(size_t)), memcpy(a->pr, pr, nnz * sizeof(double));
    return a;
}
mxArray *shim_char(const char *s) {
    mxArray *a = new_array(mxCHAR_CLASS, 1, strlen(s));
    a->str = strdup(s);
    return a;
}
mxArray *shim_funchandle(const char *func2str_text) {
    mxArray *a = new_array(mxFUNCTION_CLASS, 1, 1);
    a->str = strdup(func2str_text);
    return a;
}
mxArray *shim_scalar(double v) { return mxCreateDoubleScalar(v); }
mxArray *shim_struct(int nf, const char **names, mxArray **vals) {
    mxArray *s = mxCreateStructMatrix(1, 1, nf, names);
    for (int k = 0; k < nf; k++) mxSetField(s, 0, names[k], vals[k]);
    return s;
}
mxArray *shim_field(const mxArray *s, const char *name) { return mxGetField(s, 0, name); }
int shim_class(const mxArray *a) { return a ? (int)a->cls : -1; }
uint64_t shim_u64(const mxArray *a) { return a && a->cls == mxUINT64_CLASS ? a->u64 : 0; }
int shim_logical(const mxArray *a) { return a && a->cls == mxLOGICAL_CLASS ? a->lg : -1; }
void shim_destroy(mxArray *a) { mxDestroyArray(a); }

/* one MEX call: 0 ok, 1 mexErrMsgIdAndTxt (shim_error_id / shim_error_msg).  Afterwards the
 * runtime's clean-up: the call's mxCalloc blocks and every array it made that is not in plhs */
int shim_call(int nlhs, mxArray **plhs, int nrhs, mxArray **prhs) {
    volatile int rc = 0;
    g_err_id[0] = g_err_msg[0] = '\0';
    for (int i = 0; i < nlhs; i++) plhs[i] = NULL;
    for (mxArray *a = g_live; a; a = a->next_live) a->call_temp = 0;
    g_in_call = 1;
    if (setjmp(g_jmp) == 0) mexFunction(nlhs, plhs, nrhs, (const mxArray **)prhs);
    else rc = 1;
    g_in_call = 0;
    if (rc)
        for (int i = 0; i < nlhs; i++) plhs[i] = NULL; /* an error returns nothing */
    for (int i = 0; i < nlhs; i++)
        if (plhs[i]) plhs[i]->call_temp = 0;
    for (int again = 1; again;) {
        again = 0;
        for (mxArray *a = g_live; a; a = a->next_live)
            if (a->call_temp && !a->owned) {
                mxDestroyArray(a);
                again = 1;
                break;
            }
    }
    while (g_ncalloc > 0) free(g_calloc[--g_ncalloc]), g_live_calloc--;
    return rc;
}
const char *shim_error_id(void) { return g_err_id; }
const char *shim_error_msg(void) { return g_err_msg; }
long shim_live_arrays(void) { return g_live_arrays; }
long shim_live_calloc(void) { return g_live_calloc; }
long shim_live_mats(void) { return g_live_mats; }
long shim_live_pcs(void) { return g_live_pcs; }
/* clear mex: the gateway's mexAtExit (destroys its context) */
void shim_unload(void) {
    if (g_atexit) g_atexit(), g_atexit = NULL;
}
