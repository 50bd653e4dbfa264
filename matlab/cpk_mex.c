/*
 * cpk_mex.c -- MATLAB MEX gateway over libcpk (include/cpk.h).
 *
 * Build on a MATLAB host (not possible in this container):
 *   mex -largeArrayDims -I../include cpk_mex.c -L../cpkrylov_amd -lcpk
 *
 * Commands (first argument is the command string):
 *   h = cpk_mex('pc_create', G, B, Cneg)        % opLDL2(G, B, Cneg)       (opLDL2.m:60-92)
 *       cpk_mex('pc_set', h, opts)              % M.nitref = ... etc.      (opLDL2.m:97-115)
 *   y = cpk_mex('pc_apply', h, x)               % y = M*x                  (opLDL2.m:161-188)
 *   x = cpk_mex('pc_divide', h, b)              % x = Kp*b                 (opLDL2.m:193-195)
 *       cpk_mex('pc_destroy', h)
 *   [x, y, stats, flag] = cpk_mex('method', name, b, A, C, h, opts)
 *                                               % method(b, A, C, M, opts) (kernels/cp*.m)
 *   [x, stats, flag] = cpk_mex('reg_solve', name, b, A, B, C, G, opts)
 *                                               % reg_cpkrylov             (reg_cpkrylov.m:1-180)
 *
 * Errors: every failure becomes mexErrMsgIdAndTxt after the call's temporaries are freed
 * (mexErrMsgIdAndTxt does not return: it unwinds to MATLAB, so the device matrices this call
 * made are tracked in g_tmp and destroyed first); CPK_ERR_INDEFINITE maps to the reference's
 * identifier CPCGLanczos:IndefiniteError.  tests/test_mex_shim.py drives this file against a
 * stand-in of the mx API (tests/mex_shim/) and counts what the error paths leave behind.
 */
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "cpk.h"
#include "mex.h"

static cpk_ctx g_ctx = NULL;

/* device matrices made by the current call: destroyed on every exit, error or not */
enum { kMaxTmp = 8 };
static cpk_mat g_tmp[kMaxTmp];
static int g_ntmp = 0;

static void release_tmp(void) {
    while (g_ntmp > 0) cpk_mat_destroy(g_tmp[--g_ntmp]);
}

static void cleanup(void) {
    release_tmp();
    if (g_ctx) cpk_ctx_destroy(g_ctx), g_ctx = NULL;
}

/* the one error exit: temporaries first, then MATLAB's error (which does not return) */
static void fail_msg(const char *id, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    release_tmp();
    mexErrMsgIdAndTxt(id, "%s", buf);
}

static void fail(int st) {
    char msg[512];
    snprintf(msg, sizeof msg, "%s", cpk_last_error()); /* before release_tmp can touch it */
    fail_msg(st == CPK_ERR_INDEFINITE ? "CPCGLanczos:IndefiniteError" : "cpk:error", "%s", msg);
}

static cpk_ctx ctx(void) {
    if (!g_ctx) {
        int st = cpk_ctx_create(-1, 0, 1, NULL, &g_ctx);
        if (st) fail(st);
        mexAtExit(cleanup);
    }
    return g_ctx;
}

/* MATLAB sparse (CSC, mwIndex = size_t with -largeArrayDims) -> device matrix */
static cpk_mat to_mat(const mxArray *a) {
    cpk_mat M = NULL;
    int st;
    if (!a || !mxIsSparse(a) || mxIsComplex(a)) fail_msg("cpk:args", "expected a real sparse matrix");
    if (g_ntmp == kMaxTmp) fail_msg("cpk:args", "internal: too many temporaries");
    st = cpk_mat_create_csc(ctx(), (int64_t)mxGetM(a), (int64_t)mxGetN(a), (const size_t *)mxGetJc(a),
                            (const size_t *)mxGetIr(a), mxGetPr(a), &M);
    if (st) fail(st);
    g_tmp[g_ntmp++] = M;
    return M;
}

static cpk_pc to_pc(const mxArray *h) {
    if (!h || !mxIsUint64(h) || mxGetNumberOfElements(h) != 1) fail_msg("cpk:args", "bad handle");
    return (cpk_pc)(uintptr_t)(*(uint64_t *)mxGetData(h));
}

/* opts struct -> cpk_opts, honouring isfield() (e.g. cpminres.m:98-111) */
static void to_opts(const mxArray *s, cpk_opts *o) {
    memset(o, 0, sizeof(*o));
    if (!s || !mxIsStruct(s)) return;
#define FIELD(name)                                                      \
    do {                                                                 \
        const mxArray *f = mxGetField(s, 0, #name);                      \
        if (f && !mxIsEmpty(f)) o->name = mxGetScalar(f), o->has_##name = 1; \
    } while (0)
    FIELD(atol); FIELD(rtol); FIELD(btol); FIELD(itmax); FIELD(restart); FIELD(mem); FIELD(print);
    FIELD(nitref); FIELD(itref_tol); FIELD(force_itref); FIELD(residual_update);
#undef FIELD
}

/* @cpminres, 'cpminres' or 'minres'; func2str may also give '@cpminres' or a package-qualified
 * 'pkg.cpminres', so a leading '@' and any prefix up to the last '.' are dropped */
static int method_id(const mxArray *a) {
    static const char *names[] = {"cpcg", "cpcglanczos", "cpminres", "cpsymmlq", "cpgmres", "cpdqgmres"};
    char buf[64];
    const char *nm;
    int i;
    buf[0] = '\0';
    if (!a) fail_msg("cpk:args", "method expected");
    if (mxIsClass(a, "function_handle")) { /* @cpminres -> 'cpminres' */
        mxArray *out = NULL, *in = (mxArray *)a;
        if (mexCallMATLAB(1, &out, 1, &in, "func2str") != 0 || !out) fail_msg("cpk:args", "func2str failed");
        mxGetString(out, buf, sizeof buf);
        mxDestroyArray(out);
    } else if (mxIsChar(a)) {
        mxGetString(a, buf, sizeof buf);
    } else {
        fail_msg("cpk:args", "method must be a function handle or a name");
    }
    nm = buf[0] == '@' ? buf + 1 : buf;
    if (strrchr(nm, '.')) nm = strrchr(nm, '.') + 1;
    for (i = 0; i < 6; i++)
        if (!strcmp(nm, names[i]) || !strcmp(nm, names[i] + 2)) return i;
    fail_msg("cpk:args", "unknown method %s", buf);
    return -1;
}

static mxArray *vec(const double *v, int64_t n) {
    mxArray *a = mxCreateDoubleMatrix((mwSize)n, 1, mxREAL);
    if (n) memcpy(mxGetPr(a), v, (size_t)n * sizeof(double));
    return a;
}

/* stats / flag structs as the reference returns them (cpminres.m:250-252, cpsymmlq.m:363-367) */
static void put_stats(int method, const cpk_stats *st, mxArray **stats, mxArray **flag) {
    const char *sf[] = {"niters", "residHistory", "ptime", "stime"};
    const char *lq[] = {"niters", "cgresidHistory", "lqresidHistory", "qrresidHistory", "ptime", "stime"};
    const char *ff[] = {"solved"};
    if (method == CPK_SYMMLQ) {
        *stats = mxCreateStructMatrix(1, 1, 6, lq);
        mxSetField(*stats, 0, "cgresidHistory", vec(st->hist, st->hist_len));
        mxSetField(*stats, 0, "lqresidHistory", vec(st->hist_lq, st->lq_len));
        mxSetField(*stats, 0, "qrresidHistory", vec(st->hist_qr, st->qr_len));
    } else {
        *stats = mxCreateStructMatrix(1, 1, 4, sf);
        mxSetField(*stats, 0, "residHistory", vec(st->hist, st->hist_len));
    }
    mxSetField(*stats, 0, "niters", mxCreateDoubleScalar((double)st->niters));
    mxSetField(*stats, 0, "ptime", mxCreateDoubleScalar(st->ptime));
    mxSetField(*stats, 0, "stime", mxCreateDoubleScalar(st->stime));
    *flag = mxCreateStructMatrix(1, 1, 1, ff);
    mxSetField(*flag, 0, "solved", mxCreateLogicalScalar(st->solved != 0));
}

/* history buffers of a method call (mxCalloc: MATLAB frees them itself if the call errors) */
static void alloc_hist(cpk_stats *s, int mid, const cpk_opts *o, int64_t n, int64_t m) {
    const double itmax = o->has_itmax ? o->itmax : (double)(mid >= CPK_GMRES ? n + m : n);
    memset(s, 0, sizeof *s);
    s->hist_cap = (int64_t)itmax + 4;
    if (mid == CPK_GMRES) s->hist_cap += o->has_restart ? (int64_t)o->restart : 50;
    s->hist = mxCalloc((size_t)s->hist_cap, sizeof(double));
    s->hist_lq = mxCalloc((size_t)s->hist_cap, sizeof(double));
    s->hist_qr = mxCalloc((size_t)s->hist_cap, sizeof(double));
}
static void free_hist(cpk_stats *s) { mxFree(s->hist), mxFree(s->hist_lq), mxFree(s->hist_qr); }

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
    char cmd[32];
    int st = CPK_OK;
#define ARG(i) ((i) < nrhs ? prhs[i] : NULL)
    g_ntmp = 0;
    if (nrhs < 1 || !mxIsChar(prhs[0])) fail_msg("cpk:args", "cpk_mex: command string expected");
    mxGetString(prhs[0], cmd, sizeof cmd);
    {   /* argument counts before anything is converted or a device is touched */
        static const struct { const char *cmd; int nrhs; } need[] = {
            {"pc_create", 4}, {"pc_set", 3}, {"pc_apply", 3}, {"pc_divide", 3}, {"pc_destroy", 2},
            {"method", 6}, {"reg_solve", 7}};
        int i;
        for (i = 0; i < (int)(sizeof need / sizeof need[0]); i++)
            if (!strcmp(cmd, need[i].cmd) && nrhs < need[i].nrhs)
                fail_msg("cpk:args", "cpk_mex %s: %d arguments expected, %d given", cmd, need[i].nrhs, nrhs);
    }

    if (!strcmp(cmd, "pc_create")) {
        cpk_mat G = to_mat(ARG(1)), B = to_mat(ARG(2)), C = to_mat(ARG(3));
        cpk_pc M = NULL;
        double ptime = 0;
        st = cpk_pc_create(ctx(), G, B, C, &ptime, &M);
        if (st) fail(st);
        release_tmp();
        plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
        *(uint64_t *)mxGetData(plhs[0]) = (uint64_t)(uintptr_t)M;
    } else if (!strcmp(cmd, "pc_set")) {
        cpk_opts o;
        cpk_pc M = to_pc(ARG(1));
        to_opts(ARG(2), &o);
        if ((st = cpk_pc_set(M, &o))) fail(st);
    } else if (!strcmp(cmd, "pc_apply") || !strcmp(cmd, "pc_divide")) {
        cpk_pc M = to_pc(ARG(1));
        cpk_pc_info info;
        if ((st = cpk_pc_get_info(M, &info))) fail(st);
        if (!ARG(2) || mxIsSparse(ARG(2)) || (int64_t)mxGetNumberOfElements(ARG(2)) != info.N)
            fail_msg("cpk:dim", "expected a dense vector of length %lld", (long long)info.N);
        plhs[0] = mxCreateDoubleMatrix((mwSize)info.N, 1, mxREAL);
        st = cmd[3] == 'a' ? cpk_pc_apply(M, mxGetPr(ARG(2)), mxGetPr(plhs[0]))
                           : cpk_pc_divide(M, mxGetPr(ARG(2)), mxGetPr(plhs[0]));
        if (st) fail(st);
    } else if (!strcmp(cmd, "pc_destroy")) {
        cpk_pc_destroy(to_pc(ARG(1)));
    } else if (!strcmp(cmd, "method")) {
        const int mid = method_id(ARG(1));
        cpk_mat A = to_mat(ARG(3)), C = to_mat(ARG(4));
        cpk_pc M = to_pc(ARG(5));
        cpk_opts o;
        cpk_stats s;
        const int64_t n = (int64_t)mxGetM(ARG(3)), m = (int64_t)mxGetM(ARG(4));
        mxArray *x, *y;
        if (!ARG(2) || (int64_t)mxGetNumberOfElements(ARG(2)) != n) fail_msg("cpk:dim", "b must have length %lld", (long long)n);
        to_opts(ARG(6), &o);
        alloc_hist(&s, mid, &o, n, m);
        x = mxCreateDoubleMatrix((mwSize)n, 1, mxREAL);
        y = mxCreateDoubleMatrix((mwSize)m, 1, mxREAL);
        st = cpk_method_solve(ctx(), mid, mxGetPr(ARG(2)), A, C, M, &o, mxGetPr(x), mxGetPr(y), &s);
        if (st) fail(st);
        release_tmp();
        plhs[0] = x, plhs[1] = y;
        put_stats(mid, &s, &plhs[2], &plhs[3]);
        free_hist(&s);
    } else if (!strcmp(cmd, "reg_solve")) {
        const int mid = method_id(ARG(1));
        cpk_mat A = to_mat(ARG(3)), B = to_mat(ARG(4)), C = to_mat(ARG(5)), G = to_mat(ARG(6));
        cpk_opts o;
        cpk_stats s;
        const int64_t n = (int64_t)mxGetM(ARG(3)), m = (int64_t)mxGetM(ARG(4));
        if (!ARG(2) || (int64_t)mxGetNumberOfElements(ARG(2)) != n + m)
            fail_msg("cpk:dim", "b must have length %lld", (long long)(n + m));
        to_opts(ARG(7), &o);
        alloc_hist(&s, mid, &o, n, m);
        plhs[0] = mxCreateDoubleMatrix((mwSize)(n + m), 1, mxREAL);
        st = cpk_reg_solve(ctx(), mid, mxGetPr(ARG(2)), A, B, C, G, &o, mxGetPr(plhs[0]), &s, NULL);
        if (st) fail(st);
        release_tmp();
        put_stats(mid, &s, &plhs[1], &plhs[2]);
        free_hist(&s);
    } else {
        fail_msg("cpk:args", "cpk_mex: unknown command %s", cmd);
    }
#undef ARG
    (void)nlhs;
}
