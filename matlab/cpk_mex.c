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
 * Errors: every libcpk failure becomes mexErrMsgIdAndTxt after the call's temporaries are
 * freed; CPK_ERR_INDEFINITE maps to the reference's identifier CPCGLanczos:IndefiniteError.
 */
#include <stdint.h>
#include <string.h>

#include "cpk.h"
#include "mex.h"

static cpk_ctx g_ctx = NULL;

static void cleanup(void) {
    if (g_ctx) cpk_ctx_destroy(g_ctx), g_ctx = NULL;
}

static void fail(int st) {
    const char *id = st == CPK_ERR_INDEFINITE ? "CPCGLanczos:IndefiniteError" : "cpk:error";
    mexErrMsgIdAndTxt(id, "%s", cpk_last_error());
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
    if (!mxIsSparse(a) || mxIsComplex(a)) mexErrMsgIdAndTxt("cpk:args", "expected a real sparse matrix");
    st = cpk_mat_create_csc(ctx(), (int64_t)mxGetM(a), (int64_t)mxGetN(a), (const size_t *)mxGetJc(a),
                            (const size_t *)mxGetIr(a), mxGetPr(a), &M);
    if (st) fail(st);
    return M;
}

static cpk_pc to_pc(const mxArray *h) {
    if (!mxIsUint64(h) || mxGetNumberOfElements(h) != 1) mexErrMsgIdAndTxt("cpk:args", "bad handle");
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

static int method_id(const mxArray *a) {
    static const char *names[] = {"cpcg", "cpcglanczos", "cpminres", "cpsymmlq", "cpgmres", "cpdqgmres"};
    char buf[32];
    int i;
    if (mxIsClass(a, "function_handle")) {  /* @cpminres -> 'cpminres' */
        mxArray *out = NULL, *in = (mxArray *)a;
        mexCallMATLAB(1, &out, 1, &in, "func2str");
        mxGetString(out, buf, sizeof buf);
        mxDestroyArray(out);
    } else {
        mxGetString(a, buf, sizeof buf);
    }
    for (i = 0; i < 6; i++)
        if (!strcmp(buf, names[i]) || !strcmp(buf, names[i] + 2)) return i;
    mexErrMsgIdAndTxt("cpk:args", "unknown method %s", buf);
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

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
    char cmd[32];
    int st = CPK_OK;
    if (nrhs < 1 || !mxIsChar(prhs[0])) mexErrMsgIdAndTxt("cpk:args", "cpk_mex: command string expected");
    mxGetString(prhs[0], cmd, sizeof cmd);

    if (!strcmp(cmd, "pc_create")) {
        cpk_mat G = to_mat(prhs[1]), B = to_mat(prhs[2]), C = to_mat(prhs[3]);
        cpk_pc M = NULL;
        double ptime = 0;
        st = cpk_pc_create(ctx(), G, B, C, &ptime, &M);
        cpk_mat_destroy(G), cpk_mat_destroy(B), cpk_mat_destroy(C);
        if (st) fail(st);
        plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
        *(uint64_t *)mxGetData(plhs[0]) = (uint64_t)(uintptr_t)M;
    } else if (!strcmp(cmd, "pc_set")) {
        cpk_opts o;
        to_opts(prhs[2], &o);
        if ((st = cpk_pc_set(to_pc(prhs[1]), &o))) fail(st);
    } else if (!strcmp(cmd, "pc_apply") || !strcmp(cmd, "pc_divide")) {
        cpk_pc M = to_pc(prhs[1]);
        cpk_pc_info info;
        if ((st = cpk_pc_get_info(M, &info))) fail(st);
        if ((int64_t)mxGetNumberOfElements(prhs[2]) != info.N) mexErrMsgIdAndTxt("cpk:dim", "length mismatch");
        plhs[0] = mxCreateDoubleMatrix((mwSize)info.N, 1, mxREAL);
        st = cmd[3] == 'a' ? cpk_pc_apply(M, mxGetPr(prhs[2]), mxGetPr(plhs[0]))
                           : cpk_pc_divide(M, mxGetPr(prhs[2]), mxGetPr(plhs[0]));
        if (st) fail(st);
    } else if (!strcmp(cmd, "pc_destroy")) {
        cpk_pc_destroy(to_pc(prhs[1]));
    } else if (!strcmp(cmd, "method")) {
        const int mid = method_id(prhs[1]);
        cpk_mat A = to_mat(prhs[3]), C = to_mat(prhs[4]);
        cpk_pc M = to_pc(prhs[5]);
        cpk_opts o;
        cpk_stats s;
        int64_t n = (int64_t)mxGetM(prhs[3]), m = (int64_t)mxGetM(prhs[4]);
        double itmax;
        mxArray *x, *y;
        to_opts(nrhs > 6 ? prhs[6] : NULL, &o);
        itmax = o.has_itmax ? o.itmax : (double)(mid >= CPK_GMRES ? n + m : n);
        memset(&s, 0, sizeof s);
        s.hist_cap = (int64_t)itmax + 4;
        if (mid == CPK_GMRES) s.hist_cap += o.has_restart ? (int64_t)o.restart : 50;
        s.hist = mxCalloc((size_t)s.hist_cap, sizeof(double));
        s.hist_lq = mxCalloc((size_t)s.hist_cap, sizeof(double));
        s.hist_qr = mxCalloc((size_t)s.hist_cap, sizeof(double));
        x = mxCreateDoubleMatrix((mwSize)n, 1, mxREAL);
        y = mxCreateDoubleMatrix((mwSize)m, 1, mxREAL);
        st = cpk_method_solve(ctx(), mid, mxGetPr(prhs[2]), A, C, M, &o, mxGetPr(x), mxGetPr(y), &s);
        cpk_mat_destroy(A), cpk_mat_destroy(C);
        if (st) fail(st);
        plhs[0] = x, plhs[1] = y;
        put_stats(mid, &s, &plhs[2], &plhs[3]);
    } else if (!strcmp(cmd, "reg_solve")) {
        const int mid = method_id(prhs[1]);
        cpk_mat A = to_mat(prhs[3]), B = to_mat(prhs[4]), C = to_mat(prhs[5]), G = to_mat(prhs[6]);
        cpk_opts o;
        cpk_stats s;
        int64_t n = (int64_t)mxGetM(prhs[3]), m = (int64_t)mxGetM(prhs[4]);
        double itmax;
        to_opts(nrhs > 7 ? prhs[7] : NULL, &o);
        itmax = o.has_itmax ? o.itmax : (double)(mid >= CPK_GMRES ? n + m : n);
        memset(&s, 0, sizeof s);
        s.hist_cap = (int64_t)itmax + 4;
        if (mid == CPK_GMRES) s.hist_cap += o.has_restart ? (int64_t)o.restart : 50;
        s.hist = mxCalloc((size_t)s.hist_cap, sizeof(double));
        s.hist_lq = mxCalloc((size_t)s.hist_cap, sizeof(double));
        s.hist_qr = mxCalloc((size_t)s.hist_cap, sizeof(double));
        plhs[0] = mxCreateDoubleMatrix((mwSize)(n + m), 1, mxREAL);
        st = cpk_reg_solve(ctx(), mid, mxGetPr(prhs[2]), A, B, C, G, &o, mxGetPr(plhs[0]), &s, NULL);
        cpk_mat_destroy(A), cpk_mat_destroy(B), cpk_mat_destroy(C), cpk_mat_destroy(G);
        if (st) fail(st);
        put_stats(mid, &s, &plhs[1], &plhs[2]);
    } else {
        mexErrMsgIdAndTxt("cpk:args", "cpk_mex: unknown command %s", cmd);
    }
    (void)nlhs;
}
