/*
 * cpk_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * CPU restatement of optimizers/cpkrylov (MATLAB, read as text from /root/reference):
 *   reg_cpkrylov.m, kernels/cp{minres,cg,gmres,dqgmres,symmlq,cglanczos}.m,
 *   ops/opLDL2.m, util/SymGivens.m.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The shipped product (cpkrylov_amd/libcpk.so) never links or calls this code.
 *
 * Parity status: MATLAB and the Spot toolbox are absent, and the reference records no
 * outputs, so iterate-level parity with MATLAB is UNPINNED.  The oracle is pinned by the
 * reference's own known-answer check (the examples compare against K\rhs,
 * examples/cpk_exprog1.m:101, cpk_exprog2.m:100) on the two shipped fixtures, and by the
 * algebraic invariants listed in DESIGN.md section 3.
 */
#ifndef CPK_ORACLE_H
#define CPK_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Borrowed CSR view (sorted column indices, no duplicates). */
typedef struct {
    int64_t nrows, ncols;
    const int64_t *ptr;
    const int32_t *ind;
    const double *val;
} orc_csr;

/* Method ids: the same numbering as include/cpk.h. */
enum { ORC_CG = 0, ORC_CGLANCZOS = 1, ORC_MINRES = 2, ORC_SYMMLQ = 3, ORC_GMRES = 4, ORC_DQGMRES = 5 };

/* Status codes: the same numbering as include/cpk.h. */
enum { ORC_OK = 0, ORC_ERR_INDEFINITE = 1, ORC_ERR_DIM = 2, ORC_ERR_ARGS = 3, ORC_ERR_FACTOR = 6,
       ORC_ERR_NOMEM = 7 };

/* opts struct with MATLAB isfield() semantics: a field counts only if has_* != 0. */
typedef struct {
    double atol, rtol, btol;
    double itmax, restart, mem;
    double print;
    double nitref, itref_tol, force_itref, residual_update;
    int has_atol, has_rtol, has_btol, has_itmax, has_restart, has_mem, has_print;
    int has_nitref, has_itref_tol, has_force_itref, has_residual_update;
} orc_opts;

typedef struct {
    int64_t niters;
    int solved;
    int status;          /* cpcglanczos: 0 max iters, 1 residual small, 2 backward error small */
    double *hist;        /* residHistory (cpsymmlq: cgresidHistory); caller-allocated */
    double *hist_lq;     /* cpsymmlq lqresidHistory (may be NULL for other methods) */
    double *hist_qr;     /* cpsymmlq qrresidHistory */
    int64_t hist_cap;    /* capacity of each history buffer */
    int64_t hist_len, lq_len, qr_len;
    double ptime, stime; /* seconds, as reg_cpkrylov.m:128-132,150-178 */
} orc_stats;

/* Ordering used by the oracle's own LDL^T. */
enum { ORC_ORDER_NATURAL = 0, ORC_ORDER_GIVEN = 1, ORC_ORDER_RCM = 2 };

typedef struct orc_ldl2 orc_ldl2;

/* opLDL2(A, B, C): Kp = [A B'; B C] (ops/opLDL2.m:60-92); perm used only with ORC_ORDER_GIVEN
 * (perm[k] = original index of pivot k, i.e. P'*Kp*P = L*D*L'). */
int orc_ldl2_create(const orc_csr *A11, const orc_csr *B, const orc_csr *C22, int order_kind,
                    const int32_t *perm, orc_ldl2 **out);
/* opLDL2 built from externally supplied factors (used to check the GPU apply bit-for-bit):
 * L strictly lower in CSC (colptr/rowind/val, N columns), D diagonal, perm as above. */
int orc_ldl2_create_from_factors(const orc_csr *A11, const orc_csr *B, const orc_csr *C22,
                                 const int64_t *Lcolptr, const int32_t *Lrowind, const double *Lval,
                                 const double *D, const int32_t *perm, orc_ldl2 **out);
void orc_ldl2_destroy(orc_ldl2 *op);
/* Public property setters (ops/opLDL2.m:97-115). */
void orc_ldl2_set_nitref(orc_ldl2 *op, double v);
void orc_ldl2_set_itref_tol(orc_ldl2 *op, double v);
void orc_ldl2_set_force_itref(orc_ldl2 *op, double v);
void orc_ldl2_set_residual_update(orc_ldl2 *op, double v);
void orc_ldl2_set_handle(orc_ldl2 *op, double v); /* opt-in handle semantics of op.Aty / op.Cy */
void orc_ldl2_get_props(const orc_ldl2 *op, double *nitref, double *itref_tol, double *force_itref,
                        double *residual_update);
/* y = M*x  (opLDL2.multiply, ops/opLDL2.m:161-188) */
int orc_ldl2_apply(orc_ldl2 *op, const double *x, double *y);
/* factor queries */
int64_t orc_ldl2_nnzL(const orc_ldl2 *op);
void orc_ldl2_export(const orc_ldl2 *op, int64_t *Lp, int32_t *Li, double *Lx, double *D);
void orc_ldl2_get_perm(const orc_ldl2 *op, int32_t *perm);

/* [x, y, stats, flag] = method(b, A, C, M, opts) -- kernels/cp*.m */
int orc_method(int method, const double *b, const orc_csr *A, const orc_csr *C, orc_ldl2 *M,
               const orc_opts *opts, double *x, double *y, orc_stats *stats);

/* [x, stats, flag] = reg_cpkrylov(method, b, A, B, C, G, opts) -- reg_cpkrylov.m:1-180.
 * If M_out != NULL the preconditioner is returned to the caller (who destroys it). */
int orc_reg_cpkrylov(int method, const double *b, const orc_csr *A, const orc_csr *B,
                     const orc_csr *C, const orc_csr *G, const orc_opts *opts, int order_kind,
                     const int32_t *perm, double *x, orc_stats *stats, orc_ldl2 **M_out);

/* reg_cpkrylov.m:150-175 with an existing preconditioner M (opts' preconditioner fields are not
 * applied here): the shift, the method call and the recovery; b and x of length N */
int orc_reg_solve(int method, const double *b, const orc_csr *A, const orc_csr *B, const orc_csr *C,
                  orc_ldl2 *M, const orc_opts *opts, double *x, orc_stats *stats);

/* [c, s, d] = SymGivens(a, b) -- util/SymGivens.m:1-29 */
void orc_symgivens(double a, double b, double *c, double *s, double *d);

const char *orc_last_error(void);

/* Threads of the CPU-baseline timing leg (default 1).  T > 1 runs SpMV, elementwise updates and
 * level-scheduled sweeps under OpenMP (bit-identical) and chunked dot products (not). */
void orc_set_threads(int t);
int orc_get_threads(void);
/* Exact inner products (default off): every dot and norm is the correctly rounded exact sum of
 * its TwoProd pairs, and norm([a b]) the shared double-double formula -- the product's engine
 * option exact_dots computes the same values, so histories compare bit for bit and the thread
 * count no longer changes any result.  orc_xdot exposes one such dot (tests). */
void orc_set_exact(int on);
int orc_get_exact(void);
double orc_xdot(int64_t n, const double *a, const double *b);
double orc_xnorm2(double a, double b);

#ifdef __cplusplus
}
#endif
#endif
