/*
 * cpk_oracle.c -- TEST INFRASTRUCTURE ONLY.  See cpk_oracle.h for scope and parity status.
 *
 * A line-by-line CPU restatement of the MATLAB reference.  Every elementwise update keeps
 * MATLAB's left-to-right evaluation order with one rounding per operation; the file is
 * compiled with -ffp-contract=off so no FMA is formed.  Sparse products follow MATLAB's
 * column-oriented (CSC) accumulation order: per output row, terms are added in increasing
 * column order starting from 0.  Triangular solves follow MATLAB's column-oriented sparse
 * mldivide: per unknown, the subtractions happen in increasing (forward) or decreasing
 * (backward) pivot order.  Dot products are plain left-to-right sums (MKL's order is
 * unknown, so those are compared within tolerance only).
 */
#include "cpk_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static char g_err[512];
static int set_err(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}
const char *orc_last_error(void) { return g_err; }

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

#define EPS 2.220446049250313e-16 /* MATLAB eps */

/* Threads of the CPU-baseline leg (orc_set_threads; default 1 = the plain serial restatement).
 * With T > 1 the row-parallel parts run under OpenMP -- SpMV rows, elementwise updates and the
 * triangular sweeps by elimination-tree levels (every unknown still subtracts its terms in the
 * serial order, so these stay bit-identical) -- and the dot products sum per-thread chunks,
 * which changes their rounding (timing leg only; parity uses T = 1). */
static int g_threads = 1;
void orc_set_threads(int t) { g_threads = t < 1 ? 1 : t; }
int orc_get_threads(void) {
#ifdef _OPENMP
    return g_threads;
#else
    return 1;
#endif
}
#ifdef _OPENMP
#define PLOOP(i, lo, hi, ...)                                                                  \
    do {                                                                                       \
        const int64_t lo_ = (lo), hi_ = (hi);                                                  \
        if (g_threads > 1 && hi_ - lo_ > 4096) {                                               \
            _Pragma("omp parallel for schedule(static) num_threads(g_threads)")                \
            for (int64_t i = lo_; i < hi_; i++) { __VA_ARGS__ }                                \
        } else {                                                                               \
            for (int64_t i = lo_; i < hi_; i++) { __VA_ARGS__ }                                \
        }                                                                                      \
    } while (0)
#else
#define PLOOP(i, lo, hi, ...) for (int64_t i = (lo); i < (hi); i++) { __VA_ARGS__ }
#endif

/* ------------------------------------------------------------------------------------ */
/* owned CSR                                                                             */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    int64_t nrows, ncols;
    int64_t *ptr;
    int32_t *ind;
    double *val;
} csr;

static void csr_free(csr *a) {
    free(a->ptr);
    free(a->ind);
    free(a->val);
    memset(a, 0, sizeof *a);
}

static int csr_alloc(csr *a, int64_t nr, int64_t nc, int64_t nnz) {
    a->nrows = nr;
    a->ncols = nc;
    a->ptr = calloc((size_t)nr + 1, sizeof(int64_t));
    a->ind = malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(int32_t));
    a->val = malloc((size_t)(nnz > 0 ? nnz : 1) * sizeof(double));
    return (a->ptr && a->ind && a->val) ? 0 : -1;
}

static orc_csr view(const csr *a) {
    orc_csr v = {a->nrows, a->ncols, a->ptr, a->ind, a->val};
    return v;
}

/* transpose (rows of the result are sorted because we sweep rows in order) */
static int csr_transpose(const orc_csr *a, csr *t) {
    int64_t nnz = a->ptr[a->nrows];
    if (csr_alloc(t, a->ncols, a->nrows, nnz)) return -1;
    for (int64_t p = 0; p < nnz; p++) t->ptr[a->ind[p] + 1]++;
    for (int64_t i = 0; i < a->ncols; i++) t->ptr[i + 1] += t->ptr[i];
    int64_t *next = malloc((size_t)(a->ncols + 1) * sizeof(int64_t));
    if (!next) return -1;
    memcpy(next, t->ptr, (size_t)(a->ncols + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < a->nrows; i++)
        for (int64_t p = a->ptr[i]; p < a->ptr[i + 1]; p++) {
            int64_t q = next[a->ind[p]]++;
            t->ind[q] = (int32_t)i;
            t->val[q] = a->val[p];
        }
    free(next);
    return 0;
}

/* y = A*x  (MATLAB sparse mtimes: per row, 0 + a1*x1 + a2*x2 + ... in column order) */
static void spmv(const orc_csr *a, const double *x, double *y) {
    PLOOP(i, 0, a->nrows,
        double acc = 0.0;
        for (int64_t p = a->ptr[i]; p < a->ptr[i + 1]; p++) acc += a->val[p] * x[a->ind[p]];
        y[i] = acc;
    );
}

/* ------------------------------------------------------------------------------------ */
/* Exact inner products (orc_set_exact; the product's engine option exact_dots)           */
/* ------------------------------------------------------------------------------------ */
/* MATLAB's dot and norm go to MKL, whose summation order is unknown, so a
 * plain sum matches the GPU only within rounding.  In exact mode every inner product is the
 * correctly rounded value of the exact sum of its TwoProd pairs (p = a*b, e = fma(a, b, -p):
 * p + e = a*b exactly unless a product under- or overflows), which no summation order can
 * change: the GPU's grid reductions, the OpenMP partials and this serial loop all give the
 * same bits.  The exact sum is held in a fixed-point superaccumulator of XW - 1 signed 32-bit
 * digits in int64 words, value = sum d[i] * 2^(32 i - 1074) (every double is an integer
 * multiple of 2^-1074); word XW - 1 counts non-finite terms (result NaN).  The device keeps a
 * floating-point expansion per thread and merges into the same digit layout (xacc.hpp); the
 * two implementations share no code, only the definition of the result. */
enum { XW = 68 };
static int g_exact = 0;
void orc_set_exact(int on) { g_exact = on != 0; }
int orc_get_exact(void) { return g_exact; }

static void xs_add(int64_t *d, double x) {
    if (x == 0) return;
    if (!isfinite(x)) {
        d[XW - 1]++;
        return;
    }
    uint64_t bits;
    memcpy(&bits, &x, sizeof bits);
    const int E = (int)((bits >> 52) & 0x7ff);
    uint64_t mant = bits & ((1ull << 52) - 1);
    int off = 0;
    if (E) mant |= 1ull << 52, off = E - 1;
    const int i = off >> 5, sh = off & 31;
    const uint64_t lo = mant << sh, hi = sh ? mant >> (64 - sh) : 0;
    const int64_t c0 = (int64_t)(lo & 0xffffffffu), c1 = (int64_t)(lo >> 32), c2 = (int64_t)hi;
    if (bits >> 63) d[i] -= c0, d[i + 1] -= c1, d[i + 2] -= c2;
    else d[i] += c0, d[i + 1] += c1, d[i + 2] += c2;
}

/* TwoProd with a hardware FMA (the rest of the oracle keeps -ffp-contract=off semantics) */
__attribute__((target("fma"))) static void xs_add_prod(int64_t *d, double a, double b) {
    const double p = a * b;
    const double e = __builtin_fma(a, b, -p);
    xs_add(d, p);
    xs_add(d, e);
}

/* bits [lo, lo + 64) of the magnitude digits u[0..nd) (zeros beyond either end) */
static uint64_t xs_bits64(const uint32_t *u, int nd, int lo) {
    if (lo < 0) return 0;  /* only called with lo >= 0 */
    const int i = lo >> 5, sh = lo & 31;
    const uint64_t w0 = i < nd ? u[i] : 0, w1 = i + 1 < nd ? u[i + 1] : 0, w2 = i + 2 < nd ? u[i + 2] : 0;
    uint64_t r = (w0 | (w1 << 32)) >> sh;
    if (sh) r |= w2 << (64 - sh);
    return r;
}

/* round the exact sum to the nearest double, ties to even */
static double xs_round(const int64_t *din) {
    if (din[XW - 1]) return NAN;
    enum { ND = XW - 1 };
    uint32_t u[ND];
    int64_t carry = 0;
    for (int i = 0; i < ND; i++) {
        const int64_t t = din[i] + carry;
        u[i] = (uint32_t)(t & 0xffffffff);
        carry = t >> 32; /* arithmetic: floor division */
    }
    const int neg = carry < 0;
    if (neg) {
        carry = 0;
        for (int i = 0; i < ND; i++) {
            const int64_t t = -din[i] + carry;
            u[i] = (uint32_t)(t & 0xffffffff);
            carry = t >> 32;
        }
    }
    if (carry != 0) return neg ? -INFINITY : INFINITY;
    int top = ND - 1;
    while (top >= 0 && u[top] == 0) top--;
    if (top < 0) return 0.0;
    const int b = 32 * top + (32 - __builtin_clz(u[top])); /* bit length of the magnitude */
    uint64_t rb;
    if (b <= 53) { /* exact: V * 2^-1074 with V < 2^53 (subnormal or the lowest binade) */
        const uint64_t V = xs_bits64(u, ND, 0) & ((1ull << 53) - 1);
        if (V < (1ull << 52)) rb = V; /* subnormal: exponent field 0 */
        else rb = (1ull << 52) | (V & ((1ull << 52) - 1));
    } else {
        int sh = b - 53;
        uint64_t M = xs_bits64(u, ND, sh) & ((1ull << 53) - 1);
        const int guard = (int)(xs_bits64(u, ND, sh - 1) & 1);
        int sticky = 0;
        const int lo = sh - 1; /* bits [0, lo) */
        for (int i = 0; i < (lo >> 5) && !sticky; i++) sticky = u[i] != 0;
        if (!sticky && (lo & 31)) sticky = (u[lo >> 5] & ((1u << (lo & 31)) - 1)) != 0;
        if (guard && (sticky || (M & 1))) {
            M++;
            if (M == (1ull << 53)) M >>= 1, sh++;
        }
        const int e = sh - 1074; /* value M * 2^e, M in [2^52, 2^53) */
        const int ef = e + 52 + 1023;
        if (ef >= 2047) return neg ? -INFINITY : INFINITY;
        rb = ((uint64_t)ef << 52) | (M & ((1ull << 52) - 1));
    }
    double r;
    memcpy(&r, &rb, sizeof r);
    return neg ? -r : r;
}

static double xdot(int64_t n, const double *a, const double *b) {
    int64_t d[XW];
    memset(d, 0, sizeof d);
#ifdef _OPENMP
    if (g_threads > 1 && n > 4096) {
        _Pragma("omp parallel num_threads(g_threads)") {
            int64_t t[XW];
            memset(t, 0, sizeof t);
            _Pragma("omp for schedule(static)") for (int64_t i = 0; i < n; i++) xs_add_prod(t, a[i], b[i]);
            _Pragma("omp critical") for (int k = 0; k < XW; k++) d[k] += t[k];
        }
        return xs_round(d);
    }
#endif
    for (int64_t i = 0; i < n; i++) xs_add_prod(d, a[i], b[i]);
    return xs_round(d);
}

/* the exact mode's norm([a b]) of a 2-vector, shared operation for operation with the device
 * (xacc.hpp xnorm2) instead of two libm hypot implementations: a power-of-two scaling into
 * [2^-600, 2^600] where a*a cannot over- or underflow, a^2 + b^2 as a double-double (TwoProd by
 * FMA, TwoSum), its square root, one Newton correction against the double-double */
__attribute__((target("fma"))) static double xnorm2(double a, double b) {
    a = fabs(a), b = fabs(b);
    if (a < b) {
        const double t = a;
        a = b, b = t;
    }
    if (!(b > 0) || !isfinite(a)) return a + b; /* b == 0, inf, nan */
    double sc = 1.0, us = 1.0;
    if (a > 0x1p500) sc = 0x1p-600, us = 0x1p600;
    else if (a < 0x1p-500) sc = 0x1p600, us = 0x1p-600;
    a = a * sc, b = b * sc;
    const double p1 = a * a, e1 = __builtin_fma(a, a, -p1);
    const double p2 = b * b, e2 = __builtin_fma(b, b, -p2);
    const double s = p1 + p2, bb = s - p1, t = (p1 - (s - bb)) + (p2 - bb);
    double lo = t + (e1 + e2);
    const double hi = s + lo;
    lo = lo - (hi - s);
    const double r = sqrt(hi);
    const double res = __builtin_fma(-r, r, hi) + lo;
    return (r + res / (2.0 * r)) * us;
}

double orc_xdot(int64_t n, const double *a, const double *b) { return xdot(n, a, b); }
double orc_xnorm2(double a, double b) { return xnorm2(a, b); }

static double dot(int64_t n, const double *a, const double *b) {
    if (g_exact) return xdot(n, a, b);
    double s = 0.0;
#ifdef _OPENMP
    if (g_threads > 1 && n > 4096) {
        _Pragma("omp parallel for schedule(static) num_threads(g_threads) reduction(+ : s)")
        for (int64_t i = 0; i < n; i++) s += a[i] * b[i];
        return s;
    }
#endif
    for (int64_t i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}

static double nrm2(int64_t n, const double *a) { return sqrt(dot(n, a, a)); }

/* MATLAB norm([a b]) of a 2-vector */
static double norm2(double a, double b) { return g_exact ? xnorm2(a, b) : hypot(a, b); }

static double msign(double a) { return (a > 0) - (a < 0); } /* MATLAB sign, sign(0)=0 */

/* ------------------------------------------------------------------------------------ */
/* SymGivens (util/SymGivens.m:1-29)                                                     */
/* ------------------------------------------------------------------------------------ */
void orc_symgivens(double a, double b, double *c, double *s, double *d) {
    if (b == 0) {
        *c = (a == 0) ? 1.0 : msign(a);
        *s = 0.0;
        *d = fabs(a);
    } else if (a == 0) {
        *c = 0.0;
        *s = msign(b);
        *d = fabs(b);
    } else if (fabs(b) > fabs(a)) {
        double t = a / b;
        *s = msign(b) / sqrt(1 + t * t);
        *c = *s * t;
        *d = b / *s;
    } else {
        double t = b / a;
        *c = msign(a) / sqrt(1 + t * t);
        *s = *c * t;
        *d = a / *c;
    }
}

/* ------------------------------------------------------------------------------------ */
/* opLDL2 (ops/opLDL2.m)                                                                 */
/* ------------------------------------------------------------------------------------ */
struct orc_ldl2 {
    int64_t nA, nC, N;
    csr Kp;              /* op.A = [A B'; B C]   (opLDL2.m:81) */
    csr K12, K22;        /* op.A(1:n, n+1:N), op.A(n+1:N, n+1:N) for the residual-update branch */
    /* factors: P'*Kp*P = L*D*L' with L unit lower (opLDL2.m:82) */
    int64_t *Lp;         /* CSC of strict lower L */
    int32_t *Li;
    double *Lx;
    csr Lrow;            /* CSR of strict lower L (= CSC of L'), for the backward sweep */
    double *D;
    int32_t *perm;       /* perm[k] = original index of pivot k */
    /* public properties (opLDL2.m:45-50) */
    double nitref, itref_tol, force_itref, residual_update;
    double *w1, *w2, *w3; /* scratch */
    /* handle semantics (opt-in, not the reference's effective behaviour): op.Aty = ghn[0, nA),
     * op.Cy = ghn[nA, N) persist between applies, as reg_cpkrylov.m:47-52 and the GHN paper
     * intend; off (the default) restates MATLAB's value-object semantics, where they stay zero */
    int handle;
    double *ghn;
    /* threaded sweeps (g_threads > 1): rows by forward / backward level, built on first use */
    int64_t nlf, nlb;
    int64_t *lf_ptr, *lb_ptr;
    int32_t *lf_rows, *lb_rows;
};

static int assemble_kp(const orc_csr *A, const orc_csr *B, const orc_csr *C, csr *Kp) {
    /* dimension checks as opLDL2.m:61-75 */
    if (A->nrows != A->ncols || C->nrows != C->ncols)
        return set_err(ORC_ERR_DIM, "First and last arguments must be square.");
    if (B->ncols != A->nrows || B->nrows != C->nrows)
        return set_err(ORC_ERR_DIM, "Incompatible dimensions.");
    int64_t n = A->nrows, m = C->nrows, N = n + m;
    csr Bt;
    if (csr_transpose(B, &Bt)) return set_err(ORC_ERR_NOMEM, "out of memory");
    int64_t nnz = A->ptr[n] + 2 * B->ptr[m] + C->ptr[m];
    if (csr_alloc(Kp, N, N, nnz)) return set_err(ORC_ERR_NOMEM, "out of memory");
    int64_t q = 0;
    for (int64_t i = 0; i < n; i++) {
        for (int64_t p = A->ptr[i]; p < A->ptr[i + 1]; p++) Kp->ind[q] = A->ind[p], Kp->val[q++] = A->val[p];
        for (int64_t p = Bt.ptr[i]; p < Bt.ptr[i + 1]; p++)
            Kp->ind[q] = (int32_t)(n + Bt.ind[p]), Kp->val[q++] = Bt.val[p];
        Kp->ptr[i + 1] = q;
    }
    for (int64_t i = 0; i < m; i++) {
        for (int64_t p = B->ptr[i]; p < B->ptr[i + 1]; p++) Kp->ind[q] = B->ind[p], Kp->val[q++] = B->val[p];
        for (int64_t p = C->ptr[i]; p < C->ptr[i + 1]; p++)
            Kp->ind[q] = (int32_t)(n + C->ind[p]), Kp->val[q++] = C->val[p];
        Kp->ptr[n + i + 1] = q;
    }
    csr_free(&Bt);
    return 0;
}

/* Reverse Cuthill-McKee on the graph of a symmetric-pattern CSR (oracle's own ordering). */
static void rcm_order(const csr *K, int32_t *perm) {
    int64_t N = K->nrows;
    char *seen = calloc((size_t)N, 1);
    int32_t *queue = perm;
    int64_t head = 0, tail = 0;
    int64_t *deg = malloc((size_t)N * sizeof(int64_t));
    for (int64_t i = 0; i < N; i++) deg[i] = K->ptr[i + 1] - K->ptr[i];
    int32_t *nb = malloc((size_t)N * sizeof(int32_t));
    for (int64_t start = 0; start < N; start++) {
        if (seen[start]) continue;
        /* pick a minimum-degree node of this component as root (first unvisited min-degree) */
        int64_t root = start;
        seen[root] = 1;
        queue[tail++] = (int32_t)root;
        while (head < tail) {
            int32_t v = queue[head++];
            int64_t cnt = 0;
            for (int64_t p = K->ptr[v]; p < K->ptr[v + 1]; p++) {
                int32_t w = K->ind[p];
                if (!seen[w]) seen[w] = 1, nb[cnt++] = w;
            }
            /* insertion sort neighbours by degree (stable) */
            for (int64_t a = 1; a < cnt; a++) {
                int32_t x = nb[a];
                int64_t b = a - 1;
                while (b >= 0 && deg[nb[b]] > deg[x]) nb[b + 1] = nb[b], b--;
                nb[b + 1] = x;
            }
            for (int64_t a = 0; a < cnt; a++) queue[tail++] = nb[a];
        }
    }
    for (int64_t i = 0; i < N / 2; i++) {
        int32_t t = perm[i];
        perm[i] = perm[N - 1 - i];
        perm[N - 1 - i] = t;
    }
    free(seen);
    free(deg);
    free(nb);
}

/* Up-looking sparse LDL' of P'*Kp*P (Kp symmetric, full pattern stored). */
static int ldl_factor(struct orc_ldl2 *op) {
    const csr *K = &op->Kp;
    int64_t N = op->N;
    int32_t *pinv = malloc((size_t)N * sizeof(int32_t));
    int64_t *parent = malloc((size_t)N * sizeof(int64_t));
    int64_t *flag = malloc((size_t)N * sizeof(int64_t));
    int64_t *lnz = calloc((size_t)N, sizeof(int64_t));
    int64_t *pattern = malloc((size_t)N * sizeof(int64_t));
    double *y = calloc((size_t)N, sizeof(double));
    if (!pinv || !parent || !flag || !lnz || !pattern || !y) return set_err(ORC_ERR_NOMEM, "out of memory");
    for (int64_t k = 0; k < N; k++) pinv[op->perm[k]] = (int32_t)k;
    /* symbolic: elimination tree and column counts */
    for (int64_t k = 0; k < N; k++) {
        parent[k] = -1;
        flag[k] = k;
        int64_t r = op->perm[k];
        for (int64_t p = K->ptr[r]; p < K->ptr[r + 1]; p++) {
            int64_t i = pinv[K->ind[p]];
            if (i >= k) continue;
            for (; flag[i] != k; i = parent[i]) {
                if (parent[i] == -1) parent[i] = k;
                lnz[i]++;
                flag[i] = k;
            }
        }
    }
    op->Lp = malloc((size_t)(N + 1) * sizeof(int64_t));
    op->Lp[0] = 0;
    for (int64_t k = 0; k < N; k++) op->Lp[k + 1] = op->Lp[k] + lnz[k];
    int64_t nnzL = op->Lp[N];
    op->Li = malloc((size_t)(nnzL > 0 ? nnzL : 1) * sizeof(int32_t));
    op->Lx = malloc((size_t)(nnzL > 0 ? nnzL : 1) * sizeof(double));
    op->D = malloc((size_t)N * sizeof(double));
    if (!op->Li || !op->Lx || !op->D) return set_err(ORC_ERR_NOMEM, "out of memory");
    /* numeric */
    for (int64_t k = 0; k < N; k++) {
        int64_t top = N;
        flag[k] = k;
        lnz[k] = 0;
        int64_t r = op->perm[k];
        for (int64_t p = K->ptr[r]; p < K->ptr[r + 1]; p++) {
            int64_t i = pinv[K->ind[p]];
            if (i > k) continue;
            y[i] += K->val[p];
            int64_t len = 0;
            for (; flag[i] != k; i = parent[i]) {
                pattern[len++] = i;
                flag[i] = k;
            }
            while (len > 0) pattern[--top] = pattern[--len];
        }
        double d = y[k];
        y[k] = 0.0;
        for (; top < N; top++) {
            int64_t i = pattern[top];
            double yi = y[i];
            y[i] = 0.0;
            int64_t p2 = op->Lp[i] + lnz[i];
            for (int64_t p = op->Lp[i]; p < p2; p++) y[op->Li[p]] -= op->Lx[p] * yi;
            double lki = yi / op->D[i];
            d -= lki * yi;
            op->Li[p2] = (int32_t)k;
            op->Lx[p2] = lki;
            lnz[i]++;
        }
        if (d == 0.0) return set_err(ORC_ERR_FACTOR, "ldl: zero pivot at %lld", (long long)k);
        op->D[k] = d;
    }
    /* CSR copy of L for the column-oriented backward sweep of L' */
    orc_csr Lcsc_as_csr = {N, N, op->Lp, op->Li, op->Lx}; /* CSC(L) read as CSR = L' */
    csr Lt;
    if (csr_transpose(&Lcsc_as_csr, &Lt)) return set_err(ORC_ERR_NOMEM, "out of memory");
    op->Lrow = Lt; /* transpose of L' = L, stored by rows */
    free(pinv);
    free(parent);
    free(flag);
    free(lnz);
    free(pattern);
    free(y);
    return 0;
}

static int ldl2_common(const orc_csr *A, const orc_csr *B, const orc_csr *C, struct orc_ldl2 **out) {
    struct orc_ldl2 *op = calloc(1, sizeof *op);
    if (!op) return set_err(ORC_ERR_NOMEM, "out of memory");
    int rc = assemble_kp(A, B, C, &op->Kp);
    if (rc) {
        free(op);
        return rc;
    }
    op->nA = A->nrows;
    op->nC = C->nrows;
    op->N = op->nA + op->nC;
    /* blocks op.A(1:n, n+1:N) and op.A(n+1:N, n+1:N) used by the residual-update branch */
    csr Bt;
    csr_transpose(B, &Bt);
    op->K12 = Bt;
    csr_alloc(&op->K22, C->nrows, C->ncols, C->ptr[C->nrows]);
    memcpy(op->K22.ptr, C->ptr, (size_t)(C->nrows + 1) * sizeof(int64_t));
    memcpy(op->K22.ind, C->ind, (size_t)C->ptr[C->nrows] * sizeof(int32_t));
    memcpy(op->K22.val, C->val, (size_t)C->ptr[C->nrows] * sizeof(double));
    op->nitref = 3;          /* opLDL2.m:46 */
    op->itref_tol = 1.0e-8;  /* opLDL2.m:47 */
    op->force_itref = 0;     /* opLDL2.m:48 */
    op->residual_update = 0; /* opLDL2.m:49 */
    op->perm = malloc((size_t)op->N * sizeof(int32_t));
    op->w1 = malloc((size_t)op->N * sizeof(double));
    op->w2 = malloc((size_t)op->N * sizeof(double));
    op->w3 = malloc((size_t)op->N * sizeof(double));
    op->handle = 0;
    op->ghn = calloc((size_t)op->N, sizeof(double));
    *out = op;
    return 0;
}

int orc_ldl2_create(const orc_csr *A, const orc_csr *B, const orc_csr *C, int order_kind,
                    const int32_t *perm, orc_ldl2 **out) {
    struct orc_ldl2 *op;
    int rc = ldl2_common(A, B, C, &op);
    if (rc) return rc;
    if (order_kind == ORC_ORDER_GIVEN) {
        if (!perm) return set_err(ORC_ERR_ARGS, "perm required");
        memcpy(op->perm, perm, (size_t)op->N * sizeof(int32_t));
    } else if (order_kind == ORC_ORDER_RCM) {
        rcm_order(&op->Kp, op->perm);
    } else {
        for (int64_t i = 0; i < op->N; i++) op->perm[i] = (int32_t)i;
    }
    rc = ldl_factor(op);
    if (rc) {
        orc_ldl2_destroy(op);
        return rc;
    }
    *out = op;
    return 0;
}

int orc_ldl2_create_from_factors(const orc_csr *A, const orc_csr *B, const orc_csr *C,
                                 const int64_t *Lcolptr, const int32_t *Lrowind, const double *Lval,
                                 const double *D, const int32_t *perm, orc_ldl2 **out) {
    struct orc_ldl2 *op;
    int rc = ldl2_common(A, B, C, &op);
    if (rc) return rc;
    int64_t N = op->N, nnzL = Lcolptr[N];
    memcpy(op->perm, perm, (size_t)N * sizeof(int32_t));
    op->Lp = malloc((size_t)(N + 1) * sizeof(int64_t));
    op->Li = malloc((size_t)(nnzL ? nnzL : 1) * sizeof(int32_t));
    op->Lx = malloc((size_t)(nnzL ? nnzL : 1) * sizeof(double));
    op->D = malloc((size_t)N * sizeof(double));
    memcpy(op->Lp, Lcolptr, (size_t)(N + 1) * sizeof(int64_t));
    memcpy(op->Li, Lrowind, (size_t)nnzL * sizeof(int32_t));
    memcpy(op->Lx, Lval, (size_t)nnzL * sizeof(double));
    memcpy(op->D, D, (size_t)N * sizeof(double));
    orc_csr Lcsc_as_csr = {N, N, op->Lp, op->Li, op->Lx};
    csr_transpose(&Lcsc_as_csr, &op->Lrow);
    *out = op;
    return 0;
}

void orc_ldl2_destroy(orc_ldl2 *op) {
    if (!op) return;
    csr_free(&op->Kp);
    csr_free(&op->K12);
    csr_free(&op->K22);
    csr_free(&op->Lrow);
    free(op->Lp);
    free(op->Li);
    free(op->Lx);
    free(op->D);
    free(op->perm);
    free(op->w1);
    free(op->w2);
    free(op->w3);
    free(op->ghn);
    free(op->lf_ptr), free(op->lb_ptr), free(op->lf_rows), free(op->lb_rows);
    free(op);
}

static double mround(double v) { return v < 0 ? -floor(-v + 0.5) : floor(v + 0.5); }

/* set.nitref: max(0, round(val))  (opLDL2.m:97-99) */
void orc_ldl2_set_nitref(orc_ldl2 *op, double v) { op->nitref = fmax(0.0, mround(v)); }
/* `sef.itref_tol` (opLDL2.m:101) is a typo, so no clamping setter is in effect: stored as given */
void orc_ldl2_set_itref_tol(orc_ldl2 *op, double v) { op->itref_tol = v; }
/* set.force_itref: anything other than false/true becomes false (opLDL2.m:105-111) */
void orc_ldl2_set_force_itref(orc_ldl2 *op, double v) { op->force_itref = (v != 0 && v != 1) ? 0 : v; }
/* set.residual_update: stored as given (opLDL2.m:113-115) */
void orc_ldl2_set_residual_update(orc_ldl2 *op, double v) { op->residual_update = v; }
/* opt-in handle semantics of the residual-update state; enabling or disabling clears it */
void orc_ldl2_set_handle(orc_ldl2 *op, double v) {
    op->handle = v != 0;
    memset(op->ghn, 0, (size_t)op->N * sizeof(double));
}
void orc_ldl2_get_props(const orc_ldl2 *op, double *a, double *b, double *c, double *d) {
    *a = op->nitref, *b = op->itref_tol, *c = op->force_itref, *d = op->residual_update;
}
int64_t orc_ldl2_nnzL(const orc_ldl2 *op) { return op->Lp[op->N]; }
/* the factors P'*Kp*P = L*D*L' (strict lower L in CSC, D in pivot order); any pointer may be NULL */
void orc_ldl2_export(const orc_ldl2 *op, int64_t *Lp, int32_t *Li, double *Lx, double *D) {
    const int64_t N = op->N, nnz = op->Lp[N];
    if (Lp) memcpy(Lp, op->Lp, (size_t)(N + 1) * sizeof(int64_t));
    if (Li) memcpy(Li, op->Li, (size_t)nnz * sizeof(int32_t));
    if (Lx) memcpy(Lx, op->Lx, (size_t)nnz * sizeof(double));
    if (D) memcpy(D, op->D, (size_t)N * sizeof(double));
}
void orc_ldl2_get_perm(const orc_ldl2 *op, int32_t *perm) {
    memcpy(perm, op->perm, (size_t)op->N * sizeof(int32_t));
}

/* rows grouped by level: lev[i] = 1 + max lev of the rows it reads (counting sort); fwd
 * visits rows in increasing order (rows of L read lower rows), else decreasing (columns of L) */
static void level_sets(int64_t N, const int64_t *ptr, const int32_t *ind, int fwd, int64_t *nl,
                       int64_t **lptr, int32_t **lrows) {
    int32_t *lev = calloc((size_t)(N > 0 ? N : 1), sizeof(int32_t));
    int32_t mx = -1;
    for (int64_t s = 0; s < N; s++) {
        const int64_t i = fwd ? s : N - 1 - s;
        int32_t l = 0;
        for (int64_t p = ptr[i]; p < ptr[i + 1]; p++)
            if (lev[ind[p]] + 1 > l) l = lev[ind[p]] + 1;
        lev[i] = l;
        if (l > mx) mx = l;
    }
    *nl = mx + 1;
    *lptr = calloc((size_t)mx + 2, sizeof(int64_t));
    *lrows = malloc((size_t)(N > 0 ? N : 1) * sizeof(int32_t));
    for (int64_t i = 0; i < N; i++) (*lptr)[lev[i] + 1]++;
    for (int64_t l = 0; l <= mx; l++) (*lptr)[l + 1] += (*lptr)[l];
    int64_t *nx = malloc((size_t)(mx + 1 > 0 ? mx + 1 : 1) * sizeof(int64_t));
    for (int64_t l = 0; l <= mx; l++) nx[l] = (*lptr)[l];
    for (int64_t i = 0; i < N; i++) (*lrows)[nx[lev[i]]++] = (int32_t)i;
    free(nx);
    free(lev);
}

/* y = op.LDL * x = P * (L' \ (D \ (L \ (P' * x))))   (opLDL2.m:86) */
static void ldl_apply(struct orc_ldl2 *op, const double *x, double *y) {
    int64_t N = op->N;
    double *z = op->w3;
#ifdef _OPENMP
    if (g_threads > 1) {
        /* the same sweeps in row ("pull") form by levels: unknown i subtracts L(i,j)*z(j) in
         * increasing j (forward) and L(j,i)*z(j) in decreasing j (backward), as the column
         * sweeps below do, so the result is bit-identical */
        if (!op->lf_ptr) {
            level_sets(N, op->Lrow.ptr, op->Lrow.ind, 1, &op->nlf, &op->lf_ptr, &op->lf_rows);
            level_sets(N, op->Lp, op->Li, 0, &op->nlb, &op->lb_ptr, &op->lb_rows);
        }
        PLOOP(k, 0, N, z[k] = x[op->perm[k]];);
        for (int64_t l = 0; l < op->nlf; l++)
            PLOOP(q, op->lf_ptr[l], op->lf_ptr[l + 1],
                const int32_t i = op->lf_rows[q];
                double acc = z[i];
                for (int64_t p = op->Lrow.ptr[i]; p < op->Lrow.ptr[i + 1]; p++) acc -= op->Lrow.val[p] * z[op->Lrow.ind[p]];
                z[i] = acc;
            );
        PLOOP(j, 0, N, z[j] = z[j] / op->D[j];);
        for (int64_t l = 0; l < op->nlb; l++)
            PLOOP(q, op->lb_ptr[l], op->lb_ptr[l + 1],
                const int32_t i = op->lb_rows[q];
                double acc = z[i];
                for (int64_t p = op->Lp[i + 1] - 1; p >= op->Lp[i]; p--) acc -= op->Lx[p] * z[op->Li[p]];
                z[i] = acc;
            );
        PLOOP(k, 0, N, y[op->perm[k]] = z[k];);
        return;
    }
#endif
    for (int64_t k = 0; k < N; k++) z[k] = x[op->perm[k]]; /* P' * x */
    /* L \ z, column-oriented (unit diagonal: z_j / 1 is exact) */
    for (int64_t j = 0; j < N; j++) {
        double zj = z[j];
        for (int64_t p = op->Lp[j]; p < op->Lp[j + 1]; p++) z[op->Li[p]] -= op->Lx[p] * zj;
    }
    /* D \ z */
    for (int64_t j = 0; j < N; j++) z[j] = z[j] / op->D[j];
    /* L' \ z, column-oriented backward: column j of L' is row j of L */
    for (int64_t j = N - 1; j >= 0; j--) {
        double zj = z[j];
        for (int64_t p = op->Lrow.ptr[j]; p < op->Lrow.ptr[j + 1]; p++) z[op->Lrow.ind[p]] -= op->Lrow.val[p] * zj;
    }
    for (int64_t k = 0; k < N; k++) y[op->perm[k]] = z[k]; /* P * z */
}

/* opLDL2.multiply (opLDL2.m:161-188).  Spot operators are value objects, so the writes to
 * op.Aty / op.Cy / op.rNorm inside multiply are lost on return: Aty and Cy stay zero and
 * the residual-update SpMVs are dead work, which is restated here as MATLAB executes it.
 * With handle semantics (orc_ldl2_set_handle) the state persists between applies. */
int orc_ldl2_apply(orc_ldl2 *op, const double *x, double *y) {
    int64_t n = op->nA, N = op->N;
    double *r = op->w1, *t = op->w2;
    if (op->residual_update != 0) {
        PLOOP(i, 0, N, t[i] = x[i] - op->ghn[i];); /* [x(1:n) - op.Aty; x(n+1:N) - op.Cy] */
        ldl_apply(op, t, y);
        /* op.Aty = op.A(1:n, n+1:n+m) * y2; op.Cy = op.A(n+1:N, n+1:N) * y2 (opLDL2.m:169-171) */
        orc_csr k12 = view(&op->K12), k22 = view(&op->K22);
        spmv(&k12, y + n, r);
        spmv(&k22, y + n, r + n);
        if (op->handle) memcpy(op->ghn, r, (size_t)N * sizeof(double));
    } else {
        ldl_apply(op, x, y);
    }
    if (op->nitref > 0) {
        orc_csr kp = view(&op->Kp);
        spmv(&kp, y, r);
        PLOOP(i, 0, N, r[i] = x[i] - r[i];);
        double rNorm = nrm2(N, r);
        double xNorm = nrm2(N, x);
        double nit = 0;
        while (nit < op->nitref && (rNorm >= op->itref_tol * xNorm || op->force_itref != 0)) {
            ldl_apply(op, r, t); /* dy = op.LDL * r */
            PLOOP(i, 0, N, y[i] = y[i] + t[i];);
            spmv(&kp, y, r);
            PLOOP(i, 0, N, r[i] = x[i] - r[i];);
            rNorm = nrm2(N, r);
            nit = nit + 1;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* helpers shared by the solvers                                                         */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    double atol, rtol, btol, itmax, restart, mem;
    int print;
} sopts;

static void read_opts(const orc_opts *o, double itmax_default, sopts *s) {
    s->atol = 1.0e-6;
    s->rtol = 1.0e-6;
    s->btol = 0.0;
    s->itmax = itmax_default;
    s->restart = 50;
    s->mem = 50;
    s->print = 1;
    if (!o) return;
    if (o->has_atol) s->atol = o->atol;
    if (o->has_rtol) s->rtol = o->rtol;
    if (o->has_btol) s->btol = o->btol;
    if (o->has_itmax) s->itmax = o->itmax;
    if (o->has_restart) s->restart = o->restart;
    if (o->has_mem) s->mem = fmax(1.0, o->mem); /* cpdqgmres.m:116-118 */
    if (o->has_print) s->print = o->print != 0;
}

static int hist_push(orc_stats *st, double **h, int64_t *len, double v) {
    if (*h) {
        if (*len >= st->hist_cap) return set_err(ORC_ERR_ARGS, "history buffer too small");
        (*h)[*len] = v;
    }
    (*len)++;
    return 0;
}

#define VEC(name, len) double *name = calloc((size_t)((len) > 0 ? (len) : 1), sizeof(double))

static int indefinite(const char *where, double beta) {
    return set_err(ORC_ERR_INDEFINITE, "%s, beta (before sqrt) = %g : preconditioner does not behave as a spd matrix.",
                   where, beta);
}

/* ------------------------------------------------------------------------------------ */
/* cpminres (kernels/cpminres.m:90-254)                                                  */
/* ------------------------------------------------------------------------------------ */
static int run_minres(int64_t n, int64_t m, const double *b, const orc_csr *A, const orc_csr *C, orc_ldl2 *M,
                      const orc_opts *o, double *x, double *y, orc_stats *st) {
    sopts s;
    read_opts(o, (double)n, &s);
    int64_t N = n + m;
    VEC(u, n); VEC(t, m); VEC(vk, n); VEC(qk, m); VEC(vkm1, n); VEC(qkm1, m);
    VEC(vkp1, n); VEC(qkp1, m); VEC(wv, n); VEC(wq, m); VEC(wv1, n); VEC(wq1, m);
    VEC(wv2, n); VEC(wq2, m); VEC(in, N); VEC(vprec, N);
    int rc = 0;
    memset(x, 0, (size_t)n * sizeof(double));
    memset(y, 0, (size_t)m * sizeof(double));
    memcpy(u, b, (size_t)n * sizeof(double));
    if (s.print) printf("\n**** Constraint-preconditioned version of MINRES ****\n\n");
    memcpy(in, u, (size_t)n * sizeof(double)); /* [u; t], t = 0 */
    orc_ldl2_apply(M, in, vprec);
    PLOOP(i, 0, n, vkp1[i] = vprec[i];);
    PLOOP(i, 0, m, qkp1[i] = -vprec[n + i];);
    double beta = dot(n, u, vkp1);
    const double eps100 = 100 * EPS;
    if (beta < -eps100) {
        rc = indefinite("Iter 0", beta);
        goto done;
    }
    beta = sqrt(fabs(beta));
    if (beta > 0) {
        PLOOP(i, 0, n, vkp1[i] = vkp1[i] / beta;);
        PLOOP(i, 0, m, qkp1[i] = qkp1[i] / beta;);
    }
    memcpy(wv, vkp1, (size_t)n * sizeof(double));
    memcpy(wq, qkp1, (size_t)m * sizeof(double));
    double residNorm = beta;
    st->hist_len = 0;
    if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
    int64_t k = 0;
    double deltabar = 0, epsln = 0, taubar = beta, cs = -1, sn = 0;
    double stopTol = s.atol + s.rtol * residNorm;
    if (s.print) {
        printf("stopTol = %e\n", stopTol);
        printf("%5s  %9s\n", "iter", "|resid|");
        printf("%5lld  %9.2e\n", (long long)k, residNorm);
    }
    while (residNorm > stopTol && k < s.itmax) {
        k = k + 1;
        double *tmp;
        tmp = vkm1, vkm1 = vk, vk = vkp1, vkp1 = tmp;
        tmp = qkm1, qkm1 = qk, qk = qkp1, qkp1 = tmp;
        spmv(A, vk, u);
        spmv(C, qk, t);
        double alpha = dot(n, u, vk) + dot(m, t, qk);
        PLOOP(i, 0, n, in[i] = u[i];);
        PLOOP(i, 0, m, in[n + i] = -t[i];);
        orc_ldl2_apply(M, in, vprec);
        PLOOP(i, 0, n, vkp1[i] = vprec[i] - alpha * vk[i] - beta * vkm1[i];);
        PLOOP(i, 0, m, qkp1[i] = qk[i] - vprec[n + i];);
        PLOOP(i, 0, m, qkp1[i] = qkp1[i] - alpha * qk[i] - beta * qkm1[i];);
        beta = dot(n, u, vkp1) + dot(m, t, qkp1);
        if (beta < -eps100) {
            char where[64];
            snprintf(where, sizeof where, "Iter %lld", (long long)k);
            rc = indefinite(where, beta);
            goto done;
        }
        beta = sqrt(fabs(beta));
        if (beta > 0) {
            PLOOP(i, 0, n, vkp1[i] = vkp1[i] / beta;);
            PLOOP(i, 0, m, qkp1[i] = qkp1[i] / beta;);
        }
        double oldeps = epsln;
        double delta = cs * deltabar + sn * alpha;
        double gammabar = sn * deltabar - cs * alpha;
        epsln = sn * beta;
        deltabar = -cs * beta;
        double gamma = norm2(gammabar, beta);
        cs = gammabar / gamma;
        sn = beta / gamma;
        double tau = cs * taubar;
        taubar = sn * taubar;
        tmp = wv1, wv1 = wv2, wv2 = wv, wv = tmp;
        tmp = wq1, wq1 = wq2, wq2 = wq, wq = tmp;
        PLOOP(i, 0, n, wv[i] = (vk[i] - oldeps * wv1[i] - delta * wv2[i]) / gamma;);
        PLOOP(i, 0, m, wq[i] = (qk[i] - oldeps * wq1[i] - delta * wq2[i]) / gamma;);
        PLOOP(i, 0, n, x[i] = x[i] + tau * wv[i];);
        PLOOP(i, 0, m, y[i] = y[i] - tau * wq[i];);
        residNorm = taubar;
        if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
        if (s.print) printf("%5lld  %9.2e\n", (long long)k, residNorm);
    }
    if (s.print) printf("\n");
    st->niters = k;
    st->solved = residNorm <= stopTol;
done:
    free(u); free(t); free(vk); free(qk); free(vkm1); free(qkm1); free(vkp1); free(qkp1);
    free(wv); free(wq); free(wv1); free(wq1); free(wv2); free(wq2); free(in); free(vprec);
    return rc;
}

/* ------------------------------------------------------------------------------------ */
/* cpcg (kernels/cpcg.m:94-195)                                                          */
/* ------------------------------------------------------------------------------------ */
static int run_cg(int64_t n, int64_t m, const double *b, const orc_csr *A, const orc_csr *C, orc_ldl2 *M,
                  const orc_opts *o, double *x, double *y, orc_stats *st) {
    sopts s;
    read_opts(o, (double)n, &s);
    int64_t N = n + m;
    VEC(a, m); VEC(w, m); VEC(g, n); VEC(p, n); VEC(q, m); VEC(Ap, n); VEC(Cq, m);
    VEC(in, N); VEC(ru, N); VEC(tt, m);
    int rc = 0;
    memset(x, 0, (size_t)n * sizeof(double));
    for (int64_t i = 0; i < n; i++) g[i] = -b[i];
    for (int64_t i = 0; i < n; i++) in[i] = g[i];
    for (int64_t i = 0; i < m; i++) in[n + i] = w[i];
    orc_ldl2_apply(M, in, ru); /* r = ru(1:n), u = ru(n+1:N) */
    const double *r = ru, *uu = ru + n;
    for (int64_t i = 0; i < n; i++) p[i] = -r[i];
    for (int64_t i = 0; i < m; i++) q[i] = -uu[i];
    double residNorm2 = dot(n, g, r);
    if (residNorm2 < 0) {
        rc = set_err(ORC_ERR_INDEFINITE, "Iter 0, residNorm2 = %g < 0: complex residual norm", residNorm2);
        goto done;
    }
    double residNorm = sqrt(residNorm2);
    double stopTol = s.atol + s.rtol * residNorm;
    st->hist_len = 0;
    if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
    int64_t itn = 0;
    if (s.print) {
        printf("\n**** Constraint-preconditioned version of CG ****\n\n");
        printf("stopTol = %e\n", stopTol);
        printf("%5s  %9s  %9s  %9s  %9s\n", "iter", "resid", "pr-curv", "du-curv", "steplen");
        printf("%5lld  %9.2e  ", (long long)itn, residNorm);
    }
    while (residNorm > stopTol && itn < s.itmax) {
        itn = itn + 1;
        spmv(A, p, Ap);
        double pAp = dot(n, p, Ap);
        spmv(C, q, Cq);
        double qCq = dot(m, q, Cq);
        double alpha = residNorm2 / (pAp + qCq);
        if (s.print) printf("%9.2e  %9.2e  %9.2e\n", pAp, qCq, alpha);
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + alpha * p[i];
        for (int64_t i = 0; i < m; i++) a[i] = a[i] + alpha * q[i];
        for (int64_t i = 0; i < n; i++) g[i] = g[i] + alpha * Ap[i];
        for (int64_t i = 0; i < m; i++) w[i] = w[i] + alpha * Cq[i];
        for (int64_t i = 0; i < n; i++) in[i] = g[i];
        for (int64_t i = 0; i < m; i++) in[n + i] = w[i];
        orc_ldl2_apply(M, in, ru);
        for (int64_t i = 0; i < m; i++) tt[i] = a[i] + uu[i];
        double residNorm2_new = dot(n, g, r) + dot(m, tt, w);
        double beta = residNorm2_new / residNorm2;
        for (int64_t i = 0; i < n; i++) p[i] = -r[i] + beta * p[i];
        for (int64_t i = 0; i < m; i++) q[i] = -tt[i] + beta * q[i];
        residNorm2 = residNorm2_new;
        if (residNorm2 < 0) {
            rc = set_err(ORC_ERR_INDEFINITE, "Iter %lld, residNorm2 = %g < 0: complex residual norm",
                         (long long)itn, residNorm2);
            goto done;
        }
        residNorm = sqrt(residNorm2);
        if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
        if (s.print) printf("%5lld  %9.2e  ", (long long)itn, residNorm);
    }
    if (s.print) printf("\n\n");
    st->solved = residNorm <= stopTol;
    st->niters = itn;
    memcpy(y, a, (size_t)m * sizeof(double)); /* y = a (cpcg.m:193) */
done:
    free(a); free(w); free(g); free(p); free(q); free(Ap); free(Cq); free(in); free(ru); free(tt);
    return rc;
}

/* ------------------------------------------------------------------------------------ */
/* cpgmres (kernels/cpgmres.m:98-271)                                                    */
/* ------------------------------------------------------------------------------------ */
static int run_gmres(int64_t n, int64_t m, const double *b, const orc_csr *A, const orc_csr *C, orc_ldl2 *M,
                     const orc_opts *o, double *x, double *y, orc_stats *st) {
    sopts s;
    read_opts(o, (double)(n + m), &s);
    int64_t N = n + m;
    int64_t restart = (int64_t)s.restart;
    if (restart < 1) return set_err(ORC_ERR_ARGS, "restart must be >= 1");
    int64_t R1 = restart + 1;
    double *g = calloc((size_t)R1, sizeof(double));
    double *V = calloc((size_t)(n * R1 > 0 ? n * R1 : 1), sizeof(double));
    double *Q = calloc((size_t)(m * R1 > 0 ? m * R1 : 1), sizeof(double));
    double *H = calloc((size_t)(R1 * restart), sizeof(double)); /* H(i,j) at H[i + j*R1] (0-based) */
    double *c = calloc((size_t)restart, sizeof(double));
    double *sv = calloc((size_t)restart, sizeof(double));
    double *z = calloc((size_t)restart, sizeof(double));
    VEC(u, n); VEC(t, m); VEC(q, m); VEC(in, N); VEC(w, N); VEC(tmpn, n); VEC(tmpm, m);
    int rc = 0;
#define HH(i, j) H[(i) + (int64_t)(j) * R1]
#define VV(j) (V + (int64_t)(j) * n)
#define QQ(j) (Q + (int64_t)(j) * m)
    memset(x, 0, (size_t)n * sizeof(double));
    memset(y, 0, (size_t)m * sizeof(double));
    int finished = 0;
    int64_t outer = 0;
    double outermax = ceil(s.itmax / (double)restart);
    double residNorm = 0, stopTol = 0;
    int64_t k = 0;
    st->hist_len = 0;
    if (s.print) printf("\n**** Constraint-preconditioned version of GMRES(%lld) ****\n\n", (long long)restart);
    while (!finished && outer < outermax) {
        outer = outer + 1;
        memset(q, 0, (size_t)m * sizeof(double));
        if (outer == 1) {
            memcpy(u, b, (size_t)n * sizeof(double));
            memset(t, 0, (size_t)m * sizeof(double));
            for (int64_t i = 0; i < n; i++) in[i] = u[i];
            for (int64_t i = 0; i < m; i++) in[n + i] = -t[i];
            orc_ldl2_apply(M, in, w);
            for (int64_t i = 0; i < n; i++) VV(0)[i] = w[i];
            for (int64_t i = 0; i < m; i++) QQ(0)[i] = -w[n + i];
        } else {
            spmv(A, x, tmpn);
            for (int64_t i = 0; i < n; i++) u[i] = b[i] - tmpn[i];
            spmv(C, y, t);
            for (int64_t i = 0; i < n; i++) in[i] = u[i];
            for (int64_t i = 0; i < m; i++) in[n + i] = -t[i];
            orc_ldl2_apply(M, in, w);
            for (int64_t i = 0; i < n; i++) VV(0)[i] = w[i];
            for (int64_t i = 0; i < m; i++) QQ(0)[i] = y[i] - w[n + i];
        }
        double rn2 = dot(n, u, VV(0)) + dot(m, t, QQ(0));
        if (rn2 < 0) {
            rc = set_err(ORC_ERR_INDEFINITE, "outer %lld: dot(u,V1)+dot(t,Q1) = %g < 0: complex residual norm",
                         (long long)outer, rn2);
            goto done;
        }
        residNorm = sqrt(rn2);
        if (residNorm != 0) {
            for (int64_t i = 0; i < n; i++) VV(0)[i] = VV(0)[i] / residNorm;
            for (int64_t i = 0; i < m; i++) QQ(0)[i] = QQ(0)[i] / residNorm;
        }
        if (outer == 1) {
            stopTol = s.atol + s.rtol * residNorm;
            if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
        }
        k = 0;
        g[0] = residNorm;
        if (s.print && outer == 1) {
            printf("stopTol = %e\n", stopTol);
            printf("%5s  %9s\n", "iter", "|resid|");
            printf("%5lld  %14.7e\n", (long long)k, residNorm);
        }
        while (residNorm > stopTol && k < restart) {
            k = k + 1; /* 1-based k; column index k-1 */
            spmv(A, VV(k - 1), u);
            spmv(C, QQ(k - 1), t);
            for (int64_t i = 0; i < n; i++) in[i] = u[i];
            for (int64_t i = 0; i < m; i++) in[n + i] = -t[i];
            orc_ldl2_apply(M, in, w);
            for (int64_t i = 0; i < n; i++) VV(k)[i] = w[i];
            for (int64_t i = 0; i < m; i++) QQ(k)[i] = QQ(k - 1)[i] - w[n + i];
            for (int64_t j = 1; j <= k; j++) {
                double h = dot(n, VV(j - 1), u) + dot(m, QQ(j - 1), t);
                HH(j - 1, k - 1) = h;
                for (int64_t i = 0; i < n; i++) VV(k)[i] = VV(k)[i] - h * VV(j - 1)[i];
                for (int64_t i = 0; i < m; i++) QQ(k)[i] = QQ(k)[i] - h * QQ(j - 1)[i];
            }
            double hn2 = dot(n, u, VV(k)) + dot(m, t, QQ(k));
            if (hn2 < 0) {
                rc = set_err(ORC_ERR_INDEFINITE, "Iter %lld: H(k+1,k)^2 = %g < 0: complex norm",
                             (long long)((outer - 1) * restart + k), hn2);
                goto done;
            }
            double hk1 = sqrt(hn2);
            HH(k, k - 1) = hk1;
            if (hk1 != 0) { /* lucky breakdown if = 0 */
                for (int64_t i = 0; i < n; i++) VV(k)[i] = VV(k)[i] / hk1;
                for (int64_t i = 0; i < m; i++) QQ(k)[i] = QQ(k)[i] / hk1;
            }
            for (int64_t j = 1; j <= k - 1; j++) {
                double Hjk = c[j - 1] * HH(j - 1, k - 1) + sv[j - 1] * HH(j, k - 1);
                HH(j, k - 1) = sv[j - 1] * HH(j - 1, k - 1) - c[j - 1] * HH(j, k - 1);
                HH(j - 1, k - 1) = Hjk;
            }
            double cc, ss, dd;
            orc_symgivens(HH(k - 1, k - 1), HH(k, k - 1), &cc, &ss, &dd);
            c[k - 1] = cc, sv[k - 1] = ss, HH(k - 1, k - 1) = dd;
            HH(k, k - 1) = 0;
            g[k] = sv[k - 1] * g[k - 1];
            g[k - 1] = c[k - 1] * g[k - 1];
            residNorm = fabs(g[k]);
            if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
            if (s.print) printf("%5lld  %14.7e\n", (long long)((outer - 1) * restart + k), residNorm);
        }
        /* z = H(1:k,1:k) \ g(1:k): upper-triangular back substitution, column oriented */
        for (int64_t i = 0; i < k; i++) z[i] = g[i];
        for (int64_t j = k - 1; j >= 0; j--) {
            z[j] = z[j] / HH(j, j);
            for (int64_t i = 0; i < j; i++) z[i] = z[i] - z[j] * HH(i, j);
        }
        /* x = x + V(:,1:k)*z ; q = q + Q(:,1:k)*z ; y = y - q */
        memset(tmpn, 0, (size_t)n * sizeof(double));
        memset(tmpm, 0, (size_t)m * sizeof(double));
        for (int64_t j = 0; j < k; j++) {
            for (int64_t i = 0; i < n; i++) tmpn[i] = tmpn[i] + VV(j)[i] * z[j];
            for (int64_t i = 0; i < m; i++) tmpm[i] = tmpm[i] + QQ(j)[i] * z[j];
        }
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + tmpn[i];
        for (int64_t i = 0; i < m; i++) q[i] = q[i] + tmpm[i];
        for (int64_t i = 0; i < m; i++) y[i] = y[i] - q[i];
        finished = residNorm <= stopTol;
    }
    st->niters = (outer - 1) * restart + k;
    st->solved = residNorm <= stopTol;
done:
#undef HH
#undef VV
#undef QQ
    free(g); free(V); free(Q); free(H); free(c); free(sv); free(z);
    free(u); free(t); free(q); free(in); free(w); free(tmpn); free(tmpm);
    return rc;
}

#ifdef _OPENMP
/* Timing-leg (g_threads > 1) forms of cpdqgmres's three window loops (cpdqgmres.m:210-216 the
 * H column against the fixed (u,t) and the V/Q update, :218-225 the new basis vector's norm,
 * :254-265 the direction vector and the x/y update).  The serial restatement runs each loop as
 * the reference writes it, one full pass per window column; here every element still takes the
 * same operations in the same order (so V, Q, PV, PQ, x, y are bit-identical given equal
 * scalars), but rows are processed in blocks that keep a block of every window column in cache,
 * so the window streams from memory once per pass instead of once per column.  Dot products sum
 * per-thread partials, combined in thread order (deterministic for a given thread count). */
enum { DQ_ROWS = 2048 };

/* hj[q] = dot(V(:,jpos), u) + dot(Q(:,jpos), t) for window columns j = j0 .. j0+nj-1.  Exact
 * mode: per-thread superaccumulators per column, summed digit-wise (the same bits as xdot). */
static void dq_window_dots(int64_t n, int64_t m, const double *V, const double *Q, int64_t M1, int64_t j0,
                           int64_t nj, const double *u, const double *t, double *hj) {
    const int T = g_threads;
    const int ex = g_exact;
    const size_t nw = ex ? XW : 1; /* words per partial sum */
    double *part = ex ? NULL : calloc((size_t)(2 * T * (nj > 0 ? nj : 1)), sizeof(double));
    int64_t *xpart = ex ? calloc((size_t)(2 * T * (nj > 0 ? nj : 1)) * nw, sizeof(int64_t)) : NULL;
    _Pragma("omp parallel num_threads(T)") {
        const int th = omp_get_thread_num();
        double *pv = ex ? NULL : part + (size_t)th * 2 * nj, *pq = ex ? NULL : pv + nj;
        int64_t *xv = ex ? xpart + (size_t)th * 2 * nj * nw : NULL, *xq = ex ? xv + nj * nw : NULL;
        _Pragma("omp for schedule(static)") for (int64_t b = 0; b < n; b += DQ_ROWS) {
            const int64_t e = b + DQ_ROWS < n ? b + DQ_ROWS : n;
            for (int64_t q = 0; q < nj; q++) {
                const double *v = V + ((j0 + q - 1) % M1) * n;
                if (ex) {
                    for (int64_t i = b; i < e; i++) xs_add_prod(xv + q * nw, v[i], u[i]);
                    continue;
                }
                double s = pv[q];
                for (int64_t i = b; i < e; i++) s += v[i] * u[i];
                pv[q] = s;
            }
        }
        _Pragma("omp for schedule(static)") for (int64_t b = 0; b < m; b += DQ_ROWS) {
            const int64_t e = b + DQ_ROWS < m ? b + DQ_ROWS : m;
            for (int64_t q = 0; q < nj; q++) {
                const double *v = Q + ((j0 + q - 1) % M1) * m;
                if (ex) {
                    for (int64_t i = b; i < e; i++) xs_add_prod(xq + q * nw, v[i], t[i]);
                    continue;
                }
                double s = pq[q];
                for (int64_t i = b; i < e; i++) s += v[i] * t[i];
                pq[q] = s;
            }
        }
    }
    for (int64_t q = 0; q < nj; q++) {
        if (ex) {
            int64_t dv[XW], dq[XW];
            memset(dv, 0, sizeof dv), memset(dq, 0, sizeof dq);
            for (int th = 0; th < T; th++)
                for (int k = 0; k < XW; k++)
                    dv[k] += xpart[((size_t)th * 2 * nj + q) * nw + k], dq[k] += xpart[((size_t)th * 2 * nj + nj + q) * nw + k];
            hj[q] = xs_round(dv) + xs_round(dq);
            continue;
        }
        double sv = 0.0, sq = 0.0;
        for (int th = 0; th < T; th++) sv += part[(size_t)th * 2 * nj + q], sq += part[(size_t)th * 2 * nj + nj + q];
        hj[q] = sv + sq;
    }
    free(part);
    free(xpart);
}

/* V(:,kp1) -= hj[q] V(:,jpos) in window order (likewise Q), then returns
 * dot(u, V(:,kp1)) + dot(t, Q(:,kp1)) */
static double dq_window_orth(int64_t n, int64_t m, double *V, double *Q, int64_t M1, int64_t j0, int64_t nj,
                             const double *hj, int64_t kp1pos, const double *u, const double *t) {
    const int T = g_threads;
    const int ex = g_exact;
    double *part = calloc((size_t)(2 * T), sizeof(double));
    int64_t *xpart = ex ? calloc((size_t)(2 * T) * XW, sizeof(int64_t)) : NULL;
    double *vk = V + (kp1pos - 1) * n, *qk = Q + (kp1pos - 1) * m;
    _Pragma("omp parallel num_threads(T)") {
        const int th = omp_get_thread_num();
        double sv = 0.0, sq = 0.0;
        int64_t *xv = ex ? xpart + (size_t)(2 * th) * XW : NULL, *xq = ex ? xv + XW : NULL;
        _Pragma("omp for schedule(static)") for (int64_t b = 0; b < n; b += DQ_ROWS) {
            const int64_t e = b + DQ_ROWS < n ? b + DQ_ROWS : n;
            for (int64_t q = 0; q < nj; q++) {
                const double *v = V + ((j0 + q - 1) % M1) * n, h = hj[q];
                for (int64_t i = b; i < e; i++) vk[i] = vk[i] - h * v[i];
            }
            if (ex) for (int64_t i = b; i < e; i++) xs_add_prod(xv, u[i], vk[i]);
            else for (int64_t i = b; i < e; i++) sv += u[i] * vk[i];
        }
        _Pragma("omp for schedule(static)") for (int64_t b = 0; b < m; b += DQ_ROWS) {
            const int64_t e = b + DQ_ROWS < m ? b + DQ_ROWS : m;
            for (int64_t q = 0; q < nj; q++) {
                const double *v = Q + ((j0 + q - 1) % M1) * m, h = hj[q];
                for (int64_t i = b; i < e; i++) qk[i] = qk[i] - h * v[i];
            }
            if (ex) for (int64_t i = b; i < e; i++) xs_add_prod(xq, t[i], qk[i]);
            else for (int64_t i = b; i < e; i++) sq += t[i] * qk[i];
        }
        part[2 * th] = sv, part[2 * th + 1] = sq;
    }
    double sv = 0.0, sq = 0.0;
    if (ex) {
        int64_t dv[XW], dq[XW];
        memset(dv, 0, sizeof dv), memset(dq, 0, sizeof dq);
        for (int th = 0; th < T; th++)
            for (int k = 0; k < XW; k++) dv[k] += xpart[(size_t)(2 * th) * XW + k], dq[k] += xpart[(size_t)(2 * th + 1) * XW + k];
        sv = xs_round(dv), sq = xs_round(dq);
    } else {
        for (int th = 0; th < T; th++) sv += part[2 * th], sq += part[2 * th + 1];
    }
    free(part);
    free(xpart);
    return sv + sq;
}

/* PV(:,kpos) = (V(:,kpos) - sum_q hj[q] PV(:,jpos)) / hkk, x += gk PV(:,kpos); likewise PQ with
 * y -= gk PQ(:,kpos) */
static void dq_window_dir(int64_t n, int64_t m, const double *V, const double *Q, double *PV, double *PQ,
                          int64_t M1, int64_t j0, int64_t nj, const double *hj, int64_t kpos, double hkk, double gk,
                          double *x, double *y) {
    const int T = g_threads;
    const double *vk = V + (kpos - 1) * n, *qk = Q + (kpos - 1) * m;
    double *pvk = PV + (kpos - 1) * n, *pqk = PQ + (kpos - 1) * m;
    _Pragma("omp parallel num_threads(T)") {
        _Pragma("omp for schedule(static)") for (int64_t b = 0; b < n; b += DQ_ROWS) {
            const int64_t e = b + DQ_ROWS < n ? b + DQ_ROWS : n;
            for (int64_t i = b; i < e; i++) pvk[i] = vk[i];
            for (int64_t q = 0; q < nj; q++) {
                const double *v = PV + ((j0 + q - 1) % M1) * n, h = hj[q];
                for (int64_t i = b; i < e; i++) pvk[i] = pvk[i] - h * v[i];
            }
            for (int64_t i = b; i < e; i++) pvk[i] = pvk[i] / hkk, x[i] = x[i] + gk * pvk[i];
        }
        _Pragma("omp for schedule(static)") for (int64_t b = 0; b < m; b += DQ_ROWS) {
            const int64_t e = b + DQ_ROWS < m ? b + DQ_ROWS : m;
            for (int64_t i = b; i < e; i++) pqk[i] = qk[i];
            for (int64_t q = 0; q < nj; q++) {
                const double *v = PQ + ((j0 + q - 1) % M1) * m, h = hj[q];
                for (int64_t i = b; i < e; i++) pqk[i] = pqk[i] - h * v[i];
            }
            for (int64_t i = b; i < e; i++) pqk[i] = pqk[i] / hkk, y[i] = y[i] - gk * pqk[i];
        }
    }
}
#endif

/* ------------------------------------------------------------------------------------ */
/* cpdqgmres (kernels/cpdqgmres.m:97-282)                                                */
/* ------------------------------------------------------------------------------------ */
static int run_dqgmres(int64_t n, int64_t m, const double *b, const orc_csr *A, const orc_csr *C, orc_ldl2 *M,
                       const orc_opts *o, double *x, double *y, orc_stats *st) {
    sopts s;
    read_opts(o, (double)(n + m), &s);
    int64_t N = n + m;
    double memd = fmin(s.mem, s.itmax); /* cpdqgmres.m:125 */
    int64_t mem = (int64_t)memd;
    if (mem < 1) mem = 1;
    int64_t itmax = (int64_t)s.itmax;
    int64_t M1 = mem + 1, M2 = mem + 2;
    /* H(itmax, mem+2) as in the reference; rows are 1-based j, columns 1-based kk */
    int64_t Hrows = itmax + 1;
    double *H = calloc((size_t)(Hrows * M2), sizeof(double));
    double *g = calloc((size_t)M1, sizeof(double));
    double *V = calloc((size_t)(n * M1 > 0 ? n * M1 : 1), sizeof(double));
    double *Q = calloc((size_t)(m * M1 > 0 ? m * M1 : 1), sizeof(double));
    double *PV = calloc((size_t)(n * M1 > 0 ? n * M1 : 1), sizeof(double));
    double *PQ = calloc((size_t)(m * M1 > 0 ? m * M1 : 1), sizeof(double));
    double *c = calloc((size_t)mem, sizeof(double));
    double *sv = calloc((size_t)mem, sizeof(double));
    VEC(u, n); VEC(t, m); VEC(in, N); VEC(w, N);
    int rc = 0;
    if (!H) { rc = set_err(ORC_ERR_NOMEM, "out of memory for H"); goto done; }
#define HH(j, kk) H[(int64_t)(j) * M2 + (kk) - 1]
#define VV(pos) (V + (int64_t)((pos) - 1) * n)
#define QQ(pos) (Q + (int64_t)((pos) - 1) * m)
#define PVV(pos) (PV + (int64_t)((pos) - 1) * n)
#define PQQ(pos) (PQ + (int64_t)((pos) - 1) * m)
    memset(x, 0, (size_t)n * sizeof(double));
    memset(y, 0, (size_t)m * sizeof(double));
    memcpy(u, b, (size_t)n * sizeof(double));
    if (s.print) printf("\n**** Constraint-preconditioned version of DQGMRES - mem = %lld ****\n\n", (long long)mem);
    memcpy(in, u, (size_t)n * sizeof(double)); /* [u; t], t = 0 */
    orc_ldl2_apply(M, in, w);
    for (int64_t i = 0; i < n; i++) VV(1)[i] = w[i];
    for (int64_t i = 0; i < m; i++) QQ(1)[i] = -w[n + i];
    double rn2 = dot(n, u, VV(1));
    if (rn2 < 0) { /* cpdqgmres.m:158-160 references k before assignment: MATLAB errors here */
        rc = set_err(ORC_ERR_INDEFINITE, "Undefined variable k (dot(u,V1) = %g < 0)", rn2);
        goto done;
    }
    double residNorm = sqrt(rn2);
    if (residNorm != 0) {
        for (int64_t i = 0; i < n; i++) VV(1)[i] = VV(1)[i] / residNorm;
        for (int64_t i = 0; i < m; i++) QQ(1)[i] = QQ(1)[i] / residNorm;
    }
    int64_t k = 0;
    g[0] = residNorm;
    double stopTol = s.atol + s.rtol * residNorm;
    st->hist_len = 0;
    if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
    if (s.print) {
        printf("stopTol = %e\n", stopTol);
        printf("%5s  %9s\n", "iter", "|resid|");
        printf("%5lld  %14.7e\n", (long long)k, residNorm);
    }
    while (residNorm > stopTol && k < s.itmax) {
        k = k + 1;
        int64_t kpos = (k - 1) % M1 + 1, kp1pos = k % M1 + 1, rotpos = (k - 1) % mem + 1;
        spmv(A, VV(kpos), u);
        spmv(C, QQ(kpos), t);
        for (int64_t i = 0; i < n; i++) in[i] = u[i];
        for (int64_t i = 0; i < m; i++) in[n + i] = -t[i];
        orc_ldl2_apply(M, in, w);
        for (int64_t i = 0; i < n; i++) VV(kp1pos)[i] = w[i];
        for (int64_t i = 0; i < m; i++) QQ(kp1pos)[i] = QQ(kpos)[i] - w[n + i];
#ifdef _OPENMP
        if (g_threads > 1) { /* timing leg: the same window passes, row-blocked (see dq_window_*) */
            int64_t j0 = k - mem + 1 > 1 ? k - mem + 1 : 1, nj = k - j0 + 1;
            double hj[nj > 0 ? nj : 1];
            dq_window_dots(n, m, V, Q, M1, j0, nj, u, t, hj);
            for (int64_t q = 0; q < nj; q++) HH(j0 + q, 2 + k - (j0 + q)) = hj[q];
            double hn2 = dq_window_orth(n, m, V, Q, M1, j0, nj, hj, kp1pos, u, t);
            if (hn2 < 0) {
                rc = set_err(ORC_ERR_INDEFINITE, "Iter %lld: H(k,1)^2 = %g < 0: complex norm", (long long)k, hn2);
                goto done;
            }
            HH(k, 1) = sqrt(hn2);
            if (HH(k, 1) != 0) {
                double h = HH(k, 1);
                PLOOP(i, 0, n, VV(kp1pos)[i] = VV(kp1pos)[i] / h;);
                PLOOP(i, 0, m, QQ(kp1pos)[i] = QQ(kp1pos)[i] / h;);
            }
            goto rotations;
        }
#endif
        for (int64_t j = (k - mem + 1 > 1 ? k - mem + 1 : 1); j <= k; j++) {
            int64_t jpos = (j - 1) % M1 + 1, kk = 2 + k - j;
            double h = dot(n, VV(jpos), u) + dot(m, QQ(jpos), t);
            HH(j, kk) = h;
            for (int64_t i = 0; i < n; i++) VV(kp1pos)[i] = VV(kp1pos)[i] - h * VV(jpos)[i];
            for (int64_t i = 0; i < m; i++) QQ(kp1pos)[i] = QQ(kp1pos)[i] - h * QQ(jpos)[i];
        }
        double hn2 = dot(n, u, VV(kp1pos)) + dot(m, t, QQ(kp1pos));
        if (hn2 < 0) {
            rc = set_err(ORC_ERR_INDEFINITE, "Iter %lld: H(k,1)^2 = %g < 0: complex norm", (long long)k, hn2);
            goto done;
        }
        HH(k, 1) = sqrt(hn2);
        if (HH(k, 1) != 0) {
            double h = HH(k, 1);
            for (int64_t i = 0; i < n; i++) VV(kp1pos)[i] = VV(kp1pos)[i] / h;
            for (int64_t i = 0; i < m; i++) QQ(kp1pos)[i] = QQ(kp1pos)[i] / h;
        }
#ifdef _OPENMP
    rotations:
#endif
        for (int64_t j = (k - mem > 1 ? k - mem : 1); j <= k - 1; j++) {
            int64_t jrot = (j - 1) % mem + 1, kk = k - j + 1, kk1 = kk + 1;
            double Hjk = c[jrot - 1] * HH(j, kk1) + sv[jrot - 1] * HH(j + 1, kk);
            HH(j + 1, kk) = sv[jrot - 1] * HH(j, kk1) - c[jrot - 1] * HH(j + 1, kk);
            HH(j, kk1) = Hjk;
        }
        double cc, ss, dd;
        orc_symgivens(HH(k, 2), HH(k, 1), &cc, &ss, &dd);
        c[rotpos - 1] = cc, sv[rotpos - 1] = ss, HH(k, 2) = dd;
        HH(k, 1) = 0;
        g[kp1pos - 1] = sv[rotpos - 1] * g[kpos - 1];
        g[kpos - 1] = c[rotpos - 1] * g[kpos - 1];
#ifdef _OPENMP
        if (g_threads > 1) {
            int64_t j0 = k - mem > 1 ? k - mem : 1, nj = k - j0;
            double hj[nj > 0 ? nj : 1];
            for (int64_t q = 0; q < nj; q++) hj[q] = HH(j0 + q, 2 + k - (j0 + q));
            dq_window_dir(n, m, V, Q, PV, PQ, M1, j0, nj, hj, kpos, HH(k, 2), g[kpos - 1], x, y);
            goto pushed;
        }
#endif
        memcpy(PVV(kpos), VV(kpos), (size_t)n * sizeof(double));
        memcpy(PQQ(kpos), QQ(kpos), (size_t)m * sizeof(double));
        for (int64_t j = (k - mem > 1 ? k - mem : 1); j <= k - 1; j++) {
            int64_t jpos = (j - 1) % M1 + 1, kk = 2 + k - j;
            double h = HH(j, kk);
            for (int64_t i = 0; i < n; i++) PVV(kpos)[i] = PVV(kpos)[i] - h * PVV(jpos)[i];
            for (int64_t i = 0; i < m; i++) PQQ(kpos)[i] = PQQ(kpos)[i] - h * PQQ(jpos)[i];
        }
        double hkk = HH(k, 2);
        for (int64_t i = 0; i < n; i++) PVV(kpos)[i] = PVV(kpos)[i] / hkk;
        for (int64_t i = 0; i < m; i++) PQQ(kpos)[i] = PQQ(kpos)[i] / hkk;
        double gk = g[kpos - 1];
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + gk * PVV(kpos)[i];
        for (int64_t i = 0; i < m; i++) y[i] = y[i] - gk * PQQ(kpos)[i];
#ifdef _OPENMP
    pushed:
#endif
        residNorm = fabs(g[kp1pos - 1]);
        if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
        if (s.print) printf("%5lld  %14.7e\n", (long long)k, residNorm);
    }
    st->niters = k;
    st->solved = residNorm <= stopTol;
done:
#undef HH
#undef VV
#undef QQ
#undef PVV
#undef PQQ
    free(H); free(g); free(V); free(Q); free(PV); free(PQ); free(c); free(sv);
    free(u); free(t); free(in); free(w);
    return rc;
}

/* ------------------------------------------------------------------------------------ */
/* cpsymmlq (kernels/cpsymmlq.m:97-369)                                                  */
/* ------------------------------------------------------------------------------------ */
static int run_symmlq(int64_t n, int64_t m, const double *b, const orc_csr *A, const orc_csr *C, orc_ldl2 *M,
                      const orc_opts *o, double *x, double *y, orc_stats *st) {
    sopts s;
    read_opts(o, (double)n, &s);
    int64_t N = n + m;
    VEC(u, n); VEC(t, m); VEC(wv, n); VEC(wq, m); VEC(vk, n); VEC(qk, m); VEC(vkm1, n); VEC(qkm1, m);
    VEC(vkp1, n); VEC(qkp1, m); VEC(in, N); VEC(vprec, N);
    int rc = 0;
    const double eps100 = 100 * EPS;
    memset(x, 0, (size_t)n * sizeof(double));
    memset(y, 0, (size_t)m * sizeof(double));
    memcpy(u, b, (size_t)n * sizeof(double));
    int64_t k = 0;
    st->hist_len = st->lq_len = st->qr_len = 0;
    if (s.print) printf("\n**** Constraint-preconditioned version of SYMMLQ ****\n\n");
    memcpy(in, u, (size_t)n * sizeof(double));
    orc_ldl2_apply(M, in, vprec);
    for (int64_t i = 0; i < n; i++) vkp1[i] = vprec[i];
    for (int64_t i = 0; i < m; i++) qkp1[i] = -vprec[n + i];
    double beta1 = dot(n, u, vkp1);
    if (beta1 < -eps100) {
        rc = indefinite("Iter 0", beta1);
        goto done;
    }
    beta1 = sqrt(fabs(beta1));
    if (beta1 > 0) {
        for (int64_t i = 0; i < n; i++) vkp1[i] = vkp1[i] / beta1;
        for (int64_t i = 0; i < m; i++) qkp1[i] = qkp1[i] / beta1;
    }
    double cgresidNorm = beta1, lqresidNorm = 0, qrresidNorm = 0;
    double stopTol = s.atol + s.rtol * cgresidNorm;
    if (cgresidNorm <= stopTol) {
        lqresidNorm = beta1;
        qrresidNorm = beta1;
        hist_push(st, &st->hist, &st->hist_len, cgresidNorm);
        hist_push(st, &st->hist_lq, &st->lq_len, lqresidNorm);
        hist_push(st, &st->hist_qr, &st->qr_len, qrresidNorm);
    }
    /* NOTE: cpsymmlq.m:182 calls the undefined `printf`, so MATLAB errors when print=true.
     * The restatement prints instead (documented deviation). */
    if (s.print) {
        printf("the printed |cgresid| is one iter ahead, unless the solver\n");
        printf("stops at iter = 0\n\n");
        printf("stopTol = %e\n", stopTol);
        printf("%5s   %9s   %9s   %9s\n", "iter", "|cgresid|", "|lqresid|", "|qrresid|");
        if (cgresidNorm <= stopTol)
            printf("%5lld  %9.2e   %9.2e    %9.2e\n", (long long)k, cgresidNorm, lqresidNorm, qrresidNorm);
    }
    int isdone = cgresidNorm <= stopTol;
    if (!isdone) {
        double *tmp;
        tmp = vk, vk = vkp1, vkp1 = tmp;
        tmp = qk, qk = qkp1, qkp1 = tmp;
        spmv(A, vk, u);
        spmv(C, qk, t);
        double alpha = dot(n, u, vk) + dot(m, t, qk);
        for (int64_t i = 0; i < n; i++) in[i] = u[i];
        for (int64_t i = 0; i < m; i++) in[n + i] = -t[i];
        orc_ldl2_apply(M, in, vprec);
        for (int64_t i = 0; i < n; i++) vkp1[i] = vprec[i] - alpha * vk[i];
        for (int64_t i = 0; i < m; i++) qkp1[i] = qk[i] - vprec[n + i];
        for (int64_t i = 0; i < m; i++) qkp1[i] = qkp1[i] - alpha * qk[i];
        double beta = dot(n, u, vkp1) + dot(m, t, qkp1);
        if (beta < -eps100) {
            rc = indefinite("Iter 0, 2nd Lanczos vec", beta);
            goto done;
        }
        beta = sqrt(fabs(beta));
        if (beta > 0) {
            for (int64_t i = 0; i < n; i++) vkp1[i] = vkp1[i] / beta;
            for (int64_t i = 0; i < m; i++) qkp1[i] = qkp1[i] / beta;
        }
        double gammabar = alpha, deltabar = beta, epsdelzeta = beta1, epsilonzeta = 0, bstep = 0, snprod = 1;
        double matnorm2 = alpha * alpha + beta * beta;
        double den = 0;
        while (cgresidNorm > stopTol && k < s.itmax) {
            double matnorm = sqrt(matnorm2);
            double epsmat = matnorm * EPS;
            den = gammabar;
            if (den == 0) den = epsmat;
            lqresidNorm = norm2(epsdelzeta, epsilonzeta);
            qrresidNorm = snprod * beta1;
            cgresidNorm = qrresidNorm * beta / fabs(den);
            if ((rc = hist_push(st, &st->hist_lq, &st->lq_len, lqresidNorm))) goto done;
            if ((rc = hist_push(st, &st->hist_qr, &st->qr_len, qrresidNorm))) goto done;
            if ((rc = hist_push(st, &st->hist, &st->hist_len, cgresidNorm))) goto done;
            if (s.print)
                printf("%5lld  %9.2e   %9.2e    %9.2e\n", (long long)k, cgresidNorm, lqresidNorm, qrresidNorm);
            k = k + 1;
            /* zetabar/zeta at cpsymmlq.m:255-256 are overwritten before use (dead) */
            tmp = vkm1, vkm1 = vk, vk = vkp1, vkp1 = tmp;
            tmp = qkm1, qkm1 = qk, qk = qkp1, qkp1 = tmp;
            double betaold = beta;
            spmv(A, vk, u);
            spmv(C, qk, t);
            alpha = dot(n, u, vk) + dot(m, t, qk);
            for (int64_t i = 0; i < n; i++) in[i] = u[i];
            for (int64_t i = 0; i < m; i++) in[n + i] = -t[i];
            orc_ldl2_apply(M, in, vprec);
            for (int64_t i = 0; i < n; i++) vkp1[i] = vprec[i] - alpha * vk[i] - beta * vkm1[i];
            for (int64_t i = 0; i < m; i++) qkp1[i] = qk[i] - vprec[n + i];
            for (int64_t i = 0; i < m; i++) qkp1[i] = qkp1[i] - alpha * qk[i] - beta * qkm1[i];
            beta = dot(n, u, vkp1) + dot(m, t, qkp1);
            if (beta < -eps100) {
                char where[64];
                snprintf(where, sizeof where, "Iter %lld", (long long)k);
                rc = indefinite(where, beta);
                goto done;
            }
            beta = sqrt(fabs(beta));
            if (beta > 0) {
                for (int64_t i = 0; i < n; i++) vkp1[i] = vkp1[i] / beta;
                for (int64_t i = 0; i < m; i++) qkp1[i] = qkp1[i] / beta;
            }
            matnorm2 = matnorm2 + alpha * alpha + beta * beta + betaold * betaold;
            double gamma = norm2(gammabar, betaold);
            double cs = gammabar / gamma;
            double sn = betaold / gamma;
            double delta = cs * deltabar + sn * alpha;
            gammabar = sn * deltabar - cs * alpha;
            double epsilon = sn * beta;
            deltabar = -cs * beta;
            double zeta = epsdelzeta / gamma;
            double zcs = zeta * cs;
            double zsn = zeta * sn;
            for (int64_t i = 0; i < n; i++) x[i] = x[i] + zcs * wv[i] + zsn * vk[i];
            for (int64_t i = 0; i < m; i++) y[i] = y[i] - zcs * wq[i] - zsn * qk[i];
            for (int64_t i = 0; i < n; i++) wv[i] = sn * wv[i] - cs * vk[i];
            for (int64_t i = 0; i < m; i++) wq[i] = sn * wq[i] - cs * qk[i];
            bstep = bstep + snprod * cs * zeta;
            snprod = snprod * sn;
            epsdelzeta = epsilonzeta - delta * zeta;
            epsilonzeta = -epsilon * zeta;
        }
        double matnorm = sqrt(matnorm2);
        double epsmat = matnorm * EPS;
        den = gammabar;
        if (den == 0) den = epsmat;
        lqresidNorm = norm2(epsdelzeta, epsilonzeta);
        qrresidNorm = snprod * beta1;
        if ((rc = hist_push(st, &st->hist_lq, &st->lq_len, lqresidNorm))) goto done;
        if ((rc = hist_push(st, &st->hist_qr, &st->qr_len, qrresidNorm))) goto done;
        /* cgresidHistory = [beta1; cgresidHistory] */
        if (st->hist) {
            if (st->hist_len + 1 > st->hist_cap) {
                rc = set_err(ORC_ERR_ARGS, "history buffer too small");
                goto done;
            }
            memmove(st->hist + 1, st->hist, (size_t)st->hist_len * sizeof(double));
            st->hist[0] = beta1;
        }
        st->hist_len++;
        if (cgresidNorm < lqresidNorm) { /* move to the CG point */
            double zetabar = epsdelzeta / den;
            bstep = bstep + snprod * zetabar;
            for (int64_t i = 0; i < n; i++) x[i] = x[i] + zetabar * wv[i];
            for (int64_t i = 0; i < m; i++) y[i] = y[i] - zetabar * wq[i];
        }
        memcpy(in, b, (size_t)n * sizeof(double));
        memset(in + n, 0, (size_t)m * sizeof(double));
        orc_ldl2_apply(M, in, vprec);
        bstep = bstep / beta1;
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + bstep * vprec[i];
        for (int64_t i = 0; i < m; i++) y[i] = y[i] - bstep * (-vprec[n + i]);
        if (s.print) printf("%5lld     ---      %9.2e    %9.2e\n\n", (long long)k, lqresidNorm, qrresidNorm);
    }
    st->niters = k;
    st->solved = cgresidNorm <= stopTol;
done:
    free(u); free(t); free(wv); free(wq); free(vk); free(qk); free(vkm1); free(qkm1);
    free(vkp1); free(qkp1); free(in); free(vprec);
    return rc;
}

/* ------------------------------------------------------------------------------------ */
/* cpcglanczos (kernels/cpcglanczos.m:107-326)                                           */
/* ------------------------------------------------------------------------------------ */
static int run_cglanczos(int64_t n, int64_t m, const double *b, const orc_csr *A, const orc_csr *C, orc_ldl2 *M,
                         const orc_opts *o, double *x, double *y, orc_stats *st) {
    sopts s;
    read_opts(o, (double)n, &s);
    int64_t N = n + m;
    VEC(u, n); VEC(t, m); VEC(vk, n); VEC(qk, m); VEC(vkm1, n); VEC(qkm1, m); VEC(vkp1, n); VEC(qkp1, m);
    VEC(wv, n); VEC(wq, m); VEC(in, N); VEC(vprec, N);
    int rc = 0;
    const double eps100 = 100 * EPS;
    memset(x, 0, (size_t)n * sizeof(double));
    memset(y, 0, (size_t)m * sizeof(double));
    memcpy(u, b, (size_t)n * sizeof(double));
    double oldbeta = 0, opNorm2 = 0;
    if (s.print) printf("\n**** Constraint-preconditioned version of CP-CGLanczos ****\n\n");
    memcpy(in, u, (size_t)n * sizeof(double));
    orc_ldl2_apply(M, in, vprec);
    for (int64_t i = 0; i < n; i++) vkp1[i] = vprec[i];
    for (int64_t i = 0; i < m; i++) qkp1[i] = -vprec[n + i];
    double beta = dot(n, u, vkp1);
    if (beta < -eps100) {
        rc = set_err(ORC_ERR_INDEFINITE,
                     "CPCGLanczos:IndefiniteError: Iter 0, beta (before sqrt) = %g : preconditioner not second-order sufficient",
                     beta);
        goto done;
    }
    beta = sqrt(fabs(beta));
    if (beta > 0) {
        for (int64_t i = 0; i < n; i++) vkp1[i] = vkp1[i] / beta;
        for (int64_t i = 0; i < m; i++) qkp1[i] = qkp1[i] / beta;
    }
    memcpy(wv, vkp1, (size_t)n * sizeof(double));
    memcpy(wq, qkp1, (size_t)m * sizeof(double));
    double beta1 = beta;
    double residNorm = beta1;
    st->hist_len = 0;
    if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
    int64_t k = 0;
    double dg = 0, low = 1, eta = beta;
    double rhobar = 1, xxNorm2 = 0, xNorm = 0, tau = 0, delta = 0;
    double stopTol = s.atol + s.rtol * residNorm;
    double bstopTol = s.btol * beta1;
    double opNorm = 0, bkerr = 0;
    if (s.print) {
        printf("stopTol = %e, bstopTol = %e\n", stopTol, bstopTol);
        printf("%5s  %9s", "iter", "|resid|");
        if (s.btol > 0) printf("  %9s  %9s  %9s", "bkerr", "|op|", "|x|");
        printf("\n");
        printf("%5lld  %9.2e", (long long)k, residNorm);
        if (s.btol > 0) printf("  %9.2e  %9.2e  %9.2e", 0.0, 0.0, xNorm);
        printf("\n");
    }
    while (residNorm > stopTol && residNorm > bstopTol && k < s.itmax) {
        k = k + 1;
        double *tmp;
        tmp = vkm1, vkm1 = vk, vk = vkp1, vkp1 = tmp;
        tmp = qkm1, qkm1 = qk, qk = qkp1, qkp1 = tmp;
        spmv(A, vk, u);
        spmv(C, qk, t);
        double alpha = dot(n, u, vk) + dot(m, t, qk);
        dg = alpha - low * low * dg;
        double zeta = eta / dg;
        for (int64_t i = 0; i < n; i++) x[i] = x[i] + zeta * wv[i];
        for (int64_t i = 0; i < m; i++) y[i] = y[i] - zeta * wq[i];
        for (int64_t i = 0; i < n; i++) in[i] = u[i];
        for (int64_t i = 0; i < m; i++) in[n + i] = -t[i];
        orc_ldl2_apply(M, in, vprec);
        for (int64_t i = 0; i < n; i++) vkp1[i] = vprec[i] - alpha * vk[i] - beta * vkm1[i];
        for (int64_t i = 0; i < m; i++) qkp1[i] = qk[i] - vprec[n + i];
        for (int64_t i = 0; i < m; i++) qkp1[i] = qkp1[i] - alpha * qk[i] - beta * qkm1[i];
        /* bb1, bb2 (cpcglanczos.m:246) are never used */
        beta = dot(n, u, vkp1) + dot(m, t, qkp1);
        if (beta < -eps100) {
            rc = set_err(ORC_ERR_INDEFINITE,
                         "CPCGLanczos:IndefiniteError: Iter %lld, beta (before sqrt) = %g : preconditioner not second-order sufficient",
                         (long long)k, beta);
            goto done;
        }
        beta = sqrt(fabs(beta));
        if (beta > 0) {
            for (int64_t i = 0; i < n; i++) vkp1[i] = vkp1[i] / beta;
            for (int64_t i = 0; i < m; i++) qkp1[i] = qkp1[i] / beta;
        }
        low = beta / dg;
        eta = -low * eta;
        for (int64_t i = 0; i < n; i++) wv[i] = vkp1[i] - low * wv[i];
        for (int64_t i = 0; i < m; i++) wq[i] = qkp1[i] - low * wq[i];
        if (s.btol > 0) {
            double rho = sqrt(rhobar * rhobar + low * low);
            double cs = rhobar / rho;
            double sn = low / rho;
            double num = zeta - delta * tau;
            double taubar = num / rhobar;
            tau = num / rho;
            xNorm = sqrt(xxNorm2 + taubar * taubar);
            xxNorm2 = xxNorm2 + tau * tau;
            delta = sn;
            rhobar = -cs;
            opNorm2 = opNorm2 + alpha * alpha + beta * beta + oldbeta * oldbeta;
            opNorm = sqrt(opNorm2);
            bkerr = opNorm * xNorm + beta1;
            bstopTol = s.btol * bkerr;
        }
        residNorm = beta * fabs(zeta);
        if ((rc = hist_push(st, &st->hist, &st->hist_len, residNorm))) goto done;
        oldbeta = beta;
        if (s.print) {
            printf("%5lld  %9.2e", (long long)k, residNorm);
            if (s.btol > 0) printf("  %9.2e  %9.2e  %9.2e", residNorm / bkerr, opNorm, xNorm);
            printf("\n");
        }
    }
    if (s.print) printf("\n");
    st->niters = k;
    st->solved = 0;
    st->status = 0; /* 'maximum number of iterations attained' */
    if (residNorm <= stopTol) st->solved = 1, st->status = 1;
    if (s.btol > 0 && residNorm <= bstopTol) st->solved = 1, st->status = 2;
done:
    free(u); free(t); free(vk); free(qk); free(vkm1); free(qkm1); free(vkp1); free(qkp1);
    free(wv); free(wq); free(in); free(vprec);
    return rc;
}

/* ------------------------------------------------------------------------------------ */
int orc_method(int method, const double *b, const orc_csr *A, const orc_csr *C, orc_ldl2 *M,
               const orc_opts *opts, double *x, double *y, orc_stats *st) {
    int64_t n = A->nrows, m = C->nrows;
    if (A->ncols != n || C->ncols != m || M->nA != n || M->nC != m)
        return set_err(ORC_ERR_DIM, "dimension mismatch between A, C and M");
    st->niters = 0;
    st->solved = 0;
    st->status = 0;
    switch (method) {
    case ORC_MINRES: return run_minres(n, m, b, A, C, M, opts, x, y, st);
    case ORC_CG: return run_cg(n, m, b, A, C, M, opts, x, y, st);
    case ORC_GMRES: return run_gmres(n, m, b, A, C, M, opts, x, y, st);
    case ORC_DQGMRES: return run_dqgmres(n, m, b, A, C, M, opts, x, y, st);
    case ORC_SYMMLQ: return run_symmlq(n, m, b, A, C, M, opts, x, y, st);
    case ORC_CGLANCZOS: return run_cglanczos(n, m, b, A, C, M, opts, x, y, st);
    default: return set_err(ORC_ERR_ARGS, "unknown method %d", method);
    }
}

/* reg_cpkrylov.m:150-175 with an existing M: the shift (:152-160), the method call (:163) and the
 * recovery (:166-173) -- cpk_reg_solve_device's counterpart */
int orc_reg_solve(int method, const double *b, const orc_csr *A, const orc_csr *B, const orc_csr *C,
                  orc_ldl2 *M, const orc_opts *opts, double *x, orc_stats *st) {
    int64_t n = A->nrows, m = B->nrows, N = n + m;
    int rc;
    double t1 = now_s();
    double *xy0 = calloc((size_t)N, sizeof(double));
    double *in = calloc((size_t)N, sizeof(double));
    double *b1 = malloc((size_t)n * sizeof(double));
    double *tmp = malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    double *tmp2 = malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    double *dx = malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    double *dy = malloc((size_t)(m > 0 ? m : 1) * sizeof(double));
    int shift = 0;
    for (int64_t i = 0; i < m; i++)
        if (b[n + i] != 0) { shift = 1; break; }
    if (shift) {
        memcpy(in + n, b + n, (size_t)m * sizeof(double));
        orc_ldl2_apply(M, in, xy0);
        csr Bt;
        csr_transpose(B, &Bt);
        orc_csr vBt = view(&Bt);
        spmv(A, xy0, tmp);
        spmv(&vBt, xy0 + n, tmp2);
        for (int64_t i = 0; i < n; i++) b1[i] = b[i] - tmp[i] - tmp2[i];
        csr_free(&Bt);
    } else {
        memcpy(b1, b, (size_t)n * sizeof(double));
    }
    rc = orc_method(method, b1, A, C, M, opts, dx, dy, st);
    if (rc == 0) {
        if (shift) {
            for (int64_t i = 0; i < n; i++) x[i] = xy0[i] + dx[i];
            for (int64_t i = 0; i < m; i++) x[n + i] = xy0[n + i] + dy[i];
        } else {
            memcpy(x, dx, (size_t)n * sizeof(double));
            memcpy(x + n, dy, (size_t)m * sizeof(double));
        }
    }
    st->stime = now_s() - t1;
    free(xy0); free(in); free(b1); free(tmp); free(tmp2); free(dx); free(dy);
    return rc;
}

/* reg_cpkrylov.m:121-180 */
int orc_reg_cpkrylov(int method, const double *b, const orc_csr *A, const orc_csr *B, const orc_csr *C,
                     const orc_csr *G, const orc_opts *opts, int order_kind, const int32_t *perm, double *x,
                     orc_stats *st, orc_ldl2 **M_out) {
    double t0 = now_s();
    /* M = opLDL2(G, B, -C) */
    csr negC;
    if (csr_alloc(&negC, C->nrows, C->ncols, C->ptr[C->nrows])) return set_err(ORC_ERR_NOMEM, "oom");
    memcpy(negC.ptr, C->ptr, (size_t)(C->nrows + 1) * sizeof(int64_t));
    memcpy(negC.ind, C->ind, (size_t)C->ptr[C->nrows] * sizeof(int32_t));
    for (int64_t p = 0; p < C->ptr[C->nrows]; p++) negC.val[p] = -C->val[p];
    orc_csr vnegC = view(&negC);
    orc_ldl2 *M;
    int rc = orc_ldl2_create(G, B, &vnegC, order_kind, perm, &M);
    csr_free(&negC);
    if (rc) return rc;
    double ptime = now_s() - t0;
    if (opts) {
        if (opts->has_nitref) orc_ldl2_set_nitref(M, opts->nitref);
        if (opts->has_itref_tol) orc_ldl2_set_itref_tol(M, opts->itref_tol);
        if (opts->has_residual_update) orc_ldl2_set_residual_update(M, opts->residual_update);
        if (opts->has_force_itref) orc_ldl2_set_force_itref(M, opts->force_itref);
    }
    rc = orc_reg_solve(method, b, A, B, C, M, opts, x, st);
    st->ptime = ptime;
    if (M_out && rc == 0) *M_out = M;
    else orc_ldl2_destroy(M);
    return rc;
}
