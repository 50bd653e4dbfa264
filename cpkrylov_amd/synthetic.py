"""Synthetic regularized saddle-point systems for the throughput benchmark.

The reference ships no generator; these systems are modelled on the statistics of its
fixture cvxqp1_m (examples/cvxqp1_m_2x2_symm_iter10.mat):

  S10 (symmetric, config 4):  N = 10,000,000, n = 5,500,000, m = 4,500,000 (n/N = 0.55 as C1)
    Q = A  n x n, SPD 3-point band: Q = diag(g) + s R'R with R upper bidiagonal, entries
           +-U(0.5, 1), s = 1e3, g_i log-uniform in [5e-2, 2e4] (C1's diag(Q) range 0.0535 ...
           19864.6).  Like C1's coupled rows (diag ~ 0.5-1 x the off-diagonal row sum, sums of
           3.7e3-7e3) Q is far from diagonally dominant where g_i << s, so G = diag(Q) is a
           mediocre approximation there and CP-MINRES needs ~20 iterations (C1: 54).
    G = diag(Q)                       (examples/cpk_exprog1.m:60-61)
    B  m x n: row i has a pivot column p_i = floor(i*n/m) (distinct, so B has full row rank),
           the next row's pivot column p_{i+1} (so consecutive constraints share a variable and
           the Schur complement is one connected chain, as in a real constraint graph), and in
           20 % of the rows a third column within +-W of p_i -- C1's 2002 / 498 split of 2- and
           3-entry rows; values +-U(1/3, 1)
    C = 1e-8 * I                      (C1: C = 1e-8 I)
    rhs: b1 ~ 1e3 * N(0,1), b2 ~ N(0,1) (b2 != 0, so reg_cpkrylov's shift path runs)

The coupling window W (default 4) is narrower than SURVEY.md's +-64: with G diagonal the
preconditioner factor is [I 0; B G^-1 L_S], and a +-64 window makes the Schur complement
S = C + B G^-1 B' a band of half-width ~100 whose factor would hold ~10^9 entries; W = 4 keeps
S's half-width at ~3-7 rows, a factor of ~3-4 nnz(Kp) and an elimination-tree depth of
~O(10^2) under nested dissection -- the same order as C1's (70 levels) -- while the halos of a
row-block partition stay a few rows wide.  Seeds: one numpy PCG64 stream per block
(Q, B, rhs) derived from `seed`, so the system is identical on every host.
"""
import numpy as np
import scipy.sparse as sp

SEED = 20261015


def _rngs(seed):
    ss = np.random.SeedSequence(seed)
    return [np.random.Generator(np.random.PCG64(s)) for s in ss.spawn(3)]


def saddle_system(N=10_000_000, seed=SEED, window=4, frac_n=0.55, scale=1e3):
    """Return dict(Q, B, C, G, rhs, n, m) of the symmetric synthetic system (S10 at default N)."""
    n = int(round(frac_n * N))
    m = N - n
    rq, rb, rr = _rngs(seed)
    # ---- Q = diag(g) + s R'R, R upper bidiagonal -> SPD tridiagonal -------------------------
    g = np.exp(rq.uniform(np.log(5e-2), np.log(2e4), size=n))
    a = rq.uniform(0.5, 1.0, size=n) * np.where(rq.random(n) < 0.5, -1.0, 1.0)
    b = rq.uniform(0.5, 1.0, size=n - 1) * np.where(rq.random(n - 1) < 0.5, -1.0, 1.0)
    diag = g + scale * a * a
    diag[1:] += scale * b * b
    off = scale * a[:-1] * b
    Q = sp.diags([off, diag, off], [-1, 0, 1], shape=(n, n), format="csr", dtype=np.float64)
    Q.sort_indices()
    G = sp.diags(Q.diagonal(), 0, shape=(n, n), format="csr")
    # ---- B: m x n, pivot + 1 or 2 local entries ---------------------------------------------
    piv = np.floor(np.arange(m, dtype=np.float64) * n / m).astype(np.int64)
    nextra = np.where(rb.random(m) < 0.2, 2, 1)
    offs = np.concatenate([np.arange(-window, 0), np.arange(1, window + 1)])
    c1 = np.empty(m, dtype=np.int64)
    c1[:-1] = piv[1:]
    c1[-1] = max(piv[-1] - 1, 0) if m > 1 else min(1, n - 1)
    c2 = np.clip(piv + offs[rb.integers(0, offs.size, size=m)], 0, n - 1)
    rows = np.concatenate([np.arange(m), np.arange(m), np.nonzero(nextra == 2)[0]])
    cols = np.concatenate([piv, c1, c2[nextra == 2]])
    vals = rb.uniform(1.0 / 3.0, 1.0, size=rows.size) * np.where(rb.random(rows.size) < 0.5, -1.0, 1.0)
    B = sp.csr_matrix((vals, (rows, cols)), shape=(m, n))
    B.sum_duplicates()  # clipped collisions at the ends merge
    B.sort_indices()
    # ---- C = 1e-8 I ---------------------------------------------------------------------------
    Cm = sp.diags(np.full(m, 1e-8), 0, shape=(m, m), format="csr")
    rhs = np.concatenate([1e3 * rr.standard_normal(n), rr.standard_normal(m)])
    return dict(Q=Q, B=B, C=Cm, G=G, rhs=rhs, n=n, m=m, N=N, seed=seed, window=window)
