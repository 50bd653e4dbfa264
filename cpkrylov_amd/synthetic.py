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


def nonsym_system(N=50_000_000, seed=SEED + 1, window=4, scale=1e2, z1_range=(0.2, 60.0), s1_range=(1e-2, 1.0)):
    """Nonsymmetric 3x3-block system modelled on cvxqp2_s (examples/cvxqp2_s_3x3_nonsymm_perm_iter10.mat),
    the structure of SURVEY.md section 8d config 5 (S50 at the default N):

      A = [ H        -E1'  -E2' ]     H   nH x nH SPD tridiagonal (as Q of saddle_system)
          [ Z1 E1     S1    0   ]     E1, E2 select the variables with a lower / upper bound
          [ Z2 E2     0     S2  ]     Z, S positive diagonals (C3: z in [0.2, 60], s1 in
                                      [3e-3, 1], z2 ~ 1.5e-2, s2 ~ 9-10; here s1 >= 1e-2:
                                      below that CP-DQGMRES(40) with G = diag(A) stagnates on
                                      the synthetic system, while at 1e-2 it needs ~90 iterations,
                                      so the 40-vector window is exercised)
      B  m x n touching only the H columns (C3: 200 zero columns), built as in saddle_system
      G = diag(A), C = 1e-8 I, rhs ~ N(0, 1)

    Block sizes follow C3 (nH : nZ : m = 300 : 200 : 225), each bound set takes every
    other-ish variable so a row-block partition stays local."""
    nH = int(round(N * 300 / 725))
    nZ = int(round(N * 200 / 725))
    m = N - nH - nZ
    nZ1 = nZ // 2
    nZ2 = nZ - nZ1
    n = nH + nZ
    rq, rb, rr = _rngs(seed)
    # H: SPD tridiagonal
    g = np.exp(rq.uniform(np.log(4.0), np.log(1.3e2), size=nH))
    a = rq.uniform(0.5, 1.0, size=nH) * np.where(rq.random(nH) < 0.5, -1.0, 1.0)
    b = rq.uniform(0.5, 1.0, size=nH - 1) * np.where(rq.random(nH - 1) < 0.5, -1.0, 1.0)
    hd = g + scale * a * a
    hd[1:] += scale * b * b
    ho = scale * a[:-1] * b
    i1 = (np.arange(nZ1, dtype=np.int64) * nH) // max(nZ1, 1)
    i2 = np.minimum((np.arange(nZ2, dtype=np.int64) * nH) // max(nZ2, 1) + 1, nH - 1)
    z1 = np.exp(rq.uniform(np.log(z1_range[0]), np.log(z1_range[1]), size=nZ1))
    s1 = np.exp(rq.uniform(np.log(s1_range[0]), np.log(s1_range[1]), size=nZ1))
    z2 = rq.uniform(1.5e-2, 1.7e-2, size=nZ2)
    s2 = rq.uniform(9.0, 10.0, size=nZ2)
    k1 = nH + np.arange(nZ1)
    k2 = nH + nZ1 + np.arange(nZ2)
    r = np.arange(nH)
    rows = np.concatenate([r, r[1:], r[:-1], i1, i2, k1, k1, k2, k2])
    cols = np.concatenate([r, r[:-1], r[1:], k1, k2, i1, k1, i2, k2])
    vals = np.concatenate([hd, ho, ho, -np.ones(nZ1), -np.ones(nZ2), z1, s1, z2, s2])
    A = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    A.sum_duplicates()
    A.sort_indices()
    G = sp.diags(A.diagonal(), 0, shape=(n, n), format="csr")
    # B: m x n on the H columns only
    piv = np.floor(np.arange(m, dtype=np.float64) * nH / m).astype(np.int64)
    nextra = np.where(rb.random(m) < 0.1, 2, 1)
    offs = np.concatenate([np.arange(-window, 0), np.arange(1, window + 1)])
    c1 = np.empty(m, dtype=np.int64)
    c1[:-1] = piv[1:]
    c1[-1] = max(piv[-1] - 1, 0) if m > 1 else min(1, nH - 1)
    c2 = np.clip(piv + offs[rb.integers(0, offs.size, size=m)], 0, nH - 1)
    brow = np.concatenate([np.arange(m), np.arange(m), np.nonzero(nextra == 2)[0]])
    bcol = np.concatenate([piv, c1, c2[nextra == 2]])
    bval = rb.uniform(1.0 / 3.0, 1.0, size=brow.size) * np.where(rb.random(brow.size) < 0.5, -1.0, 1.0)
    B = sp.csr_matrix((bval, (brow, bcol)), shape=(m, n))
    B.sum_duplicates()
    B.sort_indices()
    Cm = sp.diags(np.full(m, 1e-8), 0, shape=(m, m), format="csr")
    rhs = rr.standard_normal(n + m)
    return dict(Q=A, B=B, C=Cm, G=G, rhs=rhs, n=n, m=m, N=n + m, nH=nH, nZ1=nZ1, nZ2=nZ2, seed=seed,
                window=window)
