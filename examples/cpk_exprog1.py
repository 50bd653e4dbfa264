#!/usr/bin/env python
"""CPKRYLOV example program 1 on the MI355X (examples/cpk_exprog1.m:44-104 of the reference).

CP-MINRES (or CP-CG, CP-CGLANCZOS, CP-DQGMRES(2): --method) on the symmetric saddle-point system
of problem cvxqp1-m, interior-point iteration 10, from Orban's collection: the reference's
`cvxqp1_m_2x2_symm_iter10.mat` (K, rhs, nH, nJ, nZ).  The preconditioner is opLDL2(G, A, -C) with
G = diag(Q), built and applied on the GPU; the solution is compared with K \\ rhs from a sparse
direct solve, and the program prints the reference's three lines: the 2-norm relative error,
iters / solved, and the times (preconditioner setup, solve, reg_cpkrylov).

  python examples/cpk_exprog1.py path/to/cvxqp1_m_2x2_symm_iter10.mat [--method minres]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# cpk_exprog1.m:79-95: the example's options
OPTS = dict(print=False, atol=1.0e-6, rtol=1.0e-6, itmax=500,
            residual_update=True, nitref=1, force_itref=True, itref_tol=1.0e-8)
METHODS = {"minres": ("cpminres", "CP-MINRES", {}), "cg": ("cpcg", "CP-CG", {}),
           "cglanczos": ("cpcglanczos", "CP-CGLANCZOS", {}), "dqgmres": ("cpdqgmres", "CP-DQGMRES(2)", {"mem": 2})}


def run(path, method="minres", verbose=True):
    """The program's body; returns (x, stats, flag, x_direct, relerr) for tests."""
    import scipy.sparse.linalg as spl

    import cpkrylov_amd as cpk
    d = cpk.load_mat(path)  # load(filename): K, n = dim(K), nH, nJ, nZ, rhs
    n, m = d["nH"], d["nJ"]  # cpk_exprog1.m:46-47
    Q, A, C, G = cpk.saddle_blocks(d["K"], n)
    fname, label, extra = METHODS[method]
    opts = dict(OPTS, **extra)
    if verbose:
        print("\n\n==================================================================")
        print("                   cpkrylov example program 1 (MI355X)")
        print("==================================================================\n")
        print("symmetric saddle-point system from")
        print(f"- quadratic programming problem cvxqp1-m (n = {n}, m = {m})")
        print("- interior point iteration 10\n")
        print(f"**************************** {label} ***************************\n")
        print(f"atol = {opts['atol']:8.2e},  rtol = {opts['rtol']:8.2e},  itmax = {opts['itmax']}")
        print(f"residual_update = {int(opts['residual_update'])},  nitref = {opts['nitref']},  "
              f"force_iref = {int(opts['force_itref'])},  itref_tol = {opts['itref_tol']:7.1e}\n")
    ts = time.perf_counter()
    x_cpk, stats, flag = cpk.reg_cpkrylov(getattr(cpk, fname), d["rhs"], Q, A, C, G, opts)
    ttot = time.perf_counter() - ts
    x = spl.spsolve(d["K"].tocsc(), d["rhs"])  # x = K \ rhs (the example's comparison)
    relerr = float(np.linalg.norm(x - x_cpk) / np.linalg.norm(x))
    if verbose:
        print(f"2-norm relative error in the solution = {relerr:8.2e}")
        print(f"iters = {stats['niters']},  solved (1 yes, 0 no) = {int(flag['solved'])}")
        print(f"time (prec setup, solve, reg_cpkrylov) = {stats['ptime']:9.3e},  {stats['stime']:9.3e},  {ttot:9.3e}\n")
    return x_cpk, stats, flag, x, relerr


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mat", help="cvxqp1_m_2x2_symm_iter10.mat (the reference's examples/ data file)")
    ap.add_argument("--method", choices=sorted(METHODS), default="minres")
    a = ap.parse_args()
    run(a.mat, a.method)
