#!/usr/bin/env python
"""CPKRYLOV example program 2 on the MI355X (examples/cpk_exprog2.m:44-104 of the reference).

CP-GMRES(100) (or CP-DQGMRES(100): --method dqgmres) on the nonsymmetric saddle-point system of
problem cvxqp2-s, interior-point iteration 10: the reference's
`cvxqp2_s_3x3_nonsymm_perm_iter10.mat`, with n = nH + nZ (cpk_exprog2.m:48-49).  Prints the
reference's three lines (relative error against K \\ rhs, iters / solved, times).

  python examples/cpk_exprog2.py path/to/cvxqp2_s_3x3_nonsymm_perm_iter10.mat [--method gmres]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# cpk_exprog2.m:70-93
OPTS = dict(print=False, atol=1.0e-6, rtol=1.0e-6, itmax=500,
            residual_update=True, nitref=1, force_itref=True, itref_tol=1.0e-8)
METHODS = {"gmres": ("cpgmres", "CP-GMRES(100)", {"restart": 100}),
           "dqgmres": ("cpdqgmres", "CP-DQGMRES(100)", {"mem": 100})}


def run(path, method="gmres", verbose=True):
    """The program's body; returns (x, stats, flag, x_direct, relerr) for tests."""
    import scipy.sparse.linalg as spl

    import cpkrylov_amd as cpk
    d = cpk.load_mat(path)
    n, m = d["nH"] + d["nZ"], d["nJ"]  # cpk_exprog2.m:48-49
    Q, A, C, G = cpk.saddle_blocks(d["K"], n)
    fname, label, extra = METHODS[method]
    opts = dict(OPTS, **extra)
    if verbose:
        print("\n\n==================================================================")
        print("                   cpkrylov example program 2 (MI355X)")
        print("==================================================================\n")
        print("nonsymmetric saddle-point system from")
        print(f"- quadratic programming problem cvxqp2-s (n = {n}, m = {m})")
        print("- interior point iteration 10\n")
        print(f"**************************** {label} ***************************\n")
        print(f"atol = {opts['atol']:8.2e},  rtol = {opts['rtol']:8.2e},  itmax = {opts['itmax']}")
        print(f"residual_update = {int(opts['residual_update'])},  nitref = {opts['nitref']},  "
              f"force_iref = {int(opts['force_itref'])},  itref_tol = {opts['itref_tol']:7.1e}\n")
    ts = time.perf_counter()
    x_cpk, stats, flag = cpk.reg_cpkrylov(getattr(cpk, fname), d["rhs"], Q, A, C, G, opts)
    ttot = time.perf_counter() - ts
    x = spl.spsolve(d["K"].tocsc(), d["rhs"])
    relerr = float(np.linalg.norm(x - x_cpk) / np.linalg.norm(x))
    if verbose:
        print(f"2-norm relative error in the solution = {relerr:8.2e}")
        print(f"iters = {stats['niters']},  solved (1 yes, 0 no) = {int(flag['solved'])}")
        print(f"time (prec setup, solve, reg_cpkrylov) = {stats['ptime']:9.3e},  {stats['stime']:9.3e},  {ttot:9.3e}\n")
    return x_cpk, stats, flag, x, relerr


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mat", help="cvxqp2_s_3x3_nonsymm_perm_iter10.mat (the reference's examples/ data file)")
    ap.add_argument("--method", choices=sorted(METHODS), default="gmres")
    a = ap.parse_args()
    run(a.mat, a.method)
