"""Engine option exact_dots: the HIP solvers with order-independent inner products against the
oracle's exact mode (orc_set_exact), BIT FOR BIT.

Every inner product (the Lanczos alpha/beta pairs, CG's pAp/qCq/residual, the Arnoldi window
dots, the refinement norms) is the correctly rounded value of the exact sum of its TwoProd
pairs, and norm([a b]) one shared operation sequence (xacc.hpp / cpk_oracle.c xnorm2), so the
summation order -- the grid, the rank count, the oracle's thread count -- no longer changes a
bit.  Given the product's own factors (cpk_pc_export) the oracle then runs the same arithmetic
as the device: niters, every history entry, x and y compare with ==, on one GPU and on P
simulated ranks.  The default path keeps its band tests (test_gpu_parity.py, test_gpu_dist.py).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import fixtures as F
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = [
    ("cvxqp1_m", "minres", {}),
    ("cvxqp1_m", "cg", {}),
    ("cvxqp1_m", "cglanczos", {}),
    ("cvxqp1_m", "symmlq", {}),
    ("cvxqp1_m", "dqgmres", {"mem": 2}),
    ("cvxqp1_m", "minres", {"nitref": 3, "force_itref": False}),  # live refinement norms
    ("cvxqp2_s", "gmres", {"restart": 100}),
    ("cvxqp2_s", "gmres", {"restart": 20}),
    ("cvxqp2_s", "dqgmres", {"mem": 100}),
    ("cvxqp2_s", "dqgmres", {"mem": 20}),
    ("syn_nonsym20k", "dqgmres", {"mem": 40}),
    ("syn_nonsym20k", "gmres", {"restart": 40}),
    ("syn_symm20k", "minres", {}),
    ("syn_symm20k", "cglanczos", {"btol": 1e-3}),
]

PC_PROPS = ("nitref", "itref_tol", "force_itref", "residual_update")


def _oracle(P, method, opts, factors):
    """the oracle's reg_cpkrylov in exact mode on the product's factors (reg_cpkrylov.m:135-148
    copies the preconditioner fields of opts into M)"""
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=factors)
    Mo.set(**{k: float(opts[k]) for k in PC_PROPS if k in opts})
    with O.exact():
        return O.reg_solve(method, P["rhs"], P["Q"], P["B"], P["C"], Mo, opts)


def _assert_same(x, stats, flag, xo, so):
    assert stats["niters"] == so["niters"]
    assert flag["solved"] == so["solved"]
    for k in [k for k in so if k.endswith("History")]:
        assert len(stats[k]) == len(so[k]), k
        bad = np.flatnonzero(stats[k] != so[k])
        assert bad.size == 0, (k, bad[:5], stats[k][bad[:3]], so[k][bad[:3]])
    if "status" in so:
        assert stats["status"] == so["status"]
    bad = np.flatnonzero(x != xo)
    assert bad.size == 0, (bad.size, bad[:5], np.max(np.abs(x - xo)))


@pytest.mark.parametrize("name,method,extra", CASES)
def test_exact_reg_cpkrylov_bitexact(gpu_ctx, name, method, extra):
    import cpkrylov_amd as cpk
    P = F.load(name)
    opts = dict(F.EXPROG_OPTS, **extra)
    with cpk.engine_options(exact_dots=1):
        x, stats, flag = cpk.reg_cpkrylov(getattr(cpk, "cp" + method), P["rhs"], P["Q"], P["B"], P["C"], P["G"],
                                          opts)
        factors = stats["M"].export_factors()
    xo, so = _oracle(P, method, opts, factors)
    _assert_same(x, stats, flag, xo, so)


def test_exact_oracle_thread_count_independent():
    """The point of the mode on the checker's side: the oracle's OpenMP leg (per-thread partial
    sums) returns the serial restatement's bits."""
    P = F.load("syn_nonsym20k")
    opts = dict(F.EXPROG_OPTS, mem=40)
    out = []
    for t in (1, 3, 8):
        O.set_threads(t)
        try:
            with O.exact():
                out.append(O.reg_cpkrylov("dqgmres", P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts, order="rcm"))
        finally:
            O.set_threads(1)
    for x, s in out[1:]:
        assert np.array_equal(x, out[0][0])
        assert np.array_equal(s["residHistory"], out[0][1]["residHistory"])


def test_exact_batch_and_graph_independent(gpu_ctx):
    """Graph batch sizes and eager replay change no bit (the stop test is the device's)."""
    import cpkrylov_amd as cpk
    P = F.load("cvxqp1_m")
    opts = dict(F.EXPROG_OPTS)
    runs = []
    for o in (dict(exact_dots=1), dict(exact_dots=1, batch=1), dict(exact_dots=1, no_graph=1),
              dict(exact_dots=1, batch=16)):
        with cpk.engine_options(**o):
            x, stats, flag = cpk.reg_cpkrylov(cpk.cpminres, P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts)
        runs.append((x, stats["residHistory"]))
    for x, h in runs[1:]:
        assert np.array_equal(x, runs[0][0]) and np.array_equal(h, runs[0][1])


def _run_ranks(P, fn, options):
    import cpkrylov_amd as cpk
    g = cpk.SimGroup(P)

    def one(r):
        opt = dict(options, dist1=1) if P == 1 else dict(options)
        ctx = cpk.Context(device=0, rank=r, nranks=P, simgroup=g, options=opt)
        try:
            return fn(ctx, r)
        finally:
            ctx.close()

    with ThreadPoolExecutor(P) as ex:
        return [f.result(timeout=600) for f in [ex.submit(one, r) for r in range(P)]]


DIST_CASES = [("cvxqp1_m", "minres", {}), ("cvxqp1_m", "cg", {}), ("cvxqp1_m", "symmlq", {}),
              ("cvxqp1_m", "cglanczos", {}), ("cvxqp1_m", "minres", {"nitref": 3, "force_itref": False}),
              ("cvxqp2_s", "gmres", {"restart": 20}), ("cvxqp2_s", "dqgmres", {"mem": 20}),
              ("syn_nonsym20k", "dqgmres", {"mem": 40}), ("syn_symm20k", "minres", {})]


@pytest.mark.parametrize("P", [1, 2, 3, 4])
@pytest.mark.parametrize("name,method,extra", DIST_CASES)
def test_exact_dist_bitexact(name, method, extra, P):
    """P simulated ranks (the int64 allreduce of every rank's digits, rounded on every rank):
    the serial oracle's bits, so also the 1-GPU solve's bits."""
    import cpkrylov_amd as cpk
    Pd = F.load(name)
    opts = dict(F.EXPROG_OPTS, **extra)
    fn = getattr(cpk, "cp" + method)

    def work(ctx, r):
        x, stats, flag = cpk.reg_cpkrylov(fn, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, ctx=ctx)
        f = stats["M"].export_factors() if r == 0 else None
        return x, {k: v for k, v in stats.items() if k != "M"}, flag, f

    res = _run_ranks(P, work, dict(exact_dots=1))
    x, stats, flag, factors = res[0]
    xo, so = _oracle(Pd, method, opts, factors)
    for xr, sr, fr, _ in res:
        _assert_same(xr, sr, fr, xo, so)
