"""CPU oracle (test infrastructure) pinned against the reference's own checks.

The reference has no tests and records no outputs.  What pins the
oracle: (1) the examples' known-answer check against the direct solve K\\rhs
(cpk_exprog1.m:101-104, cpk_exprog2.m:100-103); (2) algebraic invariants of each method;
(3) the committed golden vectors (regression: bit-exact reproduction)."""
import numpy as np
import pytest
import scipy.sparse as sp

import fixtures as F
from golden.make_golden import CASES, case_file, run
from oracle import oracle as O


@pytest.mark.parametrize("name,method,extra", CASES)
def test_oracle_reproduces_golden(name, method, extra):
    x, st = run(name, method, extra)
    g = np.load(case_file(name, method, extra), allow_pickle=False)
    assert st["niters"] == int(g["niters"]) and st["solved"] == bool(g["solved"])
    for k in st:
        if k.endswith("History"):
            assert np.array_equal(st[k], g[k]), k
    assert np.array_equal(x, g["x"])


@pytest.mark.parametrize("name,method,extra", CASES)
def test_oracle_known_answer(name, method, extra):
    """The examples' own check: the solution agrees with K\\rhs to the accuracy the stopping
    test implies (measured: 4.5e-7 / 7.0e-7 on cvxqp1_m, 6.6e-5 - 8.6e-5 on cvxqp2_s)."""
    P = F.load(name)
    g = np.load(case_file(name, method, extra), allow_pickle=False)
    err = np.linalg.norm(g["x"] - P["x_direct"]) / np.linalg.norm(P["x_direct"])
    if bool(g["solved"]):
        assert err < (1e-6 if name == "cvxqp1_m" else 1e-4), err
        h = g["residHistory"] if "residHistory" in g else g["cgresidHistory"]
        assert h[-1] <= 1e-6 + 1e-6 * h[0]
    else:
        assert int(g["niters"]) == 500  # itmax attained (cpdqgmres with mem = 20 stalls)


def test_minres_invariants():
    P = F.load("cvxqp1_m")
    g = np.load(case_file("cvxqp1_m", "minres", {}), allow_pickle=False)
    h = g["residHistory"]
    assert len(h) == int(g["niters"]) + 1
    assert np.all(np.diff(h) <= 1e-12 * h[0])  # MINRES residual norms never increase
    # residHistory(1)^2 = <b1, M*[b1; 0]>_1 with b1 the shifted rhs (cpminres.m:131-141)
    n, m = P["n"], P["m"]
    M = O.LDL2(P["G"], P["B"], -P["C"], order="rcm")
    M.set(nitref=1, force_itref=1)
    b = P["rhs"]
    xy0 = M @ np.concatenate([np.zeros(n), b[n:]])
    b1 = b[:n] - P["Q"] @ xy0[:n] - P["B"].T @ xy0[n:]
    v = M @ np.concatenate([b1, np.zeros(m)])
    assert abs(np.sqrt(b1 @ v[:n]) - h[0]) <= 1e-12 * h[0]


def test_gmres_niters_formula():
    # niters = (outer - 1) * restart + k   (cpgmres.m:267)
    g = np.load(case_file("cvxqp2_s", "gmres", {"restart": 20}), allow_pickle=False)
    assert len(g["residHistory"]) == int(g["niters"]) + 1
    assert int(g["niters"]) == 380


def test_symmlq_history_alignment():
    g = np.load(case_file("cvxqp1_m", "symmlq", {}), allow_pickle=False)
    k = int(g["niters"])
    # cgresidHistory = [beta1; ...] (cpsymmlq.m:331): k+1 entries; lq/qr: k+1 entries (:326-327)
    assert len(g["cgresidHistory"]) == k + 1
    assert len(g["lqresidHistory"]) == k + 1 and len(g["qrresidHistory"]) == k + 1
    assert g["cgresidHistory"][0] == g["qrresidHistory"][0]


SYMGIVENS_TABLE = [  # (a, b) -> (c, s, d) following util/SymGivens.m branch by branch
    (0.0, 0.0, (1.0, 0.0, 0.0)),
    (3.0, 0.0, (1.0, 0.0, 3.0)),
    (-3.0, 0.0, (-1.0, 0.0, 3.0)),
    (0.0, 2.0, (0.0, 1.0, 2.0)),
    (0.0, -2.0, (0.0, -1.0, 2.0)),
    (3.0, 4.0, (0.6, 0.8, 5.0)),     # |b| > |a|
    (4.0, 3.0, (0.8, 0.6, 5.0)),     # |b| <= |a|
    (-4.0, 3.0, (-0.8, 0.6, 5.0)),     # d = a / c
    (1.0, 1.0, (1 / np.sqrt(2), 1 / np.sqrt(2), np.sqrt(2))),
]


@pytest.mark.parametrize("a,b,exp", SYMGIVENS_TABLE)
def test_symgivens_branches(a, b, exp):
    c, s, d = O.symgivens(a, b)
    assert np.allclose((c, s, d), exp, rtol=1e-15, atol=0)


def test_opldl2_setters():
    P = F.load("cvxqp2_s")
    M = O.LDL2(P["G"], P["B"], -P["C"])
    assert M.props() == dict(nitref=3, itref_tol=1e-8, force_itref=0, residual_update=0)
    M.set(nitref=2.5)
    assert M.props()["nitref"] == 3  # MATLAB round half away from zero
    M.set(nitref=-4)
    assert M.props()["nitref"] == 0
    M.set(force_itref=2)
    assert M.props()["force_itref"] == 0  # neither false nor true -> false
    M.set(force_itref=1)
    assert M.props()["force_itref"] == 1
    M.set(itref_tol=-1)
    assert M.props()["itref_tol"] == -1  # the `sef.itref_tol` typo: no clamping


def test_residual_update_is_noop():
    """Spot operators are value objects: op.Aty / op.Cy written inside multiply are lost, so
    residual_update changes nothing."""
    P = F.load("cvxqp1_m")
    M = O.LDL2(P["G"], P["B"], -P["C"], order="rcm")
    z = np.random.default_rng(0).standard_normal(P["n"] + P["m"])
    M.set(nitref=1, force_itref=1)
    y0 = M @ z
    M.set(residual_update=1)
    assert np.array_equal(M @ z, y0)
    assert np.array_equal(M @ z, y0)  # and stays so on the next call


def test_handle_semantics_state():
    """Opt-in handle semantics (not the reference's effective behaviour): op.Aty / op.Cy
    persist, so the next apply solves with [x1 - Aty; x2 - Cy] (opLDL2.m:164-172).  The first
    apply equals the value-object one; the state is Kp(:, n+1:N) * y(n+1:N); re-enabling clears it."""
    P = F.load("cvxqp1_m")
    n, m = P["n"], P["m"]
    Mh = O.LDL2(P["G"], P["B"], -P["C"], order="rcm")
    Mv = O.LDL2(P["G"], P["B"], -P["C"], order="rcm")
    for M in (Mh, Mv):
        M.set(nitref=0, residual_update=1)
    Mh.set_handle(True)
    rng = np.random.default_rng(4)
    x1, x2 = rng.standard_normal(n + m), rng.standard_normal(n + m)
    y1 = Mh @ x1
    assert np.array_equal(y1, Mv @ x1)
    Kp = sp.bmat([[P["G"], P["B"].T], [P["B"], -P["C"]]]).tocsr()
    state = Kp[:, n:] @ y1[n:]
    y2 = Mh @ x2
    y2_ref = Mv @ (x2 - state)
    assert np.linalg.norm(y2 - y2_ref) <= 1e-12 * np.linalg.norm(y2_ref)
    assert not np.array_equal(y2, Mv @ x2)  # the state matters
    Mh.set_handle(True)  # clears the state
    assert np.array_equal(Mh @ x1, y1)


def test_indefinite_error():
    """beta < -100*eps raises (cpminres.m:136-139): use a G that is not positive on the
    nullspace of B."""
    P = F.load("cvxqp2_s")
    Gneg = -P["G"]
    with pytest.raises(O.OracleError) as e:
        O.reg_cpkrylov("minres", P["rhs"], P["Q"], P["B"], P["C"], Gneg, dict(F.EXPROG_OPTS), order="rcm")
    assert "does not behave as a spd matrix" in str(e.value)


def test_threaded_leg_sweeps_bitexact():
    """The OpenMP CPU-baseline leg (orc_set_threads) sweeps by elimination-tree levels in row
    form; every unknown subtracts its terms in the serial column sweep's order, so M*z is
    bit-identical to the serial restatement.  Its cpminres differs only through the chunked
    dot products: same niters, histories within the 1e-8·h0 parity floor."""
    from cpkrylov_amd.synthetic import saddle_system
    S = saddle_system(N=40000, seed=7)
    M = O.LDL2(S["G"], S["B"], -S["C"], order="rcm")
    M.set(nitref=2, force_itref=0, itref_tol=1e-14)
    z = np.random.default_rng(1).standard_normal(S["n"] + S["m"])
    y1 = M @ z
    opts = dict(F.EXPROG_OPTS)
    x1, _, s1 = O.method("minres", S["rhs"][:S["n"]], S["Q"], S["C"], M, opts)
    try:
        assert O.set_threads(4) == 4
        y4 = M @ z
        x4, _, s4 = O.method("minres", S["rhs"][:S["n"]], S["Q"], S["C"], M, opts)
    finally:
        O.set_threads(1)
    assert np.array_equal(y1, y4)
    assert s1["niters"] == s4["niters"]
    h1, h4 = s1["residHistory"], s4["residHistory"]
    assert np.max(np.abs(h1 - h4)) <= 1e-8 * h1[0]
    assert np.linalg.norm(x1 - x4) <= 1e-8 * np.linalg.norm(x1)


def test_exact_dot_correctly_rounded():
    """orc_set_exact's inner product: the correctly rounded exact sum of the TwoProd pairs, i.e.
    (no product under- or overflowing) the correctly rounded exact dot product -- checked against
    Python's exact rational arithmetic, including cancellation, subnormals, ties to even and
    overflow; and independent of the thread count."""
    from fractions import Fraction as Fr
    rng = np.random.default_rng(11)
    for _ in range(25):
        n = int(rng.integers(1, 2000))
        a = rng.standard_normal(n) * np.exp(rng.uniform(-40, 40, n))
        b = rng.standard_normal(n) * np.exp(rng.uniform(-40, 40, n))
        ref = float(sum(Fr(float(x)) * Fr(float(y)) for x, y in zip(a, b)))
        assert O.xdot(a, b) == ref
    one = np.ones(8)
    cases = [([1e100, 1.0, -1e100, 1e-300, 3.0], 4.0),
             ([5e-324, 5e-324, -1e-320], -9.99e-321),
             ([1.0, 2.0 ** -53], 1.0),                          # tie: to even
             ([1.0, 2.0 ** -53, 2.0 ** -200], 1.0 + 2.0 ** -52),  # above the tie
             ([1.0 + 2.0 ** -52, 2.0 ** -53], 1.0 + 2.0 ** -51),  # tie: to even (up)
             ([1.7e308, 1.7e308], np.inf), ([-1.5, 0.25], -1.25), ([0.0, -0.0], 0.0)]
    for v, want in cases:
        v = np.array(v)
        assert O.xdot(v, one[:len(v)]) == want, (v, O.xdot(v, one[:len(v)]), want)
    a, b = rng.standard_normal(500_000), rng.standard_normal(500_000)
    vals = []
    for t in (1, 2, 5, 8):
        O.set_threads(t)
        try:
            vals.append(O.xdot(a, b))
        finally:
            O.set_threads(1)
    assert len(set(vals)) == 1


def test_exact_norm2_formula():
    """the exact mode's norm([a b]) (shared with the device): exact on Pythagorean triples,
    no overflow or underflow at the ends of the range, within an ulp of hypot elsewhere"""
    import math
    assert O.xnorm2(3.0, 4.0) == 5.0 and O.xnorm2(-5.0, 12.0) == 13.0
    assert O.xnorm2(0.0, -2.5) == 2.5 and O.xnorm2(0.0, 0.0) == 0.0
    assert O.xnorm2(1e300, 1e300) == math.hypot(1e300, 1e300)
    assert O.xnorm2(3e-310, 4e-310) == math.hypot(3e-310, 4e-310)
    rng = np.random.default_rng(5)
    for x, y in rng.standard_normal((2000, 2)) * np.exp(rng.uniform(-20, 20, (2000, 2))):
        h = math.hypot(x, y)
        assert abs(O.xnorm2(x, y) - h) <= math.ulp(h)
