"""Device numeric LDL' factorization (ldl.hip) and refactorization.

Reference: [L,D,P] = ldl(op.A) in the opLDL2 constructor (ops/opLDL2.m:81-82), rebuilt whenever
G, B or C change (reg_cpkrylov.m:131 per outer iteration of an interior-point method).

  * bit-exact: the device factors (L, D in the exported CSC layout, perm) equal the host
    factorization's (cpk_analyze, CPK_HOST_FACTOR path) -- same up-looking algorithm, same
    operation order, no FMA;
  * bit-exact: a refactorization with new values equals a fresh construction on those values
    (factors and M*z), and M*z still equals the oracle's multiply with the exported factors;
  * independent: the oracle's own LDL' (oracle/cpk_oracle.c, Davis's stack order of the row
    reach) with the same pivot order agrees within rounding, and P'*Kp*P = L*D*L' holds to
    rounding (scipy, no shared code).
"""
import numpy as np
import pytest
import scipy.sparse as sp

import fixtures as F
from cpkrylov_amd.synthetic import nonsym_system, saddle_system
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _system(name):
    if name == "syn_symm200k":
        S = saddle_system(N=200000, seed=5)
        return dict(G=S["G"], B=S["B"], C=S["C"], Q=S["Q"])
    if name == "syn_nonsym100k":
        S = nonsym_system(N=100000, seed=6)
        return dict(G=S["G"], B=S["B"], C=S["C"], Q=S["Q"])
    return F.load(name)


NAMES = ["cvxqp1_m", "cvxqp2_s", "syn_symm200k", "syn_nonsym100k"]


def _kp(S):
    return sp.bmat([[S["G"], S["B"].T], [S["B"], -S["C"]]]).tocsr()


@pytest.mark.parametrize("name", NAMES)
def test_device_factor_equals_host(gpu_ctx, name):
    import cpkrylov_amd as cpk
    S = _system(name)
    M = cpk.opLDL2(S["G"], S["B"], -S["C"])
    L, D, perm = M.export_factors()
    H = cpk.analyze(S["G"], S["B"], -S["C"])  # host numeric phase, same symbolic analysis
    assert np.array_equal(perm, H["perm"])
    assert np.array_equal(L.indptr, H["L"].indptr) and np.array_equal(L.indices, H["L"].indices)
    assert np.array_equal(L.data, H["L"].data), np.max(np.abs(L.data - H["L"].data))
    assert np.array_equal(D, H["D"])


@pytest.mark.parametrize("name", NAMES)
def test_device_factor_independent_checks(gpu_ctx, name):
    """Against code that shares nothing with the product: the oracle's factorization in Davis's
    stack order, and the reconstruction P'*Kp*P = L*D*L' in scipy."""
    import cpkrylov_amd as cpk
    S = _system(name)
    M = cpk.opLDL2(S["G"], S["B"], -S["C"])
    L, D, perm = M.export_factors()
    Mo = O.LDL2(S["G"], S["B"], -S["C"], perm=perm)
    Lo, Do, permo = Mo.factors()
    assert np.array_equal(permo, perm)
    assert np.array_equal(Lo.indptr, L.indptr) and np.array_equal(Lo.indices, L.indices)
    scale = max(np.max(np.abs(L.data)), 1.0)
    assert np.max(np.abs(L.data - Lo.data)) <= 1e-10 * scale
    assert np.max(np.abs(D - Do) / np.abs(Do)) <= 1e-10
    K = _kp(S)[perm][:, perm]
    N = K.shape[0]
    Lu = L + sp.identity(N, format="csc")
    R = K - Lu @ sp.diags(D) @ Lu.T
    assert abs(R).max() <= 1e-12 * abs(K).max() * max(1.0, abs(Lu).max() ** 2)


@pytest.mark.parametrize("name", NAMES)
def test_refactor_equals_fresh_construction(gpu_ctx, name):
    import cpkrylov_amd as cpk
    S = _system(name)
    rng = np.random.default_rng(17)
    M = cpk.opLDL2(S["G"], S["B"], -S["C"])
    M.nitref, M.force_itref = 1, True
    # an IPM-like update: new positive diagonal G, rescaled B and C, same sparsity
    G2 = S["G"].copy()
    G2.data = G2.data * rng.uniform(0.5, 2.0, G2.data.shape[0])
    B2 = S["B"].copy()
    B2.data = B2.data * rng.uniform(0.8, 1.25, B2.data.shape[0])
    C2 = S["C"].copy()
    C2.data = C2.data * 3.0
    t = M.refactor(G2, B2, -C2)
    assert t > 0
    M2 = cpk.opLDL2(G2, B2, -C2)
    M2.nitref, M2.force_itref = 1, True
    (L, D, perm), (L2, D2, perm2) = M.export_factors(), M2.export_factors()
    assert np.array_equal(perm, perm2) and np.array_equal(L.data, L2.data) and np.array_equal(D, D2)
    z = rng.standard_normal(M.n)
    y = M * z
    assert np.array_equal(y, M2 * z)
    assert np.array_equal(M.divide(z), M2.divide(z))
    Mo = O.LDL2(G2, B2, -C2, factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    assert np.array_equal(y, Mo @ z)


def test_refactor_rejects_other_sparsity(gpu_ctx):
    import cpkrylov_amd as cpk
    S = _system("cvxqp2_s")
    M = cpk.opLDL2(S["G"], S["B"], -S["C"])
    B2 = S["B"].tolil()
    i, j = 0, int(np.setdiff1d(np.arange(B2.shape[1]), S["B"][0].indices)[0])
    B2[i, j] = 0.5
    with pytest.raises(cpk.CpkError):
        M.refactor(S["G"], B2.tocsr(), -S["C"])


def test_refactor_zero_pivot_reported(gpu_ctx):
    import cpkrylov_amd as cpk
    S = _system("cvxqp2_s")
    M = cpk.opLDL2(S["G"], S["B"], -S["C"])
    G0 = S["G"].copy()
    G0.data = G0.data * 0.0
    M.nitref, M.force_itref = 1, True
    z = np.random.default_rng(4).standard_normal(M.n)
    y0, k0 = M * z, M.divide(z)
    L0, D0, _ = M.export_factors()
    with pytest.raises(cpk.CpkError) as e:
        M.refactor(G0, S["B"], -S["C"])
    assert "pivot" in str(e.value)
    # all or nothing: the failed refactorization left Kp, the factors and the sweeps untouched
    L1, D1, _ = M.export_factors()
    assert np.array_equal(L1.data, L0.data) and np.array_equal(D1, D0)
    assert np.array_equal(M * z, y0)
    assert np.array_equal(M.divide(z), k0)


def test_refactor_resets_handle_state(gpu_ctx):
    """A refactorization is a rebuilt opLDL2, whose constructor zeroes op.Aty and op.Cy
    (opLDL2.m:90-91): with handle semantics on, the first apply after it equals the first
    apply of a fresh preconditioner."""
    import cpkrylov_amd as cpk
    S = _system("cvxqp2_s")
    rng = np.random.default_rng(6)
    z1, z2 = rng.standard_normal(S["G"].shape[0] + S["B"].shape[0]), rng.standard_normal(S["G"].shape[0] + S["B"].shape[0])
    M = cpk.opLDL2(S["G"], S["B"], -S["C"])
    M.residual_update, M.nitref = True, 1
    M.handle_semantics = True
    M * z1  # leaves a nonzero state
    G2 = S["G"].copy()
    G2.data = G2.data * 1.5
    M.refactor(G2, S["B"], -S["C"])
    F = cpk.opLDL2(G2, S["B"], -S["C"])
    F.residual_update, F.nitref = True, 1
    F.handle_semantics = True
    assert np.array_equal(M * z2, F * z2)


def test_minres_after_refactor_matches_oracle(gpu_ctx):
    """cpminres with a refactored preconditioner vs the oracle's solve with its own factors."""
    import cpkrylov_amd as cpk
    P = F.load("cvxqp1_m")
    opts = dict(F.EXPROG_OPTS)
    M = cpk.opLDL2(P["G"], P["B"], -P["C"])
    G2 = P["G"].copy()
    G2.data = G2.data * 1.7
    M.refactor(G2, P["B"], -P["C"])
    M.nitref, M.force_itref, M.itref_tol = 1, True, 1e-8
    b = P["rhs"][:P["n"]]
    x, y, st = cpk.cpminres(b, P["Q"], P["C"], M, opts)[:3]
    perm = M.export_factors()[2]
    Mo = O.LDL2(G2, P["B"], -P["C"], perm=perm)
    Mo.set(nitref=1.0, force_itref=1.0)
    xo, yo, so = O.method("minres", b, P["Q"], P["C"], Mo, opts)
    assert st["niters"] == so["niters"]
    h, ho = st["residHistory"], so["residHistory"]
    assert len(h) == len(ho) and np.max(np.abs(h - ho)) <= 1e-8 * ho[0]
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)
