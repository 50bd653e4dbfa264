"""The boundary the MATLAB side actually uses, through the C ABI on the GPU.

  * MATLAB-native CSC input (cpk_mat_create_csc: 0-based size_t jc / ir, what the MEX gateway
    hands over, matlab/cpk_mex.c) gives the same device results as the CSR entry: a bit-identical
    SpMV and M*z.
  * opLDL2's property setters through cpk_pc_set / cpk_pc_get keep the reference's edge
    semantics (ops/opLDL2.m:97-115): nitref = max(0, round(v)) with MATLAB's round-half-away,
    force_itref other than 0/1 -> false, itref_tol stored as given (the `sef` typo), and the
    apply then equals the oracle's with the same setter sequence, bit for bit.
  * cpcglanczos' backward-error stop (kernels/cpcglanczos.m:271-291, status 'backward error
    small', :320-325) on cvxqp1_m against the oracle.
  * A distributed preconditioner's operator caches die with it: two reg_cpkrylov calls that
    share the A and C Matrix objects but use different B each match the oracle (SimComm P=2).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import scipy.sparse as sp

import fixtures as F
from oracle import oracle as O
from sensitivity import band

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s"])
def test_csc_entry_bitexact(gpu_ctx, name):
    import cpkrylov_amd as cpk
    P = F.load(name)
    rng = np.random.default_rng(21)
    for M in (P["K"], P["Q"], P["B"], P["B"].T.tocsr()):
        x = rng.standard_normal(M.shape[1])
        assert np.array_equal(cpk.Matrix(M, csc=True) @ x, cpk.Matrix(M) @ x)
    mats = [cpk.Matrix(M, csc=True) for M in (P["G"], P["B"], -P["C"])]
    Mc = cpk.opLDL2(*mats)
    Mr = cpk.opLDL2(P["G"], P["B"], -P["C"])
    for M in (Mc, Mr):
        M.nitref, M.force_itref = 1, True
    for a, b in zip(Mc.export_factors(), Mr.export_factors()):
        assert (a != b).nnz == 0 if sp.issparse(a) else np.array_equal(a, b)
    z = rng.standard_normal(Mc.n)
    assert np.array_equal(Mc * z, Mr * z)


SETTER_CASES = [
    # (value set, value read back) -- opLDL2.m:97-115
    ("nitref", 2.5, 3.0), ("nitref", -4, 0.0), ("nitref", 1.49, 1.0), ("nitref", -0.5, 0.0),
    ("force_itref", 2, 0.0), ("force_itref", -1, 0.0), ("force_itref", 1, 1.0), ("force_itref", 0, 0.0),
    ("itref_tol", -1.0, -1.0), ("itref_tol", 1e300, 1e300), ("residual_update", 7.0, 7.0),
]


@pytest.mark.parametrize("prop,val,expect", SETTER_CASES)
def test_setter_semantics_through_abi(gpu_ctx, prop, val, expect):
    import cpkrylov_amd as cpk
    from cpkrylov_amd import _lib
    P = F.load("cvxqp2_s")
    M = cpk.opLDL2(P["G"], P["B"], -P["C"])
    import ctypes as C
    _lib.check(_lib.lib.cpk_pc_set(M.h, C.byref(_lib.make_opts({prop: val}))))
    got = dict(zip(("nitref", "itref_tol", "force_itref", "residual_update"), M._get()))
    assert got[prop] == expect, (prop, val, got[prop])
    # the oracle's setters restate the same semantics; with them the applies agree bit for bit
    L, D, perm = M.export_factors()
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=(L, D, perm))
    Mo.set(**{prop: float(val)})
    assert Mo.props()[prop] == expect
    z = np.random.default_rng(4).standard_normal(M.n)
    y, yo = M * z, Mo @ z  # itref_tol < 0: rNorm >= tol * xNorm always holds, every step runs
    assert np.array_equal(y, yo), np.max(np.abs(y - yo))


@pytest.mark.parametrize("btol", [1e-3, 1e-5, 1e-7, 1e-8])
def test_cglanczos_backward_error_stop(gpu_ctx, btol):
    import cpkrylov_amd as cpk
    P = F.load("cvxqp1_m")
    opts = dict(F.EXPROG_OPTS, btol=btol)
    x, stats, flag = cpk.reg_cpkrylov(cpk.cpcglanczos, P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts)
    perm = stats["M"].export_factors()[2]
    xo, so = O.reg_cpkrylov("cglanczos", P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts, perm=perm)
    assert stats["niters"] == so["niters"]
    assert flag["solved"] == so["solved"]
    assert stats["status"] == so["status"]
    if btol >= 1e-7:
        assert so["status"] == "backward error small"
    h, ho = stats["residHistory"], so["residHistory"]
    bd = band("cvxqp1_m", "cglanczos", {"btol": btol}, perm)
    assert len(h) == len(ho)
    assert np.max(np.abs(h - ho)) / ho[0] <= max(1e-8, 10 * bd["residHistory"])
    assert np.linalg.norm(x - xo) / np.linalg.norm(xo) <= max(1e-8, 10 * bd["x"])


def test_dist_operator_cache_follows_preconditioner():
    """the distributed Krylov operator and shift rows follow a preconditioner's
    dof map.  Two solves sharing the A and C Matrix objects with different B (so different
    preconditioners, possibly at a recycled address) must each match the oracle."""
    import cpkrylov_amd as cpk
    P = F.load("cvxqp1_m")
    B2 = P["B"].copy()
    B2.data = B2.data * 1.5
    B2 = (B2 + sp.random(B2.shape[0], B2.shape[1], density=2e-4, random_state=3, format="csr")).tocsr()
    opts = dict(F.EXPROG_OPTS)
    Pn = 2
    g = cpk.SimGroup(Pn)

    def one(r):
        ctx = cpk.Context(device=0, rank=r, nranks=Pn, simgroup=g)
        try:
            A, Cm, G = cpk.Matrix(P["Q"], ctx), cpk.Matrix(P["C"], ctx), cpk.Matrix(P["G"], ctx)
            out = []
            for B in (P["B"], B2, P["B"]):
                x, stats, flag = cpk.reg_cpkrylov(cpk.cpminres, P["rhs"], A, cpk.Matrix(B, ctx), Cm, G, opts,
                                                  ctx=ctx)
                perm = stats["M"].export_factors()[2] if r == 0 else None
                del stats["M"]  # the preconditioner dies here; the next one may reuse its address
                out.append((x, stats, flag, perm))
            return out
        finally:
            ctx.close()

    with ThreadPoolExecutor(Pn) as ex:
        res = [f.result(timeout=600) for f in [ex.submit(one, r) for r in range(Pn)]]
    for i, B in enumerate((P["B"], B2, P["B"])):
        x, stats, flag, perm = res[0][i]
        assert np.array_equal(res[1][i][0], x)
        xo, so = O.reg_cpkrylov("minres", P["rhs"], P["Q"], B, P["C"], P["G"], opts, perm=perm)
        assert stats["niters"] == so["niters"], i
        h, ho = stats["residHistory"], so["residHistory"]
        assert np.max(np.abs(h - ho)) / ho[0] <= 1e-8, i
        assert np.linalg.norm(x - xo) / np.linalg.norm(xo) <= 1e-8, i


def test_precond_create_dimension_errors(gpu_ctx):
    """opLDL2's dimension checks (opLDL2.m:61-75) run before any helper
    thread reads the blocks, so mismatched G and B raise CPK_ERR_DIM instead of writing past an
    array -- through the device constructor, not only the host analysis."""
    import cpkrylov_amd as cpk
    from cpkrylov_amd import _lib
    P = F.load("cvxqp1_m")
    for G, B, Cm in ((P["G"][:10, :10], P["B"], -P["C"]), (P["G"], P["B"][:, :10], -P["C"]),
                     (P["G"], P["B"], -P["C"][:5, :5]), (P["G"][:, :10], P["B"], -P["C"])):
        with pytest.raises(cpk.CpkError) as e:
            cpk.opLDL2(G, B, Cm)
        assert e.value.code == _lib.CPK_ERR_DIM
    M = cpk.opLDL2(P["G"], P["B"], -P["C"])  # the library is still usable
    assert M.n == P["n"] + P["m"]


def test_context_info_and_per_path_sweep_default(gpu_ctx):
    """cpk_ctx_get_info reports the communicator a context holds, and an unset sweep option
    reports the default of the context's path: the single-GPU one on a plain context, the
    distributed one (dist_sweep_default) on a distributed context, which its preconditioners
    then use; an explicit sweep wins on either path.  The timing stand-in is a constructor of
    its own and says so."""
    import cpkrylov_amd as cpk
    single = cpk.Context(device=0)
    try:
        assert single.info() == {"device": 0, "rank": 0, "nranks": 1, "comm": "none", "comm_ranks": 0,
                                 "distributed": False}
        assert single.get_option("sweep") == "192,576,64,512,3072,256,480"
        assert "sweep=192,576,64,512,3072,256,480;" in single.options_string()
    finally:
        single.close()
    g = cpk.SimGroup(2)

    def one(r):
        ctx = cpk.Context(device=0, rank=r, nranks=2, simgroup=g)
        try:
            info = ctx.info()
            default = ctx.get_option("sweep")
            P = F.load("cvxqp1_m")
            M = cpk.opLDL2(P["G"], P["B"], -P["C"], ctx=ctx)
            rounds = M.sweep_info()["rounds"]
            ctx.set_option("sweep", "192,576,64,512,3072,256,480")
            explicit = ctx.get_option("sweep")
            ctx.set_option("sweep_set", "0")
            back = ctx.get_option("sweep")
            del M
            return info, default, explicit, back, rounds
        finally:
            ctx.close()

    with ThreadPoolExecutor(2) as ex:
        res = [f.result(timeout=600) for f in [ex.submit(one, r) for r in range(2)]]
    for r, (info, default, explicit, back, rounds) in enumerate(res):
        assert info == {"device": 0, "rank": r, "nranks": 2, "comm": "sim", "comm_ranks": 2, "distributed": True}
        assert default == "192,576,64,1024,4096,512,0" and back == default
        assert explicit == "192,576,64,512,3072,256,480"
        assert rounds >= 1
    null = cpk.Context(device=0, rank=3, nranks=8, timing_standin=True)
    try:
        assert null.info()["comm"] == "null" and null.info()["comm_ranks"] == 1
        assert null.get_option("sweep") == "192,576,64,1024,4096,512,0"
    finally:
        null.close()
