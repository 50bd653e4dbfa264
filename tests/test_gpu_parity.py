"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the reference's
example systems with the examples' options (cpk_exprog1.m:79-90, cpk_exprog2.m:69-90).

Parity bar:
  - bit-exact: niters, len(history), flag.solved; and the preconditioner apply given identical
    factors (every row sum runs in MATLAB's order, no FMA);
  - fp64 tolerance on histories and x.  Inner products are summed in a different order than
    the oracle's (and MATLAB's MKL order is unknown anyway), so the tolerance is the problem's
    own sensitivity: band = the oracle's largest deviation when the rhs is perturbed at the
    1e-15 level (sensitivity.py), and the GPU must agree within max(1e-8, 10*band) relative to
    history[0] (histories) or ||x_oracle|| (x);  the relative error against K\\rhs must be no
    worse than the oracle's (the examples' own check) when the solve converged.
"""
import numpy as np
import pytest

import fixtures as F
from oracle import oracle as O
from sensitivity import band

pytestmark = pytest.mark.gpu

FLOOR = 1e-8
SAFETY = 10.0

CASES = [
    ("cvxqp1_m", "minres", {}),
    ("cvxqp1_m", "cg", {}),
    ("cvxqp1_m", "cglanczos", {}),
    ("cvxqp1_m", "symmlq", {}),
    ("cvxqp1_m", "dqgmres", {"mem": 2}),
    ("cvxqp2_s", "gmres", {"restart": 100}),
    ("cvxqp2_s", "gmres", {"restart": 20}),
    ("cvxqp2_s", "dqgmres", {"mem": 100}),
    ("cvxqp2_s", "dqgmres", {"mem": 20}),
    # the benchmark generators at 20k dofs (S50's nonsymmetric 3x3 structure, S10's symmetric one)
    ("syn_nonsym20k", "dqgmres", {"mem": 40}),
    ("syn_nonsym20k", "gmres", {"restart": 40}),
    ("syn_symm20k", "minres", {}),
]


def _hist(stats):
    return stats.get("residHistory", stats.get("cgresidHistory"))


@pytest.mark.parametrize("name,method,extra", CASES)
def test_reg_cpkrylov_matches_oracle(gpu_ctx, name, method, extra):
    import cpkrylov_amd as cpk
    P = F.load(name)
    opts = dict(F.EXPROG_OPTS, **extra)
    fn = getattr(cpk, "cp" + method)
    x, stats, flag = cpk.reg_cpkrylov(fn, P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts)
    # oracle with the product's own ordering (same pivot sequence, independent factorization)
    perm = stats["M"].export_factors()[2]
    xo, so = O.reg_cpkrylov(method, P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts, perm=perm)
    assert stats["niters"] == so["niters"]
    assert flag["solved"] == so["solved"]
    bd = band(name, method, extra, perm)
    h0 = _hist(so)[0]
    for k in [k for k in so if k.endswith("History")]:
        assert len(stats[k]) == len(so[k]), k
        assert abs(stats[k][0] - so[k][0]) <= 1e-12 * h0, k
        dev = np.max(np.abs(stats[k] - so[k])) / h0
        assert dev <= max(FLOOR, SAFETY * bd[k]), (k, dev, bd[k])
    if method == "cglanczos":
        assert stats["status"] == so["status"]
    dx = np.linalg.norm(x - xo) / np.linalg.norm(xo)
    assert dx <= max(FLOOR, SAFETY * bd["x"]), (dx, bd["x"])
    if so["solved"]:
        err = np.linalg.norm(x - P["x_direct"]) / np.linalg.norm(P["x_direct"])
        err_o = np.linalg.norm(xo - P["x_direct"]) / np.linalg.norm(P["x_direct"])
        assert err <= err_o + max(FLOOR, SAFETY * bd["x"]), (err, err_o)


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s"])
@pytest.mark.parametrize("props", [dict(nitref=0), dict(nitref=1, force_itref=True),
                                   dict(nitref=3, force_itref=False, itref_tol=1e-8),
                                   dict(nitref=2, force_itref=False, itref_tol=1e-30)])
def test_precond_apply_bitexact(gpu_ctx, name, props):
    """M*z on the device equals the oracle's opLDL2.multiply bit for bit given the same factors
    (the refinement branch decision depends on norms, whose summation order differs; the
    itref_tol values here keep that decision away from its threshold)."""
    import cpkrylov_amd as cpk
    P = F.load(name)
    M = cpk.opLDL2(P["G"], P["B"], -P["C"])
    for k, v in props.items():
        setattr(M, k, v)
    L, D, perm = M.export_factors()
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=(L, D, perm))
    Mo.set(**{k: float(v) for k, v in props.items()})
    rng = np.random.default_rng(7)
    for _ in range(3):
        z = rng.standard_normal(P["n"] + P["m"])
        y = M * z
        yo = Mo @ z
        assert np.array_equal(y, yo), np.max(np.abs(y - yo))


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s"])
@pytest.mark.parametrize("props", [dict(nitref=0), dict(nitref=1, force_itref=True)])
def test_precond_apply_handle_semantics_bitexact(gpu_ctx, name, props):
    """Opt-in handle semantics of the residual-update state (cpk_pc_set_handle): a sequence of
    applies carries [op.Aty; op.Cy] from one to the next, bit-identical to the oracle's."""
    import cpkrylov_amd as cpk
    P = F.load(name)
    M = cpk.opLDL2(P["G"], P["B"], -P["C"])
    for k, v in dict(props, residual_update=True).items():
        setattr(M, k, v)
    M.handle_semantics = True
    L, D, perm = M.export_factors()
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=(L, D, perm))
    Mo.set(**{k: float(v) for k, v in dict(props, residual_update=1).items()})
    Mo.set_handle(True)
    rng = np.random.default_rng(9)
    ys = []
    for _ in range(4):
        z = rng.standard_normal(P["n"] + P["m"])
        y, yo = M * z, Mo @ z
        assert np.array_equal(y, yo), np.max(np.abs(y - yo))
        ys.append(y)
    M.handle_semantics = False  # back to the reference's value semantics
    z = rng.standard_normal(P["n"] + P["m"])
    Mo.set_handle(False)
    assert np.array_equal(M * z, Mo @ z)


def test_minres_handle_semantics_matches_oracle(gpu_ctx):
    """cpminres with the stateful residual update on the device vs the oracle with the same."""
    import cpkrylov_amd as cpk
    P = F.load("cvxqp1_m")
    opts = dict(F.EXPROG_OPTS)
    M = cpk.opLDL2(P["G"], P["B"], -P["C"])
    M.handle_semantics = True
    L, D, perm = M.export_factors()
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=(L, D, perm))
    Mo.set_handle(True)
    b = P["rhs"][:P["n"]]
    x, y, st = cpk.cpminres(b, P["Q"], P["C"], M, opts)[:3]
    xo, yo, so = O.method("minres", b, P["Q"], P["C"], Mo, opts)
    assert st["niters"] == so["niters"]
    h, ho = st["residHistory"], so["residHistory"]
    assert len(h) == len(ho) and np.max(np.abs(h - ho)) <= 1e-8 * ho[0]
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s"])
def test_spmv_bitexact(gpu_ctx, name):
    import cpkrylov_amd as cpk
    P = F.load(name)
    rng = np.random.default_rng(3)
    for M in (P["K"], P["Q"], P["B"], P["B"].T.tocsr()):
        x = rng.standard_normal(M.shape[1])
        y = cpk.Matrix(M) @ x
        # MATLAB order: per row, 0 + a1*x1 + a2*x2 + ... (no FMA)
        Mc = M.tocsr()
        yr = np.zeros(M.shape[0])
        for i in range(M.shape[0]):
            acc = 0.0
            for p in range(Mc.indptr[i], Mc.indptr[i + 1]):
                acc = acc + Mc.data[p] * x[Mc.indices[p]]
            yr[i] = acc
        assert np.array_equal(y, yr)


def test_divide_and_transpose(gpu_ctx):
    import cpkrylov_amd as cpk
    P = F.load("cvxqp2_s")
    M = cpk.opLDL2(P["G"], P["B"], -P["C"])
    z = np.random.default_rng(1).standard_normal(M.n)
    Kp = __import__("scipy.sparse", fromlist=["bmat"]).bmat([[P["G"], P["B"].T], [P["B"], -P["C"]]]).tocsr()
    assert np.allclose(M.divide(z), Kp @ z, rtol=0, atol=1e-12 * np.abs(Kp).max() * np.abs(z).max())
    assert M.T is M
    M.nitref = 3
    y = M * z
    assert np.linalg.norm(Kp @ y - z) <= 1e-8 * np.linalg.norm(z)


@pytest.mark.parametrize("sweep", ["1024,3072,256", "512,1536,128", "256,768,64", "64,128,64", "256,768,128,2048,8192,512", "192,576,64", "128,512,128", "384,1152,64,2048,8192,512,400", "512,1536,64,1024,4096,256,300", "192,576,32,1024,4096,512", "128,384,32,1024,4096,512"])
@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s", "synthetic"])
def test_precond_apply_bitexact_sweep_configs(gpu_ctx, name, sweep, monkeypatch):
    """Every LDS staging configuration (and the direct path for blocks that do not fit) gives
    the same bits as the oracle's column-oriented solve."""
    import cpkrylov_amd as cpk
    from cpkrylov_amd.synthetic import saddle_system
    monkeypatch.setenv("CPK_SWEEP", sweep)
    if name == "synthetic":
        S = saddle_system(N=50000)
        G, B, C = S["G"], S["B"], S["C"]
    else:
        P = F.load(name)
        G, B, C = P["G"], P["B"], P["C"]
    M = cpk.opLDL2(G, B, -C)
    M.nitref, M.force_itref = 1, True
    L, D, perm = M.export_factors()
    Mo = O.LDL2(G, B, -C, factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    z = np.random.default_rng(11).standard_normal(M.n)
    assert np.array_equal(M * z, Mo @ z)


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s", "synthetic"])
@pytest.mark.parametrize("props", [dict(nitref=0), dict(nitref=1, force_itref=True), dict(nitref=2, force_itref=True)])
def test_precond_apply_bitexact_detached_rows(gpu_ctx, name, props, monkeypatch):
    """Opt-in schedule with the entry-less rows outside the blocks (CPK_DETACH: a streaming pass
    per sweep) and the refinement in schedule order: the same bits as the oracle."""
    import cpkrylov_amd as cpk
    from cpkrylov_amd.synthetic import saddle_system
    monkeypatch.setenv("CPK_DETACH", "1")
    if name == "synthetic":
        S = saddle_system(N=50000)
        G, B, C = S["G"], S["B"], S["C"]
    else:
        P = F.load(name)
        G, B, C = P["G"], P["B"], P["C"]
    M = cpk.opLDL2(G, B, -C)
    for k, v in props.items():
        setattr(M, k, v)
    L, D, perm = M.export_factors()
    Mo = O.LDL2(G, B, -C, factors=(L, D, perm))
    Mo.set(**{k: float(v) for k, v in props.items()})
    z = np.random.default_rng(12).standard_normal(M.n)
    assert np.array_equal(M * z, Mo @ z)


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s"])
def test_precond_apply_plain_refinement_path(gpu_ctx, name, monkeypatch):
    """CPK_NO_SCHED_RESID: the refinement through the original-order residual and scatter,
    the same bits as the schedule-order path and the oracle."""
    import cpkrylov_amd as cpk
    P = F.load(name)
    z = np.random.default_rng(13).standard_normal(P["n"] + P["m"])
    ys = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("CPK_NO_SCHED_RESID", env)
        M = cpk.opLDL2(P["G"], P["B"], -P["C"])
        M.nitref, M.force_itref = 2, True
        ys.append(M * z)
    L, D, perm = M.export_factors()
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=(L, D, perm))
    Mo.set(nitref=2.0, force_itref=1.0)
    assert np.array_equal(ys[0], ys[1]) and np.array_equal(ys[0], Mo @ z)


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s", "syn_symm20k"])
def test_precond_apply_int32_round0_columns(gpu_ctx, name, monkeypatch):
    """CPK_NO_COL16: round 0's forward sweep stages int32 global columns with the locality test
    instead of the stored block-local int16 columns; the same bits as the default path and the
    oracle."""
    import cpkrylov_amd as cpk
    P = F.load(name)
    z = np.random.default_rng(17).standard_normal(P["n"] + P["m"])
    ys = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("CPK_NO_COL16", env)
        M = cpk.opLDL2(P["G"], P["B"], -P["C"])
        M.nitref, M.force_itref = 1, True
        ys.append(M * z)
    L, D, perm = M.export_factors()
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    assert np.array_equal(ys[0], ys[1]) and np.array_equal(ys[0], Mo @ z)


@pytest.mark.parametrize("sweep", [None, "256,768,64", "256,768,128,2048,8192,512", "384,1152,64,2048,8192,512,400"])
@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s", "synthetic"])
def test_precond_apply_fused_residual(gpu_ctx, name, sweep, monkeypatch):
    """The refinement residual formed inside the round-0 forward sweep (launch_sptrsv_fwd_resid,
    opLDL2.m:175-182) against the separate residual SpMV (CPK_NO_FUSED_RESID) and the oracle:
    the same bits, for one and two refinement steps.  The cvxqp rows carry more Kps entries per
    block than one LDS chunk holds, so the kernel's chunk loop runs too."""
    import cpkrylov_amd as cpk
    from cpkrylov_amd.synthetic import saddle_system
    if sweep:
        monkeypatch.setenv("CPK_SWEEP", sweep)
    if name == "synthetic":
        S = saddle_system(N=50000)
        G, B, C = S["G"], S["B"], S["C"]
    else:
        P = F.load(name)
        G, B, C = P["G"], P["B"], P["C"]
    z = np.random.default_rng(19).standard_normal(G.shape[0] + B.shape[0])
    for steps in (1, 2):
        ys = []
        for env in (None, "1"):
            if env:
                monkeypatch.setenv("CPK_NO_FUSED_RESID", env)
            else:
                monkeypatch.delenv("CPK_NO_FUSED_RESID", raising=False)
            M = cpk.opLDL2(G, B, -C)
            M.nitref, M.force_itref = steps, True
            ys.append(M * z)
        L, D, perm = M.export_factors()
        Mo = O.LDL2(G, B, -C, factors=(L, D, perm))
        Mo.set(nitref=float(steps), force_itref=1.0)
        yo = Mo @ z
        assert np.array_equal(ys[1], yo), np.max(np.abs(ys[1] - yo))
        assert np.array_equal(ys[0], yo), np.max(np.abs(ys[0] - yo))


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s", "synthetic"])
def test_precond_apply_fused_residual_tail_launch(gpu_ctx, name, monkeypatch):
    """The rows above round 0 take their residual from a separate launch (CPK_FUSED_TAIL_LAUNCH)
    instead of the round-0 kernel's workgroups: the same bits either way, and as the oracle."""
    import cpkrylov_amd as cpk
    from cpkrylov_amd.synthetic import saddle_system
    if name == "synthetic":
        S = saddle_system(N=50000)
        G, B, C = S["G"], S["B"], S["C"]
    else:
        P = F.load(name)
        G, B, C = P["G"], P["B"], P["C"]
    z = np.random.default_rng(23).standard_normal(G.shape[0] + B.shape[0])
    ys = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("CPK_FUSED_TAIL_LAUNCH", env)
        M = cpk.opLDL2(G, B, -C)
        M.nitref, M.force_itref = 1, True
        ys.append(M * z)
    L, D, perm = M.export_factors()
    Mo = O.LDL2(G, B, -C, factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    assert np.array_equal(ys[0], ys[1]) and np.array_equal(ys[0], Mo @ z)
