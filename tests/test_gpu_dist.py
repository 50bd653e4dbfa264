"""Distributed path on the GPU, rehearsed on one MI355X: P ranks run as
threads of this process, each with its own context and stream, exchanging through a shared HBM
buffer (cpk_ctx_create_sim) instead of RCCL -- RCCL refuses two ranks on one device, so the
RCCL transport itself is exercised by the 8-GPU bench only.

Parity bar:
  * M*z of the distributed preconditioner (local sweeps + separator exchange + redundant
    separator solve + halo'd residual SpMV) equals the oracle's opLDL2 apply bit for bit;
  * distributed solves match the oracle as the 1-GPU solves do (same niters, histories within
    the sensitivity band); only the inner products' summation order differs.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import fixtures as F
from cpkrylov_amd.synthetic import saddle_system
from oracle import oracle as O
from sensitivity import band

pytestmark = pytest.mark.gpu

FLOOR = 1e-8
SAFETY = 10.0


def _run_ranks(P, fn, options=None):
    """fn(ctx, rank) on P simulated ranks; returns the list of results.  options: engine options
    of every rank's context (a dict), or a function rank -> dict.  P = 1 sets dist1 (a 1-rank
    communicator otherwise runs the single-GPU path)."""
    import cpkrylov_amd as cpk
    g = cpk.SimGroup(P)

    def one(r):
        opt = options(r) if callable(options) else options
        if P == 1:
            opt = dict(opt or {}, dist1=1)
        ctx = cpk.Context(device=0, rank=r, nranks=P, simgroup=g, options=opt)
        try:
            return fn(ctx, r)
        finally:
            ctx.close()

    with ThreadPoolExecutor(P) as ex:
        futs = [ex.submit(one, r) for r in range(P)]
        return [f.result(timeout=600) for f in futs]


def _system(name):
    if name == "synthetic20k":
        S = saddle_system(N=20000, seed=3)
        return dict(Q=S["Q"], B=S["B"], C=S["C"], G=S["G"], n=S["n"], m=S["m"], rhs=S["rhs"])
    return F.load(name)


@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("name", ["cvxqp1_m", "synthetic20k"])
@pytest.mark.parametrize("props", [dict(nitref=0), dict(nitref=1, force_itref=True),
                                   dict(nitref=3, force_itref=False, itref_tol=1e-8)])
def test_dist_apply_bitexact(name, P, props):
    import cpkrylov_amd as cpk
    S = _system(name)
    z = np.random.default_rng(5).standard_normal(S["n"] + S["m"])

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        for k, v in props.items():
            setattr(M, k, v)
        d, nl = M.local_dofs()
        return M * z, M.export_factors() if r == 0 else None, d, nl

    res = _run_ranks(P, work)
    L, D, perm = res[0][1]
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(**{k: float(v) for k, v in props.items()})
    yo = Mo @ z
    for y, _, _, _ in res:
        assert np.array_equal(y, yo), np.max(np.abs(y - yo))
    # ownership: the local slices partition the dofs, x-part first
    alld = np.concatenate([d for _, _, d, _ in res])
    assert np.array_equal(np.sort(alld), np.arange(S["n"] + S["m"]))
    for _, _, d, nl in res:
        assert np.all(d[:nl] < S["n"]) and np.all(d[nl:] >= S["n"])


@pytest.mark.parametrize("P", [1, 2, 4])
@pytest.mark.parametrize("name", ["cvxqp1_m", "synthetic20k"])
def test_dist_apply_sweep_chain_bitexact(name, P):
    """The sweep chains on a distributed preconditioner: each rank's forward upper rounds in one
    launch (kChainFwd, before the separator exchange) and its backward upper rounds in one launch
    (kChainBwd, after the separator solve) -- at P = 1 the full chain with the last round fused --
    against one launch per round (no_chain) and the oracle, with small upper blocks (many rounds),
    three applies with one forced refinement step."""
    import cpkrylov_amd as cpk
    S = _system(name)
    rng = np.random.default_rng(53)
    zs = [rng.standard_normal(S["n"] + S["m"]) for _ in range(3)]

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        M.nitref, M.force_itref = 1, True
        return [M * z for z in zs], M.export_factors() if r == 0 else None, M.sweep_info()["chain_tasks"]

    res = {}
    for off in (False, True):
        res[off] = _run_ranks(P, work, dict(sweep="64,192,64,128,512,512", no_chain=off))
        chains = [ch for _, _, ch in res[off]]
        assert (max(chains) > 0) != off, chains
    L, D, perm = res[False][0][1]
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    for i, z in enumerate(zs):
        yo = Mo @ z
        for off in (False, True):
            for ys, _, _ in res[off]:
                assert np.array_equal(ys[i], yo), (off, np.max(np.abs(ys[i] - yo)))


@pytest.mark.parametrize("P", [1, 2, 3, 4])
@pytest.mark.parametrize("name", ["cvxqp1_m", "synthetic20k"])
def test_dist_refinement_without_kp_halo(name, P):
    """One forced refinement step (the example options) without the Kp halo exchange: every
    rank's local rows read T's solution from its own separator solve, the T rows' residual is
    formed after the refinement's separator exchange.  Three paths: the default keeps the first
    solve's solution in schedule order and fuses the subtree rows' residual into the refinement
    solve's forward sweep (Precond::dist_sched_apply); engine option no_sched_resid runs the
    residual as a local SpMV in the original order; no_tkr restores the Kp halo exchange.  A
    sequence of applies, each bit for bit the oracle's on every path (P = 1: no separator)."""
    import cpkrylov_amd as cpk
    S = _system(name)
    rng = np.random.default_rng(41)
    zs = [rng.standard_normal(S["n"] + S["m"]) for _ in range(3)]

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        M.nitref, M.force_itref = 1, True
        return [M * z for z in zs], M.export_factors() if r == 0 else None, M.sep_info()

    for opts in (None, dict(no_fused_resid=True), dict(no_sched_resid=True), dict(no_tkr=True)):
        res = _run_ranks(P, work, opts)
        for _, _, info in res:
            sep = info["nT"] > 0
            assert info["sched"] == (0 if opts and ("no_sched_resid" in opts or ("no_tkr" in opts and sep)) else 1), (opts, info)
            assert info["tkr"] == (1 if sep and not (opts and "no_tkr" in opts) else 0), (opts, info)
            if opts and "no_fused_resid" in opts:
                assert info["fused"] == 0, (opts, info)
            assert sep == (P > 1)
        if name == "synthetic20k" and not opts:  # (a rank without subtree rows has nothing to fuse)
            assert all(info["fused"] == 1 for _, _, info in res), [info for _, _, info in res]
        L, D, perm = res[0][1]
        Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
        Mo.set(nitref=1.0, force_itref=1.0)
        for k, z in enumerate(zs):
            yo = Mo @ z
            for ys, _, _ in res:
                assert np.array_equal(ys[k], yo), (opts, k, np.max(np.abs(ys[k] - yo)))


DIST_CASES = [("cvxqp1_m", "minres", {}), ("cvxqp1_m", "cg", {}), ("cvxqp1_m", "cglanczos", {}),
              ("cvxqp1_m", "symmlq", {}), ("cvxqp1_m", "dqgmres", {"mem": 2}),
              ("cvxqp2_s", "gmres", {"restart": 20}), ("cvxqp2_s", "gmres", {"restart": 100}),
              ("cvxqp2_s", "dqgmres", {"mem": 20}), ("cvxqp2_s", "dqgmres", {"mem": 100}),
              ("syn_nonsym20k", "dqgmres", {"mem": 40})]


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("name,method,extra", DIST_CASES)
def test_dist_reg_cpkrylov_matches_oracle(name, method, extra, P):
    import cpkrylov_amd as cpk
    Pd = F.load(name)
    opts = dict(F.EXPROG_OPTS, **extra)
    fn = getattr(cpk, "cp" + method)

    def work(ctx, r):
        x, stats, flag = cpk.reg_cpkrylov(fn, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, ctx=ctx)
        perm = stats["M"].export_factors()[2] if r == 0 else None
        return x, {k: v for k, v in stats.items() if k != "M"}, flag, perm

    res = _run_ranks(P, work)
    x, stats, flag, perm = res[0]
    for xr, sr, fr, _ in res[1:]:  # every rank returns the same global answer
        assert np.array_equal(xr, x) and sr["niters"] == stats["niters"] and fr == flag
    xo, so = O.reg_cpkrylov(method, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, perm=perm)
    assert stats["niters"] == so["niters"]
    assert flag["solved"] == so["solved"]
    bd = band(name, method, extra, perm)
    h0 = stats.get("residHistory", stats.get("cgresidHistory"))[0]
    for k in [k for k in so if k.endswith("History")]:
        assert len(stats[k]) == len(so[k]), k
        dev = np.max(np.abs(stats[k] - so[k])) / h0
        assert dev <= max(FLOOR, SAFETY * bd[k]), (k, dev, bd[k])
    dx = np.linalg.norm(x - xo) / np.linalg.norm(xo)
    assert dx <= max(FLOOR, SAFETY * bd["x"]), (dx, bd["x"])


@pytest.mark.parametrize("P", [4, 8])
def test_dist_live_refinement_solve(P):
    """Data-dependent refinement (nitref = 3, force_itref = false: the norms and the predicate live
    on the device) inside a distributed cpminres, at rank counts where a rank of cvxqp1_m's split
    may own no rows (its solver vectors are then empty: round 5 found such a rank passing null
    vectors to the accumulating backward sweep).  Every rank returns the same answer and the
    solve tracks the oracle within the sensitivity band."""
    import cpkrylov_amd as cpk
    name, method, extra = "cvxqp1_m", "minres", {"nitref": 3, "force_itref": False}
    Pd = F.load(name)
    opts = dict(F.EXPROG_OPTS, **extra)

    def work(ctx, r):
        x, stats, flag = cpk.reg_cpkrylov(cpk.cpminres, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, ctx=ctx)
        M = stats["M"]
        perm = M.export_factors()[2] if r == 0 else None
        return x, {k: v for k, v in stats.items() if k != "M"}, flag, perm, len(M.local_dofs()[0])

    res = _run_ranks(P, work)
    x, stats, flag, perm, _ = res[0]
    sizes = [s for *_, s in res]
    for xr, sr, fr, _, _ in res[1:]:
        assert np.array_equal(xr, x) and sr["niters"] == stats["niters"] and fr == flag, sizes
    xo, so = O.reg_cpkrylov(method, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, perm=perm)
    assert stats["niters"] == so["niters"] and flag["solved"] == so["solved"], sizes
    bd = band(name, method, extra, perm)
    dev = np.max(np.abs(stats["residHistory"] - so["residHistory"])) / stats["residHistory"][0]
    assert dev <= max(FLOOR, SAFETY * bd["residHistory"]), (dev, bd["residHistory"], sizes)
    dx = np.linalg.norm(x - xo) / np.linalg.norm(xo)
    assert dx <= max(FLOOR, SAFETY * bd["x"]), (dx, bd["x"], sizes)


def test_dist_device_vectors_synthetic():
    """Device-resident local slices (the bench's path): shift + cpminres on 4 ranks agree with
    the 1-GPU solve of the same system."""
    import ctypes as C

    import cpkrylov_amd as cpk
    from cpkrylov_amd import _lib
    from devbuf import DeviceArray
    S = saddle_system(N=60000, seed=9)
    opts = dict(F.EXPROG_OPTS)
    x1, st1, fl1 = cpk.reg_cpkrylov(cpk.cpminres, S["rhs"], S["Q"], S["B"], S["C"], S["G"], opts)

    def work(ctx, r):
        A, B, Cm = (cpk.Matrix(S[k], ctx) for k in ("Q", "B", "C"))
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        M.nitref, M.force_itref = 1, True
        d, nl = M.local_dofs()
        b = DeviceArray.of(S["rhs"][d])
        b1, xy0, xy = DeviceArray(nl), DeviceArray(len(d)), DeviceArray(len(d))
        sh = C.c_int()
        _lib.check(_lib.lib.cpk_reg_shift_device(ctx.h, b.p, A.h, B.h, Cm.h, M.h, b1.p, xy0.p, C.byref(sh)))
        st = _lib.Stats()
        hist = np.zeros(600)
        st.hist = hist.ctypes.data_as(C.POINTER(C.c_double))
        st.hist_cap = 600
        _lib.check(_lib.lib.cpk_method_solve_device(ctx.h, 2, b1.p, A.h, Cm.h, M.h, C.byref(_lib.make_opts(opts)),
                                                    xy.p, C.byref(st)))
        ctx.synchronize()
        x = xy0.numpy() + xy.numpy()
        return d, x, int(st.niters), hist[:st.hist_len].copy(), bool(sh.value)

    res = _run_ranks(4, work)
    x = np.empty(S["n"] + S["m"])
    for d, xl, it, h, sh in res:
        x[d] = xl
        assert sh and it == st1["niters"]
        assert np.max(np.abs(h - st1["residHistory"])) <= 1e-8 * st1["residHistory"][0]
    assert np.linalg.norm(x - x1) <= 1e-8 * np.linalg.norm(x1)


def test_rccl_one_rank_graph_capture():
    """The RCCL transport and hipGraph capture of its collectives, on the one GPU available.  A
    1-rank communicator runs the single-GPU path by default (nothing to exchange); with engine
    option dist1 it runs the distributed path (allreduce epilogues captured in the iteration
    graph).  With one rank every sum is the local one: both are bit-identical to the single-GPU
    path."""
    import cpkrylov_amd as cpk
    Pd = F.load("cvxqp1_m")
    opts = dict(F.EXPROG_OPTS)
    x1, s1, f1 = cpk.reg_cpkrylov(cpk.cpminres, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts)
    z = np.random.default_rng(5).standard_normal(Pd["n"] + Pd["m"])
    s1["M"].nitref, s1["M"].force_itref = 1, True
    y1 = s1["M"] * z
    for dist1 in (False, True):
        ctx = cpk.Context(device=0, rank=0, nranks=1, unique_id=cpk.get_unique_id(),
                          options={"dist1": 1} if dist1 else None)
        try:
            info = ctx.info()
            assert info["comm"] == "rccl" and info["comm_ranks"] == 1 and info["distributed"] == dist1, info
            x2, s2, f2 = cpk.reg_cpkrylov(cpk.cpminres, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, ctx=ctx)
            assert s2["niters"] == s1["niters"] and f2 == f1
            assert np.array_equal(s2["residHistory"], s1["residHistory"])
            assert np.array_equal(x2, x1)
            # dist1: the distributed apply runs the single-GPU kernel sequence (schedule order,
            # fused residual); without it the preconditioner is the single-GPU one
            sep = s2["M"].sep_info()
            assert sep["dist"] == int(dist1), sep
            if dist1:
                assert sep["sched"] == 1 and sep["fused"] == 1 and sep["nT"] == 0, sep
            s2["M"].nitref, s2["M"].force_itref = 1, True
            assert np.array_equal(s2["M"] * z, y1)
            # dist1 decides the path when the operators are built: flipping it afterwards is refused
            ctx.set_option("dist1", "0" if dist1 else "1")
            with pytest.raises(cpk.CpkError, match="dist1"):
                cpk.cpminres(Pd["rhs"][:Pd["n"]], Pd["Q"], Pd["C"], s2["M"], opts)
            del s2
        finally:
            ctx.close()


@pytest.mark.parametrize("P", [8])
def test_dist_more_ranks_than_subtrees(P):
    """A small system on many ranks: the separator set takes most rows and some ranks own
    nothing; the apply and a solve still agree with the oracle."""
    import cpkrylov_amd as cpk
    Pd = F.load("cvxqp2_s")
    z = np.random.default_rng(2).standard_normal(Pd["n"] + Pd["m"])
    opts = dict(F.EXPROG_OPTS, mem=20)

    def work(ctx, r):
        M = cpk.opLDL2(Pd["G"], Pd["B"], -Pd["C"], ctx=ctx)
        M.nitref, M.force_itref = 1, True
        y = M * z
        x, stats, flag = cpk.reg_cpkrylov(cpk.cpdqgmres, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, ctx=ctx)
        return y, M.export_factors() if r == 0 else None, len(M.local_dofs()[0]), stats["niters"], x

    res = _run_ranks(P, work)
    L, D, perm = res[0][1]
    Mo = O.LDL2(Pd["G"], Pd["B"], -Pd["C"], factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    yo = Mo @ z
    for y, _, _, it, x in res:
        assert np.array_equal(y, yo)
        assert it == res[0][3] and np.array_equal(x, res[0][4])
    assert sum(nl for _, _, nl, _, _ in res) == Pd["n"] + Pd["m"]
    xo, so = O.reg_cpkrylov("dqgmres", Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, perm=perm)
    assert res[0][3] == so["niters"]


@pytest.mark.gpu
@pytest.mark.parametrize("P", [2, 3])
def test_dist_minres_merged_exchanges(P):
    """cpminres's scalar exchanges ride in other collectives (alpha's partials in the first
    separator allgather, beta's in the next Lanczos vector's halo allgather, which the owners'
    normalisation is then applied to).  Each partial sum is then taken in rank order; the
    iteration must match the plain-allreduce path to rounding."""
    import cpkrylov_amd as cpk
    Pd = F.load("cvxqp1_m")
    opts = dict(F.EXPROG_OPTS)

    def run(options):
        def work(ctx, r):
            x, stats, flag = cpk.reg_cpkrylov(cpk.cpminres, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts,
                                              ctx=ctx)
            return x, stats["residHistory"], stats["niters"]
        return _run_ranks(P, work, options)[0]

    variants = {}
    for name, options in [("merged", {}), ("no_halo_merge", {"no_halo_merge": 1}), ("plain", {"no_piggy": 1})]:
        variants[name] = run(options)
    x0, h0, n0 = variants["plain"]
    for name in ("merged", "no_halo_merge"):
        x, h, n = variants[name]
        assert n == n0, name
        assert np.max(np.abs(h - h0)) <= 1e-10 * h0[0], name
        assert np.linalg.norm(x - x0) <= 1e-10 * np.linalg.norm(x0), name


@pytest.mark.gpu
@pytest.mark.parametrize("P", [2, 3])
def test_dist_minres_fused_update_bitexact(P):
    """Distributed cpminres with the update folded into the Lanczos step and the Krylov product
    (the halo the product reads is normalised by the owners' formula) equals the separate
    MinresUpdate pass bit for bit, with each exchange variant."""
    import cpkrylov_amd as cpk
    Pd = F.load("cvxqp1_m")
    opts = dict(F.EXPROG_OPTS)

    def work(ctx, r):
        x, stats, flag = cpk.reg_cpkrylov(cpk.cpminres, Pd["rhs"], Pd["Q"], Pd["B"], Pd["C"], Pd["G"], opts, ctx=ctx)
        return x, stats["residHistory"], stats["niters"]

    for variant in ({}, {"no_halo_merge": 1}, {"no_piggy": 1}):
        a = _run_ranks(P, work, dict(variant))[0]
        b = _run_ranks(P, work, dict(variant, no_minres_fuse=1))[0]
        assert a[2] == b[2] and np.array_equal(a[1], b[1]), variant
        assert np.array_equal(a[0], b[0]), (variant, np.max(np.abs(a[0] - b[0])))


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["tsolve_global", "tsolve_sweep", "tsolve_sweep,all_dataflow",
                                  "tsolve_sweep,no_dataflow", "tsolve_sweep,all_colsweep",
                                  "tsolve_sweep,all_colsweep,no_chain"])
@pytest.mark.parametrize("P", [2, 4])
def test_dist_apply_separator_fallbacks_bitexact(P, path):
    """The separator solve's other paths -- records left in HBM (a separator too large for LDS),
    and T solved by the block sweeps (the path of a T no workgroup holds; its upper rounds and
    the ranks' own on either level loop) -- give the same bits as the staged solve and the
    oracle."""
    import cpkrylov_amd as cpk
    S = _system("synthetic20k")
    z = np.random.default_rng(7).standard_normal(S["n"] + S["m"])

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        M.nitref, M.force_itref = 1, True
        return M * z, M.export_factors() if r == 0 else None

    res = _run_ranks(P, work, {k: 1 for k in path.split(",")})
    L, D, perm = res[0][1]
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    yo = Mo @ z
    for y, _ in res:
        assert np.array_equal(y, yo), np.max(np.abs(y - yo))


@pytest.mark.parametrize("P", [2, 4, 8])
def test_dist_apply_large_separator_bitexact(P):
    """A separator larger than one workgroup can hold: S10's generator at 1M dofs with SURVEY
    8d's +-64 coupling window and a tight split tolerance gives |T| = 10 000 rows (> 8192, the
    old one-workgroup cap, and more steps than the stepped solve's table), so T is solved by the
    block sweeps (dsep_sweep_setup).  Every rank's M*z -- plain, and with the forced refinement
    step in schedule order -- equals the oracle's bit for bit."""
    import cpkrylov_amd as cpk
    S = saddle_system(N=1_000_000, window=64, seed=21)
    z = np.random.default_rng(13).standard_normal(S["n"] + S["m"])

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        M.nitref = 0
        y0 = M * z
        M.nitref, M.force_itref = 1, True
        return y0, M * z, M.sep_info(), M.export_factors() if r == 0 else None

    res = _run_ranks(P, work, {"split_tol": "0.0005"})
    info = res[0][2]
    assert info["nT"] > 8192 and info["tsweep"] == 1 and info["sched"] == 1, info
    L, D, perm = res[0][3]
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(nitref=0.0)
    y0o = Mo @ z
    Mo.set(nitref=1.0, force_itref=1.0)
    yo = Mo @ z
    for y0, y, _, _ in res:
        assert np.array_equal(y0, y0o), np.max(np.abs(y0 - y0o))
        assert np.array_equal(y, yo), np.max(np.abs(y - yo))


def test_dist_apply_separator_records_overflow_lds():
    """A separator whose step records really exceed the 160 KB of LDS (a small split tolerance
    grows T): the stepped solve reads its records from HBM (lds == 0, lds_g > 0), and the
    apply still equals the oracle's bit for bit.  (The tsolve_global test above forces
    that path on a separator that would fit.)"""
    import cpkrylov_amd as cpk
    S = saddle_system(N=400000, seed=21)
    z = np.random.default_rng(8).standard_normal(S["n"] + S["m"])
    P = 4
    for tol in ("0.002", "0.0005", "0.0002", "0.0001"):
        def work(ctx, r):
            M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
            M.nitref, M.force_itref = 1, True
            return M * z, M.sep_info(), M.export_factors() if r == 0 else None

        res = _run_ranks(P, work, {"split_tol": tol})
        info = res[0][1]
        if info["lds"] == 0:
            break
    assert info["lds"] == 0 and info["lds_g"] > 0 and info["nrec"] > 0, info
    L, D, perm = res[0][2]
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    yo = Mo @ z
    for y, _, _ in res:
        assert np.array_equal(y, yo), np.max(np.abs(y - yo))


@pytest.mark.parametrize("P", [3, 4])
def test_dist_placement_hint_nonsym(P):
    """cpk_pc_create_hint: the Krylov operator's A places the isolated rows (the slack block of
    the nonsymmetric 3x3 system); M*z is still bit-exact and a cpdqgmres solve on the device
    vectors of that placement matches the oracle."""
    import cpkrylov_amd as cpk
    from cpkrylov_amd.synthetic import nonsym_system
    S = nonsym_system(N=30000, seed=4)
    z = np.random.default_rng(9).standard_normal(S["N"])
    opts = dict(F.EXPROG_OPTS, mem=20, itmax=60)

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx, krylov_A=S["Q"])
        M.nitref, M.force_itref = 1, True
        y = M * z
        x, yy, st = cpk.cpdqgmres(S["rhs"][:S["n"]], S["Q"], S["C"], M, opts)[:3]
        return y, M.export_factors() if r == 0 else None, x, yy, st

    res = _run_ranks(P, work)
    L, D, perm = res[0][1]
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    yo = Mo @ z
    for y, *_ in res:
        assert np.array_equal(y, yo)
    xo, yyo, so = O.method("dqgmres", S["rhs"][:S["n"]], S["Q"], S["C"], Mo, opts)
    _, _, x, yy, st = res[0]
    assert st["niters"] == so["niters"]
    h, ho = st["residHistory"], so["residHistory"]
    assert len(h) == len(ho) and np.max(np.abs(h - ho)) <= 1e-8 * ho[0]
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)


@pytest.mark.parametrize("option,value", [("sweep", "256,768,64"), ("split_tol", "0.06"), ("no_piggy", 1)])
def test_dist_plan_mismatch_fails_on_every_rank(option, value):
    """Every rank builds the global plan on its own, so ranks whose engine options differ would
    exchange mismatched payloads.  At setup the ranks allgather a hash of the plan and of every
    option: with one rank's option changed, every rank fails with the same clean error before
    any apply (no hang, no wrong answer)."""
    import cpkrylov_amd as cpk
    S = _system("synthetic20k")

    def work(ctx, r):
        try:
            cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        except cpk.CpkError as e:
            return str(e)
        return None

    res = _run_ranks(2, work, lambda r: {option: value} if r == 1 else {})
    assert all(m is not None and "plan of rank(s) 1 differs" in m for m in res), res
    # the same options on every rank: no error
    assert _run_ranks(2, work, {option: value}) == [None, None]


@pytest.mark.parametrize("P", [2, 4])
def test_dist_analysis_broadcast_bitexact(P):
    """The global analysis run once on rank 0 and broadcast (default) against every rank running
    it on its own (engine option no_bcast_analysis): the same factors and the same applies, bit
    for bit, and the oracle's; one rank alone asking for its own analysis takes every rank there
    (and the plan agreement then names it)."""
    import cpkrylov_amd as cpk
    S = _system("synthetic20k")
    z = np.random.default_rng(17).standard_normal(S["n"] + S["m"])

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        M.nitref, M.force_itref = 1, True
        return M * z, M.export_factors() if r == 0 else None

    res_b = _run_ranks(P, work)
    res_l = _run_ranks(P, work, {"no_bcast_analysis": 1})
    L, D, perm = res_b[0][1]
    L2, D2, perm2 = res_l[0][1]
    assert np.array_equal(perm, perm2) and np.array_equal(L.data, L2.data) and np.array_equal(D, D2)
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    yo = Mo @ z
    for (yb, _), (yl, _) in zip(res_b, res_l):
        assert np.array_equal(yb, yo) and np.array_equal(yl, yo)

    def work_err(ctx, r):
        try:
            cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        except cpk.CpkError as e:
            return str(e)
        return None

    res = _run_ranks(P, work_err, lambda r: {"no_bcast_analysis": 1} if r == 1 else {})
    assert all(m is not None and "plan of rank(s) 1 differs" in m for m in res), res


def test_dist_inputs_differ_fail_on_every_rank():
    """With the analysis broadcast from rank 0, a rank given other matrix values than rank 0's
    would build its plan on rank 0's analysis: every rank hashes its own inputs (pattern and value
    bits) into the plan agreement, so all of them fail with the same clean error."""
    import cpkrylov_amd as cpk
    S = _system("synthetic20k")

    def work(ctx, r):
        C = S["C"] * (2.0 if r == 1 else 1.0)
        try:
            cpk.opLDL2(S["G"], S["B"], -C, ctx=ctx)
        except cpk.CpkError as e:
            return str(e)
        return None

    res = _run_ranks(3, work)
    assert all(m is not None and "plan of rank(s) 1 differs" in m for m in res), res


def _new_values(S, seed):
    """IPM-like new values with the same sparsity: G rescaled, B and C scaled."""
    rng = np.random.default_rng(seed)
    G2 = S["G"].copy()
    G2.data = G2.data * rng.uniform(0.5, 2.0, G2.data.shape[0])
    B2 = S["B"].copy()
    B2.data = B2.data * rng.uniform(0.8, 1.25, B2.data.shape[0])
    C2 = S["C"].copy()
    C2.data = C2.data * 3.0
    return G2, B2, C2


@pytest.mark.parametrize("P", [2, 4, 8])
def test_dist_refactor_equals_fresh_single_gpu(P):
    """Distributed device factorization (opLDL2.m:81-82 rebuilt per IPM
    iteration, reg_cpkrylov.m:128-132): every rank factors the whole system on its GPU and takes
    its values through maps.  A refactorization with new G, B, C gives factors bit-identical to a
    fresh single-GPU construction on those values, and every rank's M*z equals the oracle's
    multiply with them; a cpminres solve after it matches the oracle."""
    import cpkrylov_amd as cpk
    S = _system("synthetic20k")
    G2, B2, C2 = _new_values(S, 17)
    z = np.random.default_rng(3).standard_normal(S["n"] + S["m"])
    opts = dict(F.EXPROG_OPTS)
    b = S["rhs"][:S["n"]]

    G3 = S["G"].copy()
    G3.data = G3.data * 1.7  # a second refactorization, to values the solve converges on

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        M.nitref, M.force_itref = 1, True
        y0 = M * z  # the caches built before the refactorization must not survive it
        x0 = cpk.cpminres(b, S["Q"], S["C"], M, dict(opts, itmax=5))[0]
        t = M.refactor(G2, B2, -C2)
        y = M * z
        f = M.export_factors() if r == 0 else None
        M.refactor(G3, S["B"], -S["C"])
        x, yy, st = cpk.cpminres(b, S["Q"], S["C"], M, opts)[:3]
        return y, f, x, st["niters"], st["residHistory"], t, y0, x0

    res = _run_ranks(P, work)
    ref = cpk.opLDL2(G2, B2, -C2)
    L, D, perm = ref.export_factors()
    Ld, Dd, permd = res[0][1]
    assert np.array_equal(perm, permd) and np.array_equal(L.indptr, Ld.indptr) and np.array_equal(L.indices, Ld.indices)
    assert np.array_equal(L.data, Ld.data) and np.array_equal(D, Dd)
    Mo = O.LDL2(G2, B2, -C2, factors=(L, D, perm))
    Mo.set(nitref=1.0, force_itref=1.0)
    yo = Mo @ z
    for y, *_ in res:
        assert np.array_equal(y, yo), np.max(np.abs(y - yo))
    M3 = cpk.opLDL2(G3, S["B"], -S["C"])
    Mo = O.LDL2(G3, S["B"], -S["C"], factors=M3.export_factors())
    Mo.set(nitref=1.0, force_itref=1.0)
    xo, yyo, so = O.method("minres", b, S["Q"], S["C"], Mo, opts)
    assert so["solved"]
    _, _, x, it, h, t, _, _ = res[0]
    assert t > 0 and it == so["niters"]
    assert len(h) == len(so["residHistory"]) and np.max(np.abs(h - so["residHistory"])) <= 1e-8 * so["residHistory"][0]
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)


def test_dist_refactor_failure_leaves_preconditioner_intact():
    """A zero pivot in a distributed refactorization fails on every rank and changes nothing:
    M*z afterwards equals M*z before it, bit for bit."""
    import cpkrylov_amd as cpk
    S = _system("synthetic20k")
    G0 = S["G"].copy()
    G0.data = G0.data * 0.0
    z = np.random.default_rng(4).standard_normal(S["n"] + S["m"])

    def work(ctx, r):
        M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
        M.nitref, M.force_itref = 1, True
        y0 = M * z
        try:
            M.refactor(G0, S["B"], -S["C"])
            err = None
        except cpk.CpkError as e:
            err = str(e)
        return y0, M * z, err

    for y0, y1, err in _run_ranks(2, work):
        assert err is not None and "pivot" in err
        assert np.array_equal(y0, y1)


@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("site", ["setup", "batch:1", "chain:1"])
def test_dist_rank_failure_reaches_every_rank(P, site):
    """A failure local to one rank of a distributed solve -- before the solve's first collective,
    a host error after a graph batch, or a sweep chain's timed-out wait (its device error word) --
    reaches every rank through the solve's status agreement (solvers.hip, agree_status): every
    rank returns the SAME error code promptly, none waits in a collective its peer never enters
    (kernels/cpminres.m:195-199: the caller sees error(...); SURVEY 8b's status codes).  The
    injected failure is engine option fail_inject (rank 1 only).  The contexts stay usable: the
    same solve without the hook then matches on every rank."""
    import time
    import cpkrylov_amd as cpk
    S = _system("synthetic20k")
    opts = dict(F.EXPROG_OPTS)

    def work(ctx, r):
        t0 = time.perf_counter()
        err = None
        try:
            cpk.reg_cpkrylov(cpk.cpminres, S["rhs"], S["Q"], S["B"], S["C"], S["G"], opts, ctx=ctx)
        except cpk.CpkError as e:
            err = (e.code, str(e))
        dt = time.perf_counter() - t0
        ctx.set_option("fail_inject", "")
        x, stats, flag = cpk.reg_cpkrylov(cpk.cpminres, S["rhs"], S["Q"], S["B"], S["C"], S["G"], opts, ctx=ctx)
        return err, dt, x, stats["niters"], flag["solved"]

    res = _run_ranks(P, work, {"fail_inject": f"1:{site}", "batch": 1})
    errs = [e for e, *_ in res]
    assert all(e is not None for e in errs), errs
    assert len({e[0] for e in errs}) == 1, errs
    assert "fail_inject" in errs[1][1] or "timed out" in errs[1][1], errs[1]
    for r, e in enumerate(errs):
        if r != 1:
            assert "rank 1 failed" in e[1], e
    assert max(dt for _, dt, *_ in res) < 60.0, [dt for _, dt, *_ in res]
    x0, it0, ok0 = res[0][2], res[0][3], res[0][4]
    assert ok0
    for _, _, x, it, ok in res[1:]:
        assert np.array_equal(x, x0) and it == it0 and ok == ok0
