"""Host half of the preconditioner (no GPU): ordering, static-pivot LDL', sweep schedule.

The device sweeps are replayed here in numpy following the schedule exactly (rounds, blocks,
intra-block levels, MATLAB's accumulation order); the replay must (a) never read an
unfinished value and (b) equal the oracle's column-oriented solve with the same factors bit
for bit -- the contract the HIP kernels implement."""
import numpy as np
import pytest
import scipy.sparse as sp

import cpkrylov_amd as cpk
import fixtures as F
from cpkrylov_amd.synthetic import saddle_system
from oracle import oracle as O


def _systems():
    out = []
    for name in ("cvxqp1_m", "cvxqp2_s"):
        P = F.load(name)
        out.append((name, P["G"], P["B"], -P["C"]))
    S = saddle_system(N=20000)
    out.append(("synthetic20k", S["G"], S["B"], -S["C"]))
    return out


SYSTEMS = _systems()


def replay(an, x):
    """Schedule position q solves exported-factor row order[q]; each row sums its entries in the
    exported factor's order (forward: ascending column, backward: descending row)."""
    L, D, perm, order = an["L"], an["D"], an["perm"], an["order"]
    rp, bl, lr = an["round_ptr"], an["blk_lvl"], an["lvl_row"]
    N = len(D)
    Lr = L.tocsr()
    Lr.sort_indices()
    Lc = L.tocsc()
    Lc.sort_indices()
    w = np.full(N, np.nan)
    assert lr[0] == 0  # every row is in a block
    for r in range(len(rp) - 1):
        for b in range(rp[r], rp[r + 1]):
            for lv in range(bl[b], bl[b + 1]):
                for q in range(lr[lv], lr[lv + 1]):
                    k = order[q]
                    acc = x[perm[k]]
                    for e in range(Lr.indptr[k], Lr.indptr[k + 1]):
                        assert not np.isnan(w[Lr.indices[e]]), "forward dependency not ready"
                        acc -= Lr.data[e] * w[Lr.indices[e]]
                    w[k] = acc
    done = np.zeros(N, bool)
    y = np.zeros(N)
    for r in range(len(rp) - 2, -1, -1):
        for b in range(rp[r], rp[r + 1]):
            for lv in range(bl[b + 1] - 1, bl[b] - 1, -1):
                for q in range(lr[lv], lr[lv + 1]):
                    k = order[q]
                    acc = w[k] / D[k]
                    for e in range(Lc.indptr[k + 1] - 1, Lc.indptr[k] - 1, -1):
                        assert done[Lc.indices[e]], "backward dependency not ready"
                        acc -= Lc.data[e] * w[Lc.indices[e]]
                    w[k] = acc
                    done[k] = True
                    y[perm[k]] = acc
    return y


@pytest.mark.parametrize("name,G,B,C22", SYSTEMS, ids=[s[0] for s in SYSTEMS])
def test_factor_and_schedule(name, G, B, C22):
    an = cpk.analyze(G, B, C22)
    N = an["info"]["N"]
    perm = an["perm"]
    assert np.array_equal(np.sort(perm), np.arange(N))  # P is a permutation (P*P' = I)
    Kp = sp.bmat([[G, B.T], [B, C22]]).tocsr()
    L1 = an["L"] + sp.eye(N)
    R = Kp[perm][:, perm] - L1 @ sp.diags(an["D"]) @ L1.T
    scale = abs(L1) @ sp.diags(np.abs(an["D"])) @ abs(L1).T  # componentwise backward error
    assert abs(R).max() <= 1e-14 * max(abs(scale).max(), abs(Kp).max())
    # schedule covers every row once, rounds/blocks/levels consistent
    assert an["lvl_row"][0] >= 0 and an["lvl_row"][-1] == N
    assert np.all(np.diff(an["lvl_row"]) > 0)
    assert an["blk_lvl"][-1] == len(an["lvl_row"]) - 1
    x = np.random.default_rng(5).standard_normal(N)
    y = replay(an, x)
    Mo = O.LDL2(G, B, C22, factors=(an["L"], an["D"], perm))
    Mo.set(nitref=0)
    assert np.array_equal(y, Mo @ x)
    assert np.linalg.norm(Kp @ y - x) <= 1e-6 * np.linalg.norm(x)


def test_synthetic_s10_shape_of_schedule():
    """At 200k dofs the nested-dissection schedule needs only a few launches per sweep."""
    S = saddle_system(N=200000)
    an = cpk.analyze(S["G"], S["B"], -S["C"])
    assert an["info"]["ordering"] == 1  # G-first + nested dissection
    assert an["info"]["nrounds"] <= 4
    assert an["info"]["nnz_l"] <= an["info"]["nnz_kp"]


def test_dimension_errors():
    P = F.load("cvxqp2_s")
    with pytest.raises(cpk.CpkError) as e:
        cpk.analyze(P["G"], P["B"][:, :10], -P["C"])
    assert "Incompatible dimensions" in str(e.value)
    with pytest.raises(cpk.CpkError) as e:
        cpk.analyze(P["G"][:, :10], P["B"], -P["C"])
    assert "must be square" in str(e.value)


def test_zero_pivot_reported():
    P = F.load("cvxqp2_s")
    G0 = sp.csr_matrix(P["G"].shape)
    with pytest.raises(cpk.CpkError) as e:
        cpk.analyze(G0, P["B"], -P["C"])
    assert e.value.code == 6


def test_csc_boundary_matches_csr():
    """cpk_mat_create_csc -- MATLAB's own sparse storage (0-based size_t jc / ir, the MEX
    gateway's entry, matlab/cpk_mex.c) -- yields the same analysis as the CSR entry: identical
    ordering, factor, D and schedule."""
    P = F.load("cvxqp1_m")
    mats_csc = [cpk.Matrix(M, host_only=True, csc=True) for M in (P["G"], P["B"], -P["C"])]
    a = cpk.analyze(*mats_csc)
    b = cpk.analyze(P["G"], P["B"], -P["C"])
    for k in ("D", "perm", "round_ptr", "blk_lvl", "lvl_row", "order"):
        assert np.array_equal(a[k], b[k]), k
    assert (a["L"] != b["L"]).nnz == 0
    assert a["info"] == b["info"]


def test_engine_option_from_env_validated(monkeypatch):
    """Engine options start from CPK_<NAME> (read when a context or a host-only analysis is
    made); a malformed value is an error, not a silent default, and a valid sweep option changes
    the schedule."""
    S = saddle_system(N=20000, seed=3)
    for bad in ("abc", "0,0,64", "192,576,48", "100000,576,64"):
        monkeypatch.setenv("CPK_SWEEP", bad)
        with pytest.raises(cpk.CpkError):
            cpk.analyze(S["G"], S["B"], -S["C"])
    monkeypatch.setenv("CPK_SWEEP", "64,128,64")
    small = cpk.analyze(S["G"], S["B"], -S["C"])["info"]
    monkeypatch.delenv("CPK_SWEEP")
    monkeypatch.setenv("CPK_NO_PIPE", "maybe")
    with pytest.raises(cpk.CpkError):
        cpk.analyze(S["G"], S["B"], -S["C"])
    monkeypatch.delenv("CPK_NO_PIPE")
    default = cpk.analyze(S["G"], S["B"], -S["C"])["info"]
    assert small["nblocks"] > default["nblocks"]


@pytest.mark.parametrize("name", ["r0_xcd_chunk", "batch"])
def test_integer_engine_options_validated(monkeypatch, name):
    """Integer engine options (round-0 XCD run length, fixed graph batch) accept 0..4096 and
    reject anything else, whether from CPK_<NAME> or not an integer at all."""
    S = saddle_system(N=20000, seed=3)
    env = "CPK_" + name.upper()
    for bad in ("abc", "-1", "4097", "16x", "1.5"):
        monkeypatch.setenv(env, bad)
        with pytest.raises(cpk.CpkError):
            cpk.analyze(S["G"], S["B"], -S["C"])
    for good in ("0", "3", "4096"):
        monkeypatch.setenv(env, good)
        cpk.analyze(S["G"], S["B"], -S["C"])
    monkeypatch.delenv(env)


def test_split_tol_option_validated(monkeypatch):
    """CPK_SPLIT_TOL (a diagnostic of the distributed plan) must be a finite number in (0, 1):
    every rank builds the same plan from it, so a malformed value is an error, not a default."""
    S = saddle_system(N=20000, seed=3)
    for bad in ("abc", "0", "1.5", "nan", "-0.1", "0.03x"):
        monkeypatch.setenv("CPK_SPLIT_TOL", bad)
        with pytest.raises(cpk.CpkError):
            cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], 2, 0)
    monkeypatch.setenv("CPK_SPLIT_TOL", "0.06")
    p6 = cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], 2, 0)
    monkeypatch.delenv("CPK_SPLIT_TOL")
    p3 = cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], 2, 0)
    assert p6["nT"] <= p3["nT"]
    # the same option handed over explicitly (as a context's cpk_ctx_get_options string or a
    # dict): the analysis and the plan follow it, not the environment
    q6 = cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], 2, 0, options={"split_tol": 0.06})
    q6s = cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], 2, 0, options="split_tol=0.06;")
    for k in ("T", "dofs", "node_rank"):
        assert np.array_equal(q6[k], p6[k]) and np.array_equal(q6s[k], p6[k]), k
    with pytest.raises(cpk.CpkError):
        cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], 2, 0, options="split_tol")
    small = cpk.analyze(S["G"], S["B"], -S["C"], options={"sweep": "64,128,64"})["info"]
    assert small["nblocks"] > cpk.analyze(S["G"], S["B"], -S["C"])["info"]["nblocks"]


@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s"])
def test_host_factor_vs_oracle_factor(name):
    """The product's host factorization (rows' reach in ascending order, the order the device
    numeric phase uses) against the oracle's (Davis's stack order), same pivot order: equal
    structure, values within rounding; and P'*Kp*P = L*D*L' to rounding in scipy."""
    import scipy.sparse as sp

    from oracle import oracle as O
    P = F.load(name)
    H = cpk.analyze(P["G"], P["B"], -P["C"])
    Mo = O.LDL2(P["G"], P["B"], -P["C"], perm=H["perm"])
    Lo, Do, permo = Mo.factors()
    L, D = H["L"], H["D"]
    assert np.array_equal(permo, H["perm"])
    assert np.array_equal(Lo.indptr, L.indptr) and np.array_equal(Lo.indices, L.indices)
    assert np.max(np.abs(L.data - Lo.data)) <= 1e-10 * max(1.0, np.max(np.abs(L.data)))
    assert np.max(np.abs(D - Do) / np.abs(Do)) <= 1e-10
    K = sp.bmat([[P["G"], P["B"].T], [P["B"], -P["C"]]]).tocsr()[H["perm"]][:, H["perm"]]
    Lu = L + sp.identity(K.shape[0], format="csc")
    R = K - Lu @ sp.diags(D) @ Lu.T
    assert abs(R).max() <= 1e-12 * abs(K).max() * max(1.0, abs(Lu).max() ** 2)
