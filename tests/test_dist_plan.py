"""Row-block distributed plan, host side, no GPU.

The plans the library builds for P ranks are replayed in numpy (tests/dist_emul.py) and must
reproduce the single-process results bit for bit:
  * the distributed M*z (local sweeps + separator allgather + redundant separator solve)
    equals the oracle's opLDL2 apply with the exported factor;
  * the distributed SpMVs of Kp, blkdiag(A, C) and [A B'] with their halo buffers equal the
    global row sums in the same column order;
  * ownership is a partition of the dofs and the local [x; y] layout keeps the split.
The world_size-2 test runs the same exchange through torch.distributed (gloo) between two
processes."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import cpkrylov_amd as cpk
import fixtures as F
from cpkrylov_amd.synthetic import saddle_system
from dist_emul import RankApply, dist_spmv, halo_payload, seq_rowsum
from oracle import oracle as O


def _systems():
    out = []
    for name in ("cvxqp1_m", "cvxqp2_s"):
        P = F.load(name)
        out.append((name, P["Q"], P["B"], P["C"], P["G"]))
    S = saddle_system(N=6000, seed=7)
    out.append(("synthetic6k", S["Q"], S["B"], S["C"], S["G"]))
    return out


SYSTEMS = _systems()


def _plans(Q, B, Cm, G, P):
    return [cpk.dist_plan(G, B, -Cm, Q, Cm, P, r) for r in range(P)]


def _global_rowsum(K, x):
    K = sp.csr_matrix(K)
    K.sort_indices()
    return seq_rowsum(K.indptr, K.data * x[K.indices])


def _apply_all(plans, xs, negs):
    ra = [RankApply(p) for p in plans]
    ph = [r.phase1(x, nf) for r, x, nf in zip(ra, xs, negs)]
    recv = np.concatenate([pay for _, pay in ph])  # the allgather
    return [r.phase2(w, recv) for r, (w, _) in zip(ra, ph)]


@pytest.mark.parametrize("P", [2, 3, 4])
@pytest.mark.parametrize("name,Q,B,Cm,G", SYSTEMS, ids=[s[0] for s in SYSTEMS])
def test_distributed_apply_bitexact(name, Q, B, Cm, G, P):
    plans = _plans(Q, B, Cm, G, P)
    n, N = plans[0]["n"], plans[0]["N"]
    # ownership: a partition of the dofs, x-part first in every local vector
    allg = np.concatenate([p["dofs"] for p in plans])
    assert np.array_equal(np.sort(allg), np.arange(N))
    for p in plans:
        assert np.all(p["dofs"][:p["n_loc"]] < n) and np.all(p["dofs"][p["n_loc"]:] >= n)
    an = cpk.analyze(G, B, -Cm)
    Mo = O.LDL2(G, B, -Cm, factors=(an["L"], an["D"], an["perm"]))
    Mo.set(nitref=0)
    x = np.random.default_rng(P).standard_normal(N)
    for negate in (False, True):
        xs = [x[p["dofs"]] for p in plans]
        negs = [p["n_loc"] if negate else p["N_loc"] for p in plans]
        ys = _apply_all(plans, xs, negs)
        y = np.empty(N)
        for p, yl in zip(plans, ys):
            y[p["dofs"]] = yl
        xin = np.concatenate([x[:n], -x[n:]]) if negate else x
        assert np.array_equal(y, Mo @ xin), f"{name} P={P} negate={negate}"


@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("name,Q,B,Cm,G", SYSTEMS, ids=[s[0] for s in SYSTEMS])
def test_distributed_spmv_bitexact(name, Q, B, Cm, G, P):
    plans = _plans(Q, B, Cm, G, P)
    n, N = plans[0]["n"], plans[0]["N"]
    Kp = sp.bmat([[G, B.T], [B, -Cm]]).tocsr()
    AC = sp.block_diag([Q, Cm]).tocsr()
    AB = sp.hstack([Q, B.T]).tocsr()
    x = np.random.default_rng(11).standard_normal(N)
    for kind, K, rows in (("kp", Kp, N), ("ac", AC, N), ("ab", AB, n)):
        ref = _global_rowsum(K, x)
        xs = [x[p["dofs"]] for p in plans]
        recv = np.concatenate([halo_payload(p, kind, xl) for p, xl in zip(plans, xs)])
        got = np.empty(rows)
        for p, xl in zip(plans, xs):
            yl = dist_spmv(p, kind, xl, recv)
            got[p["dofs"][:len(yl)]] = yl
        assert np.array_equal(got, ref), kind


def test_plan_balance_s200k():
    """At 200k dofs with 8 ranks the subtrees balance and the separator set stays small."""
    S = saddle_system(N=200000)
    plans = [cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], 8, r) for r in (0, 7)]
    p0 = plans[0]
    assert p0["nT"] <= 2000
    nsub = [cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], 8, r)["nsub"] for r in range(1, 7)]
    nsub += [p["nsub"] for p in plans]
    assert max(nsub) <= 1.25 * (sum(nsub) / len(nsub))
    for kind in ("kp", "ac", "ab"):
        assert p0[kind + "_kmax"] <= 2000  # halos stay small on the banded system


def _gloo_worker(rank, world, port, name, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        P_ = F.load(name)
        pl = cpk.dist_plan(P_["G"], P_["B"], -P_["C"], P_["Q"], P_["C"], world, rank)
        N = pl["N"]
        x = np.random.default_rng(3).standard_normal(N)
        xl = x[pl["dofs"]]
        ra = RankApply(pl)
        w, pay = ra.phase1(xl, pl["N_loc"])
        bufs = [torch.zeros(pl["kt"], dtype=torch.float64) for _ in range(world)]
        dist.all_gather(bufs, torch.from_numpy(pay))
        y = ra.phase2(w, torch.cat(bufs).numpy())
        # Kp halo exchange + local residual rows
        hp = [torch.zeros(pl["kp_kmax"], dtype=torch.float64) for _ in range(world)]
        dist.all_gather(hp, torch.from_numpy(halo_payload(pl, "kp", y)))
        r = xl - dist_spmv(pl, "kp", y, torch.cat(hp).numpy())
        # gather the global vectors on every rank
        ng = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(ng, torch.tensor([pl["N_loc"]]))
        mx = int(max(t.item() for t in ng))
        def gather(v):
            outs = [torch.zeros(mx, dtype=torch.float64) for _ in range(world)]
            pad = torch.zeros(mx, dtype=torch.float64)
            pad[:len(v)] = torch.from_numpy(v)
            dist.all_gather(outs, pad)
            return outs
        ys, rs = gather(y), gather(r)
        ds = gather(pl["dofs"].astype(np.float64))
        if rank == 0:
            yg, rg = np.empty(N), np.empty(N)
            for k in range(world):
                nl = int(ng[k].item())
                d = ds[k][:nl].numpy().astype(np.int64)
                yg[d], rg[d] = ys[k][:nl].numpy(), rs[k][:nl].numpy()
            q.put((yg, rg))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_apply_and_residual():
    import socket
    import torch.multiprocessing as mp
    name = "cvxqp1_m"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    yg, rg = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    P_ = F.load(name)
    an = cpk.analyze(P_["G"], P_["B"], -P_["C"])
    Mo = O.LDL2(P_["G"], P_["B"], -P_["C"], factors=(an["L"], an["D"], an["perm"]))
    Mo.set(nitref=0)
    x = np.random.default_rng(3).standard_normal(len(yg))
    assert np.array_equal(yg, Mo @ x)
    Kp = sp.bmat([[P_["G"], P_["B"].T], [P_["B"], -P_["C"]]]).tocsr()
    assert np.array_equal(rg, x - _global_rowsum(Kp, yg))


def test_plan_balances_rows_with_isolated_stretches():
    """S50's slack blocks (dofs no constraint touches: isolated rows of the factor) are long
    contiguous stretches; the plan deals them out so every rank holds ~N/P rows (the Krylov
    vectors and SpMV rows), instead of all of them following one neighbouring dof."""
    from cpkrylov_amd.synthetic import nonsym_system
    S = nonsym_system(N=200000, seed=11)
    P = 8
    plans = [cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], P, r) for r in range(P)]
    rows = [int(p["sizes"][7]) for p in plans]
    assert sum(rows) <= S["N"] and max(rows) <= 1.05 * S["N"] / P, rows
    # with the Krylov operator as placement hint (the plan gets A), each slack row sits with
    # the bounded variable A couples it with: the Krylov SpMV's halo stays a small fraction
    ac_kmax = max(int(p["sizes"][12]) for p in plans)
    assert ac_kmax <= 0.2 * S["N"] / P, (ac_kmax, rows)
