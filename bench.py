#!/usr/bin/env python
"""Krylov iters/sec of CP-MINRES on the synthetic 10M-dof saddle-point system of SURVEY.md 8d.

Metric (BASELINE.json): "Krylov iters/sec + SpMV GB/s (% HBM peak), cpminres 10M-dof".
  system    SURVEY 8d's S10 generator with its +-64 B coupling window (nnz(L) 40.9 M, elimination
            tree 255 deep): the headline (round 6; rounds 1-5 quoted the +-4 window, now the `w4`
            block).  The `s50` block is config 5 (cpdqgmres(40) at 50 M dofs); both blocks are
            child runs of this script with their own timing, parity and CPU sample.
  step      one converging cpminres solve (the method call, kernels/cpminres.m) with the
            example options (cpk_exprog1.m:79-90: atol = rtol = 1e-6, itmax = 500, nitref = 1,
            force_itref, residual_update); b1 (the shifted rhs, reg_cpkrylov.m:152-160) and the
            solution are HBM-resident, the factorization (ptime) and the shift are outside the
            timed region.
  value     Krylov iterations completed by all ranks / max over ranks of the timed wall time.
  roofline  the dominant kernel, the triangular sweeps of one LDL' solve (a forward and a
            backward sweep, every round; an M*z runs two solves): algorithmic bytes / HIP-event-
            timed duration, vs 8 TB/s; spmv_roofline the same for the saddle-point SpMV
            r = x - Kp*y (the refinement residual inside every M*z).
  cpu_baseline  the C restatement (oracle/) of the same solve on the host, timed on a
            bounded sample of the same workload: one core, and OpenMP on the cores the box grants.
Multi-GPU (one process per GPU): ONE solve of the same S10 system row-block partitioned over
the ranks (strong scaling): RCCL allreduce for the inner products,
allgathered halos for the SpMVs and the separator exchange of the distributed LDL' sweeps.
value = that solve's iterations / max-over-ranks wall time.  `bench.py --gpus N` (N > 1) outside
torchrun starts `python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child
process before anything touches a GPU and exits with its return code; under torchrun,
WORLD_SIZE must equal --gpus, and the line's config.rccl_ranks is the communicator's own rank
count (ncclCommCount), so a run cannot silently measure fewer GPUs than it claims.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
EXPROG_OPTS = dict(print=False, atol=1.0e-6, rtol=1.0e-6, itmax=500,
                   residual_update=True, nitref=1, force_itref=True, itref_tol=1.0e-8)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the job; default WORLD_SIZE under torchrun, else 1")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the launch plan (the torchrun command for --gpus N > 1) as JSON and exit")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=("s10", "s50"), default="s10",
                    help="s10: symmetric 10M cpminres (the headline metric); s50: nonsymmetric 3x3-block "
                         "50M cpdqgmres(40) (SURVEY.md section 8d config 5)")
    ap.add_argument("--size", type=int, default=None, help="total dofs N (default 10M for s10, 50M for s50)")
    ap.add_argument("--window", type=int, default=64,
                    help="s10: the B coupling window (+-W columns; SURVEY.md 8d's 64 is the headline, 4 the w4 block)")
    ap.add_argument("--method", default=None)
    ap.add_argument("--itmax", type=int, default=None, help="s50: iterations per step (default 120)")
    ap.add_argument("--cpu-seconds", type=float, default=None,
                    help="budget of the CPU-baseline sample (default 40 s for the +-64 system, whose serial leg "
                         "must converge for the parity block; 20 s otherwise)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-reps", type=int, default=20)
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 FETCH_SIZE/WRITE_SIZE passes")
    ap.add_argument("--dist", action="store_true",
                    help="one GPU through a 1-rank RCCL communicator (a torchrun world of one: the single-GPU path)")
    ap.add_argument("--dist1", action="store_true",
                    help="with --dist: engine option dist1, the distributed kernels at one rank (diagnostic)")
    ap.add_argument("--pmc-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-exact", action="store_true",
                    help="skip the exact_dots block (the same solve with order-independent inner products, "
                         "timed, and compared bit for bit with the oracle's exact mode)")
    ap.add_argument("--no-sub", action="store_true",
                    help="skip the w4 and s50 blocks (child runs: the +-4 window system and config 5)")
    ap.add_argument("--no-w4", action="store_true", help="skip the w4 block")
    ap.add_argument("--no-s50", action="store_true", help="skip the s50 block")
    ap.add_argument("--rhs-perturb", type=float, default=0.0,
                    help="scale the rhs by (1 + eps*u), u uniform in [-1, 1] (sensitivity runs; never the bench line)")
    ap.add_argument("--perturb-seed", type=int, default=1)
    a = ap.parse_args(argv)
    s50 = a.config == "s50"
    if a.size is None:
        a.size = 50_000_000 if s50 else 10_000_000
    if a.method is None:
        a.method = "dqgmres" if s50 else "minres"
    if a.cpu_seconds is None:
        a.cpu_seconds = 40.0 if (not s50 and a.window >= 64) else 20.0
    a.opts = dict(EXPROG_OPTS)
    if s50:
        a.opts.update(mem=40, restart=40, itmax=a.itmax or 120)
    elif a.itmax:
        a.opts["itmax"] = a.itmax
    return a


class _quiet_stdout:
    """Send fd 1 to stderr while RCCL initialises (it prints a version banner on stdout; the
    bench's stdout is its one JSON line)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(args, argv):
    """What this invocation does before any GPU work: ("run", None) in-process, ("launch", cmd)
    to start torchrun with one rank per GPU, or ("error", message) for a world-size mismatch."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            return "error", f"--gpus {args.gpus} but WORLD_SIZE={world}: the job would measure {world} GPU(s)"
        return "run", None
    gpus = 1 if args.gpus is None else args.gpus
    if gpus < 1:
        return "error", f"--gpus {gpus}"
    if gpus == 1:
        return "run", None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
    return "launch", cmd + [a for a in argv if a != "--dry-run"]


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.pmc_probe:
        return pmc_probe(args)
    kind, what = launch_plan(args, argv)
    if args.dry_run:
        print(json.dumps({"plan": kind, "cmd" if kind == "launch" else "detail": what}), flush=True)
        return 2 if kind == "error" else 0
    if kind == "error":
        print(f"bench: {what}", file=sys.stderr, flush=True)
        return 2
    if kind == "launch":
        # a child process, not an exec: nothing in this process has touched a GPU; rank 0's JSON
        # line reaches our stdout through the inherited descriptor
        import subprocess
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        return subprocess.run(what, env=env).returncode
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        with _quiet_stdout():
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dist.barrier()
    import torch

    import cpkrylov_amd as cpk
    from cpkrylov_amd import _lib
    from cpkrylov_amd.synthetic import nonsym_system, saddle_system

    t_setup = time.perf_counter()
    S = nonsym_system(N=args.size) if args.config == "s50" else saddle_system(N=args.size, window=args.window)
    n, m, N = S["n"], S["m"], S["N"]
    # N > 1 (or --dist): one distributed solve over all ranks (strong scaling), RCCL collectives
    # and halo exchanges inside the solver; every rank holds its row block
    distributed = world > 1 or args.dist or args.dist1
    dev = torch.device("cuda", local)
    if distributed:
        # every rank must finish its setup before any rank enters a collective: a rank that fails
        # (e.g. out of memory) would otherwise leave the others waiting in RCCL.  No fallback to
        # replicas: a failed distributed setup ends the job with a non-zero exit on every rank.
        err = None
        try:
            uid = [cpk.get_unique_id() if rank == 0 else None]
            if dist:
                dist.broadcast_object_list(uid, src=0)
            with _quiet_stdout():
                ctx = cpk.Context(device=local, rank=rank, nranks=world, unique_id=uid[0],
                                  options={"dist1": 1} if args.dist1 else None)
            cinfo = ctx.info()
            if cinfo["comm"] != "rccl" or cinfo["comm_ranks"] != world:
                raise RuntimeError(f"the RCCL communicator holds {cinfo['comm_ranks']} rank(s), expected {world}")
            A, B, Cm, G = (cpk.Matrix(S[k], ctx) for k in ("Q", "B", "C", "G"))
            M = cpk.opLDL2(G, B, -S["C"], ctx=ctx, krylov_A=A)  # A: placement hint (cpk_pc_create_hint)
        except Exception as e:  # noqa: BLE001  (reported, then every rank exits)
            err = f"{type(e).__name__}: {e}"
        ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
        if dist:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            print(f"bench: distributed setup failed on rank {rank}: {err or 'another rank failed'}",
                  file=sys.stderr, flush=True)
            if dist:
                dist.destroy_process_group()
            sys.exit(3)
    else:
        ctx = cpk.Context(device=local)
        cinfo = ctx.info()
        A, B, Cm, G = (cpk.Matrix(S[k], ctx) for k in ("Q", "B", "C", "G"))
        M = cpk.opLDL2(G, B, -S["C"], ctx=ctx)
    M.nitref, M.itref_tol = EXPROG_OPTS["nitref"], EXPROG_OPTS["itref_tol"]
    M.residual_update, M.force_itref = EXPROG_OPTS["residual_update"], EXPROG_OPTS["force_itref"]
    dofs, n_loc = M.local_dofs()
    N_loc = len(dofs)
    rhs = S["rhs"]
    if args.rhs_perturb:
        u = np.random.default_rng(args.perturb_seed).uniform(-1.0, 1.0, rhs.shape[0])
        rhs = rhs * (1.0 + args.rhs_perturb * u)
    b = torch.from_numpy(np.ascontiguousarray(rhs[dofs])).to(dev)
    b1 = torch.empty(max(n_loc, 1), dtype=torch.float64, device=dev)
    xy0 = torch.empty(max(N_loc, 1), dtype=torch.float64, device=dev)
    xy = torch.empty(max(N_loc, 1), dtype=torch.float64, device=dev)
    torch.cuda.synchronize(dev)
    shifted = C.c_int()
    _lib.check(_lib.lib.cpk_reg_shift_device(ctx.h, C.c_void_p(b.data_ptr()), A.h, B.h, Cm.h, M.h,
                                             C.c_void_p(b1.data_ptr()), C.c_void_p(xy0.data_ptr()), C.byref(shifted)))
    opts = _lib.make_opts(args.opts)
    mid = _lib.METHODS[args.method]
    cap = int(args.opts["itmax"]) + 64
    hist = np.zeros(cap)
    st = _lib.Stats()
    st.hist = hist.ctypes.data_as(C.POINTER(C.c_double))
    st.hist_cap = cap

    def step():
        _lib.check(_lib.lib.cpk_method_solve_device(ctx.h, mid, C.c_void_p(b1.data_ptr()), A.h, Cm.h, M.h,
                                                    C.byref(opts), C.c_void_p(xy.data_ptr()), C.byref(st)))
        return int(st.niters)

    setup_s = time.perf_counter() - t_setup
    try:
        for _ in range(args.warmup):
            step()
        if dist:
            dist.barrier()
        ctx.synchronize()
        t0 = time.perf_counter()
        iters = 0
        loop_ms = 0.0
        for _ in range(args.steps):
            iters += step()
            loop_ms += st.loop_ms
        ctx.synchronize()
    except cpk.CpkError as e:
        # a distributed solve's status agreement makes every rank return the same error
        # (INTEGRATION.md section 5): every rank reports it and exits non-zero, none waits
        print(f"bench: solve failed on rank {rank}: {e}", file=sys.stderr, flush=True)
        sys.exit(4)
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    solved = bool(st.solved)
    niters_last = int(st.niters)
    hist_gpu = hist[:st.hist_len].copy()
    bytes_per_iter = st.bytes_moved / max(niters_last, 1)
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # one solve over all ranks: its iterations are the job's iterations (strong scaling)
    total_iters = float(iters)

    prof = _lib.Profile()
    _lib.check(_lib.lib.cpk_profile_kernels(ctx.h, A.h, Cm.h, M.h, args.profile_reps, C.byref(prof)))
    gbs = lambda byts, ms: byts / (ms * 1e-3) / 1e9  # noqa: E731
    # the dominant kernel: the triangular sweeps of one LDL' solve (forward + backward, every
    # round: sptrsv_pipe_kernel for round 0, sptrsv_upper_kernel above and sptrsv_last_kernel for
    # the last round's forward + backward), 2 per M*z
    sweep_ms, sweep_bytes = prof.fwd_ms + prof.bwd_ms, prof.fwd_bytes + prof.bwd_bytes
    achieved = gbs(sweep_bytes, sweep_ms)
    roofline = {"bound": "hbm", "kernel": "sptrsv_pipe_kernel (round 0) + sptrsv_upper_kernel / sptrsv_last_kernel "
                                          "(upper rounds): one LDL' solve (forward + backward sweep, all rounds)",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "bytes_per_launch": sweep_bytes,
                # y = LDL^-1 x with y the output: since r04 v13 round 0 no longer stores the dead
                # work vector, which the byte model dropped (8 B per round-0 row); the fraction on
                # the r03/r04-v12 model (the solve's bytes plus that store) keeps rounds comparable
                "frac_prev_model": round(gbs(sweep_bytes + prof.bwd_dead_store_bytes, sweep_ms) / HBM_PEAK_GBS, 4),
                "avg_ms": round(sweep_ms, 5), "launches": int(prof.fwd_launches) + int(prof.bwd_launches)}
    # the metric's "SpMV GB/s": the saddle-point SpMV inside every M*z (refinement residual)
    spmv_achieved = gbs(prof.resid_bytes, prof.resid_ms)
    spmv_roofline = {"kernel": "spmv_stream<EpiResidSched> (r = x - P'Kp P y, all in schedule order)",
                     "achieved": round(spmv_achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(spmv_achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "bytes_per_launch": prof.resid_bytes, "avg_ms": round(prof.resid_ms, 5)}
    kernels = {k: {"avg_ms": round(getattr(prof, k + "_ms"), 5), "bytes": getattr(prof, k + "_bytes"),
                   "GBps": round(gbs(getattr(prof, k + "_bytes"), getattr(prof, k + "_ms")), 1)}
               for k in ("spmv", "resid", "fwd", "bwd", "apply")}
    kernels["fwd"]["launches"], kernels["bwd"]["launches"] = int(prof.fwd_launches), int(prof.bwd_launches)
    if prof.fwd_resid_ms > 0:  # the refinement's residual + forward sweep, fused (launch_sptrsv_fwd_resid)
        kernels["fwd_resid"] = {"avg_ms": round(prof.fwd_resid_ms, 5), "bytes": prof.fwd_resid_bytes,
                                "GBps": round(gbs(prof.fwd_resid_bytes, prof.fwd_resid_ms), 1),
                                "replaces_ms": round(prof.resid_ms + prof.fwd_ms, 5)}

    passes = None
    if rank == 0 and world == 1 and not distributed and args.config == "s50":
        passes = s50_passes(ctx, step, M, N, n, m, args, prof, gbs)
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not distributed:
        if args.config == "s50":
            cpu = cpu_baseline_s50(S, b1.cpu().numpy(), M, args)
        else:
            cpu, parity = cpu_baseline(S, b1.cpu().numpy(), M, args, hist_gpu, niters_last)
    exact = None
    if rank == 0 and world == 1 and not distributed and not args.no_exact:
        exact = exact_block(ctx, S, M, step, st, hist, xy, b1, xy0, args, iters / dt)
    pmc = None
    if rank == 0 and world == 1 and not args.no_pmc and not distributed and args.config == "s10":
        pmc = pmc_traffic(args)
        if pmc and pmc.get("resid"):
            spmv_roofline["traffic"] = pmc["resid"]["bytes"]
        if pmc and pmc.get("fwd") and pmc.get("bwd"):
            roofline["traffic"] = pmc["fwd"]["bytes"] + pmc["bwd"]["bytes"]
        if pmc and pmc.get("fwd_resid") and "fwd_resid" in kernels:
            kernels["fwd_resid"]["traffic"] = pmc["fwd_resid"]["bytes"]

    ms_per_step = dt / args.steps * 1e3
    value = total_iters / dt
    if rank == 0:
        line = {
            "metric": ("Krylov iters/sec + SpMV GB/s (% HBM peak), cpminres 10M-dof, 1/2/4/8 GPU"
                       if args.config == "s10" else
                       "Krylov iters/sec, cpdqgmres(40) 50M-dof nonsymmetric 3x3-block"),
            "value": round(value, 2), "unit": "iters/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": (f"S10 synthetic symmetric saddle-point system, SURVEY 8d generator with B window "
                                    f"+-{args.window}{' (the headline system)' if args.window == 64 else ''}, "
                                    f"cp{args.method} to convergence (cpk_exprog1 options), step = one method call"
                                    if args.config == "s10" else
                                    f"S50 synthetic nonsymmetric 3x3-block saddle-point system, cp{args.method}"
                                    f"(mem 40), step = one method call TRUNCATED at {args.opts['itmax']} iterations "
                                    "(cpk_exprog1 tolerances; convergence takes 611-1039 iterations, rounding-"
                                    "dependent, DESIGN.md sec. 6), parity checked on the same truncated run"),
                       "N": N, "n": n, "m": m, "nnz_kp": M.info["nnz_kp"], "nnz_l": M.info["nnz_l"],
                       "sweep_launches": M.info["nrounds"], "elim_tree_depth": M.info["depth"],
                       "parallelism": f"rowblock{world}" if cinfo["distributed"] else "single",
                       "rccl_ranks": cinfo["comm_ranks"] if cinfo["comm"] == "rccl" else 0,
                       "sweep": ctx.get_option("sweep"),
                       "seed": S["seed"], "window": S["window"],
                       "rows_local_rank0": N_loc,
                       **({"rhs_perturb": args.rhs_perturb, "perturb_seed": args.perturb_seed}
                          if args.rhs_perturb else {})},
            "iters_per_step": round(float(iters) / args.steps, 2), "solved": solved,
            "roofline": roofline,
            "spmv_roofline": spmv_roofline,
            "roofline_iteration": {"bytes_per_iter_rank0": bytes_per_iter,
                                   "achieved": round(bytes_per_iter * total_iters / dt / 1e9, 1),
                                   "frac": round(bytes_per_iter * total_iters / dt / 1e9 / HBM_PEAK_GBS, 4)},
            "kernels": kernels,
            "device_loop_ms_per_step": round(loop_ms / args.steps, 3),
            "setup_s": round(setup_s, 2),
            "cpu_baseline": cpu,
            "pmc": pmc,
            "parity": parity,
            "exact_dots": exact,
        }
        if passes is not None:
            line["passes"] = passes
        if world == 1 and not distributed and args.config == "s10" and args.window == 64 and not args.no_sub:
            if not args.no_w4:
                line["w4"] = sub_block(args, ["--window", "4"], "the S10 system with the +-4 B window (rounds 1-5's headline)")
            if not args.no_s50:
                line["s50"] = sub_block(args, ["--config", "s50"], "config 5: S50, cpdqgmres(40), 120 iterations")
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def host_cpu():
    """Model name (lscpu / /proc/cpuinfo), logical CPUs of the machine (nproc --all) and of this
    process's affinity mask, and the thread budget the box grants (OMP_NUM_THREADS)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = max(1, min(aff or 1, int(omp) if omp and omp.isdigit() else (aff or 1)))
    limit = ("OMP_NUM_THREADS" if omp and omp.isdigit() and int(omp) < (aff or 1)
             else "affinity mask" if (aff or 0) < (os.cpu_count() or 0) else "none")
    return {"model": model, "nproc_all": os.cpu_count(), "affinity": aff, "omp_num_threads": omp,
            "threads": threads,
            "thread_limit": limit + (": the GPU box grants this process that many CPU threads (its CPU "
                                     "share of the shared host), so the OpenMP leg uses all of them"
                                     if limit != "none" else "")}


def cpu_baseline(S, b1, M_gpu, args, hist_gpu, niters_gpu):
    """The oracle's solve of the same system and shifted rhs on the host:
    one core (the serial restatement, MATLAB's sparse kernels being single-threaded) and OpenMP
    on the cores this process may use.  Both legs run the same pivot order as the GPU and the
    reference's work, including the dead residual-update SpMVs.  The serial leg, run to
    convergence, is also the parity reference of the GPU's histories; the OpenMP leg and two
    1e-15-perturbed rhs give the problem's own sensitivity band (tests/sensitivity.py)."""
    from oracle import oracle as O
    host = host_cpu()
    L, D, perm = M_gpu.export_factors()
    t = time.perf_counter()
    Mo = O.LDL2(S["G"], S["B"], -S["C"], perm=perm)  # the oracle's own factorization, same pivot order
    t_factor = time.perf_counter() - t
    Mo.set(nitref=args.opts["nitref"], itref_tol=args.opts["itref_tol"],
           force_itref=1.0, residual_update=1.0)

    def leg(threads, budget_s, opts_extra=None, rhs=None):
        got = O.set_threads(threads)
        try:
            rhs_ = b1 if rhs is None else rhs
            t = time.perf_counter()  # probe two iterations to size a bounded sample
            O.method(args.method, rhs_, S["Q"], S["C"], Mo, dict(args.opts, itmax=2))
            per_iter = (time.perf_counter() - t) / 3.0  # init M-apply + 2 iterations
            itmax = int(max(2, min(args.opts["itmax"], budget_s / max(per_iter, 1e-9))))
            if opts_extra is not None:
                itmax = int(args.opts["itmax"])
            t = time.perf_counter()
            x, y, st = O.method(args.method, rhs_, S["Q"], S["C"], Mo, dict(args.opts, itmax=itmax))
            return got, itmax, time.perf_counter() - t, x, st
        finally:
            O.set_threads(1)

    half = args.cpu_seconds / 2
    _, it1max, dt1, x1, st1 = leg(1, half)
    T, itTmax, dtT, xT, stT = leg(host["threads"], half)
    it1, itT = int(st1["niters"]), int(stT["niters"])
    cpu = {"value": round(it1 / dt1, 4), "unit": "iters/s", "cores": 1, "kind": "port",
           "sample": f"oracle cp{args.method} on {args.config.upper()} (same b1, same pivot order, dead "
                     f"residual-update SpMVs included), {it1} iterations (itmax {it1max}, solved "
                     f"{bool(st1['solved'])}) in {dt1:.1f} s, gcc -O3 -ffp-contract=off, one thread",
           "omp": {"value": round(itT / dtT, 4), "unit": "iters/s", "cores": T,
                   "sample": f"same solve, OpenMP on {T} threads (row-parallel SpMV and updates, "
                             f"level-scheduled sweeps), {itT} iterations (itmax {itTmax}) in {dtT:.1f} s"},
           "host": host, "oracle_factor_s": round(t_factor, 2)}
    parity = None
    if st1["solved"]:
        h = st1["residHistory"]
        h0 = h[0]
        dev = float(np.max(np.abs(h - hist_gpu[:len(h)])) / h0) if len(h) == len(hist_gpu) else None
        # sensitivity band: the OpenMP leg (different dot rounding) and four perturbed rhs; each
        # sample's own deviation is reported, so the GPU's can be read against their spread
        samples = []
        if stT["solved"] and len(stT["residHistory"]) == len(h):
            samples.append(float(np.max(np.abs(stT["residHistory"] - h)) / h0))
        rng = np.random.default_rng(12345)
        for _ in range(4):
            bp = b1 * (1 + 1e-15 * rng.standard_normal(b1.shape[0]))
            _, _, _, _, sp_ = leg(host["threads"], 0, opts_extra={}, rhs=bp)
            hp = sp_["residHistory"]
            L_ = min(len(hp), len(h))
            samples.append(float(np.max(np.abs(hp[:L_] - h[:L_])) / h0))
        band = max(samples) if samples else 0.0
        # one perturbed rhs on the serial leg (the reference's own order): what the perturbation
        # alone moves, against the order changes the samples above carry
        bp = b1 * (1 + 1e-15 * rng.standard_normal(b1.shape[0]))
        _, _, _, _, sp_ = leg(1, 0, opts_extra={}, rhs=bp)
        hp = sp_["residHistory"]
        L_ = min(len(hp), len(h))
        serial_pert = float(np.max(np.abs(hp[:L_] - h[:L_])) / h0)
        tol = max(1e-8, 10 * band)
        parity = {"niters_gpu": niters_gpu, "niters_oracle": it1, "niters_equal": niters_gpu == it1,
                  "max_hist_dev_over_h0": dev, "band_over_h0": band, "band_samples_over_h0": samples,
                  "serial_perturbed_over_h0": serial_pert,
                  "tolerance_over_h0": tol,
                  "pass": bool(niters_gpu == it1 and dev is not None and dev <= tol),
                  "method": "serial oracle run to convergence = reference; band = max history deviation of "
                            "the OpenMP leg and of four rhs perturbed by 1e-15 relative (each in "
                            "band_samples_over_h0, the OpenMP leg first); tolerance = max(1e-8, 10 x band) "
                            "(tests/test_gpu_parity.py)"}
    return cpu, parity


def exact_block(ctx, S, M, step, st, hist, xy, b1, xy0, args, value_default):
    """The same method call with engine option exact_dots (every inner product the correctly
    rounded exact sum of its TwoProd pairs, xacc.hpp): timed like the headline (its overhead is
    the ratio), and compared BIT FOR BIT with the oracle's exact mode run on the product's own
    factors -- niters, every history entry, x and y.  The oracle's OpenMP leg gives the serial
    restatement's bits in this mode (tests/test_gpu_exact.py), so it runs on the granted cores."""
    from oracle import oracle as O
    ctx.set_option("exact_dots", 1)
    try:
        step()  # warm-up: the exact solver's graphs
        ctx.synchronize()
        reps = max(1, min(args.steps, 5))
        t = time.perf_counter()
        it = 0
        for _ in range(reps):
            it += step()
        ctx.synchronize()
        dt = time.perf_counter() - t
        h_gpu = hist[:st.hist_len].copy()
        xy_gpu = xy.cpu().numpy()
        niters = int(st.niters)
    finally:
        ctx.set_option("exact_dots", 0)
    v = it / dt
    out = {"value": round(v, 2), "unit": "iters/s", "ms_per_step": round(dt / reps * 1e3, 3),
           "overhead_vs_default": round(value_default / v, 4) if v > 0 else None}
    golden = os.path.join(ROOT, "tests", "golden", f"{args.config}_exact_golden.npz")
    if args.config == "s50":
        # the serial oracle's 120 exact iterations at 50 M take ~20 minutes on 8 cores: the bench
        # compares with their record (tests/golden/make_exact_golden.py), made on the product's
        # host-analysis factors -- whose hashes the GPU's exported factors must match
        import hashlib
        if not os.path.exists(golden) or args.size != 50_000_000 or args.opts["itmax"] != 120:
            out["parity"] = None
            return out
        g = np.load(golden)
        L, D, perm = M.export_factors()
        sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()  # noqa: E731
        same_f = sha(np.asarray(perm, np.int32)) == bytes(g["perm_sha256"]) and sha(L.data) == bytes(g["L_sha256"]) \
            and sha(D) == bytes(g["D_sha256"])
        same_h = len(g["hist"]) == len(h_gpu) and bool(np.array_equal(g["hist"], h_gpu))
        # the record holds reg_cpkrylov's x: the shift's xy0 plus the method's [dx; dy]
        # (reg_cpkrylov.m:166-173, the same additions as the device's recovery)
        x_rec = xy0.cpu().numpy()[:int(g["N"])] + xy_gpu[:int(g["N"])]
        same_x = sha(np.ascontiguousarray(x_rec)) == bytes(g["x_sha256"])
        out["parity"] = {"niters_gpu": niters, "niters_oracle": int(g["niters"]), "factors_equal": bool(same_f),
                         "history_bitexact": same_h, "xy_bitexact": bool(same_x),
                         "pass": bool(niters == int(g["niters"]) and same_f and same_h and same_x),
                         "oracle": "the serial oracle's exact-mode record on the product's host-analysis factors "
                                   "(tests/golden/s50_exact_golden.npz: history, SHA-256 of x and of the factors)"}
        return out
    L, D, perm = M.export_factors()
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    # residual_update off: the value object's dead SpMVs subtract zeros, same bits
    Mo.set(nitref=args.opts["nitref"], itref_tol=args.opts["itref_tol"], force_itref=1.0, residual_update=0.0)
    threads = host_cpu()["threads"]
    O.set_threads(threads)
    try:
        t = time.perf_counter()
        with O.exact():
            x, y, so = O.method(args.method, b1.cpu().numpy(), S["Q"], S["C"], Mo, dict(args.opts, residual_update=False))
        t_or = time.perf_counter() - t
    finally:
        O.set_threads(1)
    ho = so["residHistory"]
    xyo = np.concatenate([x, y])
    same_h = len(ho) == len(h_gpu) and bool(np.array_equal(ho, h_gpu))
    same_x = bool(np.array_equal(xyo, xy_gpu[:len(xyo)]))
    out["parity"] = {"niters_gpu": niters, "niters_oracle": int(so["niters"]),
                     "history_bitexact": same_h, "xy_bitexact": same_x,
                     "pass": bool(niters == int(so["niters"]) and same_h and same_x),
                     "oracle": f"oracle cp{args.method} in exact mode (orc_set_exact) on the product's exported "
                               f"factors, OpenMP {threads} threads ({t_or:.1f} s): the serial restatement's bits"}
    return out


def sub_block(args, extra, what):
    """A secondary configuration measured by a child run of this script (its own setup, timing,
    CPU sample, parity, exact-mode and PMC blocks), embedded in the headline line."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--no-sub"] + extra
    for flag in ("no_pmc", "no_cpu_baseline", "no_exact"):
        if getattr(args, flag):
            cmd.append("--" + flag.replace("_", "-"))
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=420)
    except subprocess.TimeoutExpired:
        return {"error": "child timed out (420 s)", "what": what}
    if r.returncode != 0:
        return {"error": f"child exited {r.returncode}: {r.stderr[-400:]}", "what": what}
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    keep = ("metric", "value", "unit", "ms_per_step", "iters_per_step", "solved", "roofline", "spmv_roofline",
            "kernels", "cpu_baseline", "pmc", "parity", "exact_dots", "setup_s", "passes")
    out = {"what": what}
    out.update({k: d.get(k) for k in keep if k in d})
    out["config"] = d["config"]
    return out


def s50_passes(ctx, step, M, N, n, m, args, prof, gbs):
    """Config 5's per-pass rates: one more 120-iteration cpdqgmres(40) call with engine option
    profile_passes (eager batches, HIP events between the passes; cpk_debug_pass_times), each
    pass's algorithmic bytes summed over the iterations at their own window sizes nv (kernels/
    cpdqgmres.m:194-275; solvers.hip):
      window dots   arnoldi_dots_kernel: nv basis vectors, ut, w read, the new vector written,
                    the old one read for its y part: (nv + 3) 8N + 8m
      orthogonal.   ArnoldiOrth: nv basis vectors, the new vector read and written, ut:
                    (nv + 3) 8N
      direction     DqgmresDirection: nv' directions, v_k, the new vector read and written, the
                    new direction written, xy read and written: (nv' + 6) 8N
      M*z           Precond::apply_bytes per iteration; Krylov SpMV as cpk_profile_kernels."""
    from cpkrylov_amd import _lib
    ctx.set_option("profile_passes", 1)
    try:
        step()
        v = (C.c_double * 8)()
        _lib.check(_lib.lib.cpk_debug_pass_times(ctx.h, v))
    finally:
        ctx.set_option("profile_passes", 0)
    its, spmv_ms, apply_ms, dots_ms, orth_ms, dir_ms, wd, wr = list(v)
    if its <= 0:
        return None
    its_i = int(its)
    byts = {"krylov_spmv": prof.spmv_bytes * its, "mz": prof.apply_bytes * its,
            "dots": (wd + 3 * its) * 8.0 * N + 8.0 * m * its, "orth": (wd + 3 * its) * 8.0 * N,
            "direction": (wr + 6 * its) * 8.0 * N}
    ms = {"krylov_spmv": spmv_ms, "mz": apply_ms, "dots": dots_ms, "orth": orth_ms, "direction": dir_ms}
    out = {"iterations": its_i, "mean_window": round(wd / its, 2),
           "method": "one extra call with engine option profile_passes (eager, HIP events between passes); "
                     "bytes: the byte model in bench.py s50_passes at each iteration's window size"}
    for k in ms:
        a = gbs(byts[k], ms[k]) if ms[k] > 0 else 0.0
        out[k] = {"ms_per_iter": round(ms[k] / its, 4), "bytes_per_iter": round(byts[k] / its),
                  "GBps": round(a, 1), "frac": round(a / HBM_PEAK_GBS, 4)}
    out["iteration_ms_eager"] = round(sum(ms.values()) / its, 4)
    return out


def cpu_baseline_s50(S, b1, M_gpu, args):
    """Config 5's CPU sample: the oracle's cpdqgmres(40) on the same system and shifted rhs with
    the product's factors, OpenMP on the granted cores, a few iterations (the serial window
    loops take ~10 s per iteration at 50 M dofs)."""
    from oracle import oracle as O
    host = host_cpu()
    L, D, perm = M_gpu.export_factors()
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(nitref=args.opts["nitref"], itref_tol=args.opts["itref_tol"], force_itref=1.0, residual_update=1.0)
    T = O.set_threads(host["threads"])
    try:
        itmax = 3
        t = time.perf_counter()
        _, _, st = O.method(args.method, b1, S["Q"], S["C"], Mo, dict(args.opts, itmax=itmax))
        dt = time.perf_counter() - t
    finally:
        O.set_threads(1)
    it = int(st["niters"])
    return {"value": round(it / dt, 4), "unit": "iters/s", "cores": T, "kind": "port",
            "sample": f"oracle cp{args.method}(mem 40) on S50 (same b1, the product's factors), {it} iterations "
                      f"(the initial M*b included) in {dt:.1f} s, OpenMP on {T} threads, gcc -O3 -ffp-contract=off "
                      "(no serial leg: ~10 s per iteration)",
            "host": host}


PMC_REPS = 5


def pmc_probe(args):
    """Child program run under rocprofv3 --pmc: the kernel profile of S10 and nothing else.
    Launch order (solvers.hip profile_kernels): (1 + reps) Krylov SpMVs, (1 + reps) residual
    SpMVs, then the forward and backward sweeps, round by round."""
    import cpkrylov_amd as cpk
    from cpkrylov_amd import _lib
    from cpkrylov_amd.synthetic import nonsym_system, saddle_system
    S = nonsym_system(N=args.size) if args.config == "s50" else saddle_system(N=args.size, window=args.window)
    ctx = cpk.Context(device=0)
    A, Cm = cpk.Matrix(S["Q"], ctx), cpk.Matrix(S["C"], ctx)
    M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
    M.nitref, M.force_itref = EXPROG_OPTS["nitref"], EXPROG_OPTS["force_itref"]
    prof = _lib.Profile()
    _lib.check(_lib.lib.cpk_profile_kernels(ctx.h, A.h, Cm.h, M.h, PMC_REPS, C.byref(prof)))
    print(json.dumps({"resid_bytes": prof.resid_bytes, "spmv_bytes": prof.spmv_bytes,
                      "fwd_bytes": prof.fwd_bytes, "bwd_bytes": prof.bwd_bytes,
                      "fwd_resid_bytes": prof.fwd_resid_bytes,
                      "fwd_launches": int(prof.fwd_launches), "bwd_launches": int(prof.bwd_launches)}), flush=True)


def pmc_traffic(args):
    """HBM bytes per launch from rocprofv3 counters, one pass per counter (FETCH_SIZE and
    WRITE_SIZE do not fit one TCC pass).  Corrections per MI355X_MICROARCH.md (HBM section):
    counters are in KiB; FETCH_SIZE counts 128-B read requests at 64 B, so it is doubled.
    Returns None when rocprofv3 is unavailable or a pass fails (traffic is then reported null)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    out = {}
    reps = PMC_REPS
    with tempfile.TemporaryDirectory(prefix="cpk_pmc_") as tmp:
        counts = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-probe", "--size", str(args.size),
                   "--window", str(args.window)]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            except subprocess.TimeoutExpired:
                return None
            if r.returncode != 0:
                return {"error": f"rocprofv3 {ctr} pass exited {r.returncode}"}
            probe = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
            files = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
            if not files:
                return {"error": f"no counter file from the {ctr} pass"}
            rows = sorted(csv.DictReader(open(files[0])), key=lambda q: int(q["Dispatch_Id"]))
            counts[ctr] = rows
        kib = 1024.0

        def per_call(name_pred, sel, calls):
            """bytes per call: the selected launches' counters summed, divided by the calls"""
            f = [float(q["Counter_Value"]) for q in counts["FETCH_SIZE"] if name_pred(q["Kernel_Name"])]
            w = [float(q["Counter_Value"]) for q in counts["WRITE_SIZE"] if name_pred(q["Kernel_Name"])]
            f, w = sel(f), sel(w)
            if not f or len(f) != len(w):
                return None
            fb, wb = 2.0 * kib * sum(f) / calls, kib * sum(w) / calls
            return {"fetch": round(fb), "write": round(wb), "bytes": round(fb + wb), "launches": len(f) // calls}

        spmv = lambda nm: nm.split("<")[0].split("(")[0].strip().endswith("spmv_stream")  # noqa: E731
        # launch order of cpk_profile_kernels: (1 + reps) Krylov SpMVs, (1 + reps) residual SpMVs
        out["resid"] = per_call(spmv, lambda v: v[reps + 2:2 * reps + 2], reps)
        out["spmv"] = per_call(spmv, lambda v: v[1:reps + 1], reps)
        # sweeps (round-0 pipe, upper-round and fused last-round kernels): (1 + reps) forward
        # sweeps of Lf launches, then (1 + reps) pairs of Lf + Lb launches (the forward again,
        # then the backward, whose Lb launches include the fused last round when there is one)
        Lf, Lb = probe["fwd_launches"], probe["bwd_launches"]
        sweep = lambda nm: "sptrsv" in nm  # noqa: E731
        out["fwd"] = per_call(sweep, lambda v: v[Lf:Lf * (reps + 1)], reps)
        p0 = Lf * (reps + 1) + (Lf + Lb)  # the pairs after the warm-up pair

        def bwd_of_pairs(v):
            return [x for i in range(reps) for x in v[p0 + i * (Lf + Lb) + Lf:p0 + (i + 1) * (Lf + Lb)]]
        out["bwd"] = per_call(sweep, bwd_of_pairs, reps)
        if probe.get("fwd_resid_bytes", 0) > 0:
            # the fused residual + forward sweep (all rounds, nothing deferred): the last reps calls
            R = Lb
            out["fwd_resid"] = per_call(sweep, lambda v: v[len(v) - R * reps:], reps)
        for k in ("resid", "spmv", "fwd", "bwd", "fwd_resid"):
            if out.get(k):
                out[k]["algorithmic"] = probe[k + "_bytes"]
                out[k]["ratio"] = round(out[k]["bytes"] / probe[k + "_bytes"], 3)
        out["method"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over the S10 kernel "
                         "profile; FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B), KiB -> bytes")
    return out


if __name__ == "__main__":
    sys.exit(main() or 0)
