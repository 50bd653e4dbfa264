"""Per-rank work of a P-way distributed S10 solve, timed on ONE GPU (diagnostic).

Context(timing_standin=True) (cpk_ctx_create_null) gives the context a communicator without
peers: collectives are no-ops, so the numbers are meaningless but the kernels are exactly one
rank's share of the P-way solve.
Prints, per (P, rank): the local rows, the construction time of the rank's preconditioner
(ptime, and a refactorization with the same values), kernel timings (cpk_profile_kernels), the
wall time per iteration of an ITMAX-iteration solve (collective latency NOT included), the process's
peak host RSS and the device memory the rank's objects hold.
CONFIG=s10 (default): S10, cpminres.  CONFIG=s50: S50 (nonsymmetric 3x3 block, 50M dofs),
cpdqgmres(40), with the Krylov A as the placement hint -- SURVEY.md section 8d config 5.
"""
import ctypes as C
import json
import os
import resource
import sys
import time

import numpy as np
import torch  # before libcpk initialises HIP

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd import _lib  # noqa: E402
from cpkrylov_amd.synthetic import nonsym_system, saddle_system  # noqa: E402

torch.cuda.init()
CONFIG = os.environ.get("CONFIG", "s10")
if CONFIG == "s50":
    S = nonsym_system(int(os.environ.get("N", "50000000")))
    METHOD, MOPTS = 5, dict(mem=40, restart=40)
    # the bench line's truncated run: the 40-vector window fills over the first 40 iterations
    ITMAX = int(os.environ.get("ITMAX", "120"))
else:
    ITMAX = int(os.environ.get("ITMAX", "20"))
    S = saddle_system(int(os.environ.get("N", "10000000")), window=int(os.environ.get("WINDOW", "4")))
    METHOD, MOPTS = 2, {}
runs = [(int(a.split(":")[0]), int(a.split(":")[1])) for a in sys.argv[1:]] or [(1, 0), (2, 0), (4, 0), (8, 0), (8, 7)]
# CPK_SWEEPS="cfg1;cfg2": repeat every run under each CPK_SWEEP staging configuration
sweeps = [x for x in os.environ.get("CPK_SWEEPS", "").split(";") if x] or [os.environ.get("CPK_SWEEP", "")]
runs = [(P, r, sw) for sw in sweeps for P, r in runs]
for P, r, sw in runs:
    if sw:
        os.environ["CPK_SWEEP"] = sw
    free0 = torch.cuda.mem_get_info(0)[0]
    ctx = cpk.Context(device=0, rank=r, nranks=P, timing_standin=True) if P > 1 else cpk.Context(device=0)
    A, B, Cm, G = (cpk.Matrix(S[k], ctx) for k in ("Q", "B", "C", "G"))
    t0 = time.perf_counter()
    M = cpk.opLDL2(G, B, -S["C"], ctx=ctx, krylov_A=A)
    construct_s, ptime_s = time.perf_counter() - t0, M.ptime
    refactor_s = M.refactor(S["G"], S["B"], -S["C"])
    M.nitref, M.force_itref = 1, True
    dofs, n_loc = M.local_dofs()
    p = _lib.Profile()
    _lib.check(_lib.lib.cpk_profile_kernels(ctx.h, A.h, Cm.h, M.h, 20, C.byref(p)))
    # a fixed ITMAX-iteration solve (tolerance 0): wall time per iteration of the rank's kernels
    dev = torch.device("cuda", 0)
    b1 = torch.from_numpy(np.ascontiguousarray(S["rhs"][dofs[:n_loc]])).to(dev)
    xy = torch.empty(max(len(dofs), 1), dtype=torch.float64, device=dev)
    opts = _lib.make_opts(dict(atol=0.0, rtol=0.0, itmax=ITMAX, print=False, nitref=1, force_itref=True, **MOPTS))
    st = _lib.Stats()
    hist = np.zeros(ITMAX + 64)
    st.hist = hist.ctypes.data_as(C.POINTER(C.c_double))
    st.hist_cap = ITMAX + 64
    per_it = None
    err = None
    try:
        for rep in range(3):
            ctx.synchronize()
            t = time.perf_counter()
            _lib.check(_lib.lib.cpk_method_solve_device(ctx.h, METHOD, C.c_void_p(b1.data_ptr()), A.h, Cm.h, M.h,
                                                        C.byref(opts), C.c_void_p(xy.data_ptr()), C.byref(st)))
            ctx.synchronize()
            dt = time.perf_counter() - t
        per_it = dt / max(int(st.niters), 1) * 1e3
    except cpk.CpkError as e:
        err = str(e)[:120]
    dev_gb = (free0 - torch.cuda.mem_get_info(0)[0]) / 2**30
    print(json.dumps({"config": CONFIG, "P": P, "rank": r, "sweep": ctx.get_option("sweep"), "N_loc": len(dofs),
                      "nrounds": M.info["nrounds"], "sep": M.sep_info(),
                      "host_rss_peak_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 2),
                      "device_gb": round(dev_gb, 2),
                      "construct_s": round(construct_s, 3), "ptime_s": round(ptime_s, 3), "refactor_s": round(refactor_s, 4),
                      "spmv_us": round(p.spmv_ms * 1e3, 1), "resid_us": round(p.resid_ms * 1e3, 1),
                      "fwd_us": round(p.fwd_ms * 1e3, 1), "bwd_us": round(p.bwd_ms * 1e3, 1),
                      "apply_us": round(p.apply_ms * 1e3, 1), "niters": int(st.niters),
                      "ms_per_iter_no_comm": per_it and round(per_it, 4), "error": err}), flush=True)
    del M, A, B, Cm, G
    ctx.close()
