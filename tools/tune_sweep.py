"""Time the triangular sweeps at S10 for several LDS staging configurations (GPU)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd import _lib  # noqa: E402
from cpkrylov_amd.synthetic import saddle_system  # noqa: E402

S = saddle_system(int(os.environ.get("N", "10000000")))
ctx = cpk.Context(device=0)
A, Cm = cpk.Matrix(S["Q"], ctx), cpk.Matrix(S["C"], ctx)
for cfg in sys.argv[1:]:
    ctx.set_option("sweep", cfg)  # engine options live in the context (read when M is built)
    M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
    M.nitref, M.force_itref = 1, True
    p = _lib.Profile()
    _lib.check(_lib.lib.cpk_profile_kernels(ctx.h, A.h, Cm.h, M.h, int(os.environ.get("REPS", "20")), C.byref(p)))
    print(f"{cfg:16s} rounds {M.info['nrounds']} blocks {M.info['nblocks']:6d} fwd {p.fwd_ms*1e3:7.1f} us "
          f"({p.fwd_bytes/p.fwd_ms/1e6:6.0f} GB/s) bwd {p.bwd_ms*1e3:7.1f} us ({p.bwd_bytes/p.bwd_ms/1e6:6.0f} GB/s) "
          f"apply {p.apply_ms*1e3:7.1f} us resid {p.resid_ms*1e3:6.1f} us spmv {p.spmv_ms*1e3:6.1f} us "
          f"fused resid+fwd {p.fwd_resid_ms*1e3:7.1f} us", flush=True)
    del M
