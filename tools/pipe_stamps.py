"""Per-workgroup start/end of the round-0 sweep kernel at S10 (diagnostic library built with
-DCPK_PIPE_STAMPS, loaded through CPK_LIB_PATH): how much of a launch is the tail after most
workgroups have finished.  Two launches: the fused residual + forward sweep (the last launch of
cpk_profile_kernels) and the accumulating backward sweep (the last of one M*z)."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd import _lib  # noqa: E402
from cpkrylov_amd.synthetic import saddle_system  # noqa: E402

S = saddle_system(int(os.environ.get("N", "10000000")), window=int(os.environ.get("W", "4")))
ctx = cpk.Context(device=0)
A, Cm = cpk.Matrix(S["Q"], ctx), cpk.Matrix(S["C"], ctx)
M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
M.nitref, M.force_itref = 1, True
fn = _lib.lib.cpk_debug_pipe_stamps
fn.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.POINTER(C.c_int)]


def stamps(label):
    buf = (C.c_uint64 * (2 * 16384))()
    got = C.c_int(0)
    _lib.check(fn(buf, 16384, C.byref(got)))
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2)[:got.value].astype(np.int64)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0  # 100 MHz -> us
    dur = en - st
    q = np.percentile(en, [50, 90, 99, 100])
    print(json.dumps({"launch": label, "workgroups": int(len(a)), "span_us": round(float(en.max()), 2),
                      "start_spread_us": round(float(st.max()), 2),
                      "end_p50_p90_p99_max_us": [round(float(x), 2) for x in q],
                      "wg_dur_mean_min_max_us": [round(float(dur.mean()), 2), round(float(dur.min()), 2),
                                                 round(float(dur.max()), 2)],
                      "tail_after_p50_us": round(float(q[3] - q[0]), 2)}), flush=True)
    # per XCD (blocks b and b + 8 share one) and per dispatch round (blockIdx // 2048): is the
    # spread of workgroup durations tied to where a workgroup runs?
    g = np.arange(len(dur))
    xcd = [round(float(dur[g % 8 == x].mean()), 1) for x in range(8)]
    xmax = [round(float(dur[g % 8 == x].max()), 1) for x in range(8)]
    half = [round(float(dur[(g // 256) == h].mean()), 1) for h in range(min(16, (len(dur) + 255) // 256))]
    print(json.dumps({"launch": label, "dur_mean_by_xcd": xcd, "dur_max_by_xcd": xmax,
                      "dur_mean_by_256_block_group": half}), flush=True)


p = _lib.Profile()
_lib.check(_lib.lib.cpk_profile_kernels(ctx.h, A.h, Cm.h, M.h, 5, C.byref(p)))
stamps("fused residual + forward (round 0)")
z = np.random.default_rng(1).standard_normal(M.n)
_ = M * z
stamps("accumulating backward (round 0)")
