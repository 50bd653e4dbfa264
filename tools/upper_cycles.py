"""Phase cycles of the upper-round sweep blocks at S10 (diagnostic library built with
-DCPK_PIPE_STAMPS, loaded through CPK_LIB_PATH): for every block of the rounds above round 0
that runs through sptrsv_upper_kernel, the s_memtime cycles of its staging (loads, gathers, LDS
image), prefix fold, one-wave level loop and write-back, forward and backward, from the last
apply.  Prints one JSON line per (round, direction) with the phase means / medians / maxima and
the block shape (rows, levels, entries)."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd import _lib  # noqa: E402
from cpkrylov_amd.synthetic import saddle_system  # noqa: E402

KMAX = 1 << 20  # kBlkCycMax (kernels.hip)
S = saddle_system(int(os.environ.get("N", "10000000")), window=int(os.environ.get("W", "4")))
H = cpk.analyze(S["G"], S["B"], -S["C"])
rp, bl, lr, order, L = H["round_ptr"], H["blk_lvl"], H["lvl_row"], H["order"], H["L"]
fcnt = np.diff(L.tocsr().indptr)[order]
bcnt = np.diff(L.indptr)[order]
cum = lambda c: np.concatenate([[0], np.cumsum(c)])  # noqa: E731
cf, cb = cum(fcnt), cum(bcnt)

ctx = cpk.Context(device=0, options={"no_chain": 1})  # one launch per round: stamps per round
M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
M.nitref, M.force_itref = 1, True
z = np.random.default_rng(1).standard_normal(M.n)
for _ in range(3):
    _ = M * z
buf = np.zeros(12 * KMAX, np.uint64)
got = C.c_int64(0)
_lib.check(_lib.lib.cpk_debug_blk_cycles(buf.ctypes.data_as(C.POINTER(C.c_uint64)), buf.size, C.byref(got)))
cyc = buf.reshape(12, KMAX).astype(np.float64)
phases = ["staging", "fold", "levels", "writeback"]
for r in range(1, len(rp) - 1):
    b0, b1 = int(rp[r]), int(rp[r + 1])
    r0, r1 = lr[bl[b0:b1]], lr[bl[b0 + 1:b1 + 1]]
    shape = {"blocks": b1 - b0, "rows_mean": round(float(np.mean(r1 - r0)), 1),
             "levels_mean": round(float(np.mean(bl[b0 + 1:b1 + 1] - bl[b0:b1])), 1)}
    for d, name in ((0, "fwd"), (1, "bwd")):
        c = cyc[4 + 4 * d: 8 + 4 * d, b0:b1]
        if not np.any(c > 0):
            print(json.dumps({"round": r, "dir": name, "stamps": 0, **shape}), flush=True)
            continue
        ent = (cf if d == 0 else cb)
        out = {"round": r, "dir": name, **shape,
               "entries_mean": round(float(np.mean(ent[r1] - ent[r0])), 1)}
        for k, p in enumerate(phases):
            out[p] = [round(float(np.mean(c[k])), 0), round(float(np.median(c[k])), 0), round(float(np.max(c[k])), 0)]
        tot = c.sum(0)
        out["total_mean_median_max"] = [round(float(tot.mean()), 0), round(float(np.median(tot)), 0),
                                        round(float(tot.max()), 0)]
        print(json.dumps(out), flush=True)

# per-block records (BLOCKS=<path>): the loop-cost model of every upper block and direction
# (cpk_debug_block_model) beside its measured phase cycles -- the model's calibration data
if os.environ.get("BLOCKS"):
    n = C.c_int64(0)
    _lib.check(_lib.lib.cpk_debug_block_model(M.h, None, 1 << 40, C.byref(n)))
    mod = np.zeros(max(n.value, 1), np.int64)
    _lib.check(_lib.lib.cpk_debug_block_model(M.h, mod.ctypes.data_as(C.POINTER(C.c_int64)), n.value, C.byref(n)))
    mod = mod[:n.value].reshape(-1, 8)
    with open(os.environ["BLOCKS"], "w") as f:
        for b, d, nr, lt, dt, outs, valid, choice in mod.tolist():
            ph = cyc[4 + 4 * d: 8 + 4 * d, b].tolist() if b < KMAX else [0, 0, 0, 0]
            f.write(json.dumps({"b": b, "dir": d, "nr": nr, "lt": lt, "dt": dt, "outs": outs, "valid": valid,
                                "choice": choice, "cyc": ph}) + "\n")

