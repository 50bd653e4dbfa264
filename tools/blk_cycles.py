"""Per-block cycles of the round-0 sweep kernels at S10 (diagnostic library built with
-DCPK_PIPE_STAMPS, loaded through CPK_LIB_PATH), against the block's static features (levels,
rows, entries, Kps entries; env W = B window, default 4), and a least-squares cost model per kernel variant: the input of
the host-side longest-processing-time assignment of round-0 blocks to workgroups.
Writes gpurun_out/blk_cycles.npz and prints the fits as JSON."""
import ctypes as C
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd import _lib  # noqa: E402
from cpkrylov_amd.synthetic import saddle_system  # noqa: E402

S = saddle_system(int(os.environ.get("N", "10000000")), window=int(os.environ.get("W", "4")))
H = cpk.analyze(S["G"], S["B"], -S["C"])
rp, bl, lr, order, perm, L = H["round_ptr"], H["blk_lvl"], H["lvl_row"], H["order"], H["perm"], H["L"]
nb = int(rp[1] - rp[0])
r0, r1 = lr[bl[:nb]], lr[bl[1:nb + 1]]
nl = bl[1:nb + 1] - bl[:nb]
fcnt = np.diff(L.tocsr().indptr)[order]
bcnt = np.diff(L.indptr)[order]
Kp = sp.bmat([[S["G"], S["B"].T], [S["B"], -S["C"]]]).tocsr()
kcnt = np.diff(Kp.indptr)[perm[order]]
cum = lambda c: np.concatenate([[0], np.cumsum(c)])
fe, be, ke = (cum(c)[r1] - cum(c)[r0] for c in (fcnt, bcnt, kcnt))
rows = r1 - r0

ctx = cpk.Context(device=0)
M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
M.nitref, M.force_itref = 1, True
z = np.random.default_rng(1).standard_normal(M.n)
for _ in range(3):
    _ = M * z
KMAX = 1 << 20  # kBlkCycMax: round-0 cycles are keyed by the block's first level
buf = np.zeros(4 * KMAX, np.uint64)
got = C.c_int64(0)
_lib.check(_lib.lib.cpk_debug_blk_cycles(buf.ctypes.data_as(C.POINTER(C.c_uint64)), buf.size, C.byref(got)))
cyc = buf.reshape(4, KMAX)[:, bl[:nb]].astype(np.float64)
np.savez(os.path.join(os.environ.get("OUT", "gpurun_out"), f"blk_cycles_w{os.environ.get('W', '4')}.npz"), cyc=cyc, rows=rows, nl=nl, fe=fe, be=be,
         ke=ke)
names = ["fwd", "fwd_resid", "bwd", "bwd_add"]
for v in range(4):
    y = cyc[v]
    if not np.any(y > 0):
        print(json.dumps({"variant": names[v], "blocks": 0}))
        continue
    ent = be if v >= 2 else fe
    X = np.stack([np.ones(nb), nl, rows, ent] + ([ke] if v == 1 else []), 1).astype(np.float64)
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    pred = X @ coef
    r2 = 1 - np.sum((y - pred) ** 2) / np.sum((y - y.mean()) ** 2)
    # the levels-only model the assignment uses (kR0Cost): its R^2 for comparison
    c1, *_ = np.linalg.lstsq(X[:, :2], y, rcond=None)
    r2l = 1 - np.sum((y - X[:, :2] @ c1) ** 2) / np.sum((y - y.mean()) ** 2)
    print(json.dumps({"variant": names[v], "levels_only_coef": [round(float(c), 2) for c in c1],
                      "levels_only_r2": round(float(r2l), 3)}), flush=True)
    print(json.dumps({"variant": names[v], "blocks": nb, "mean_cycles": round(float(y.mean()), 1),
                      "cv": round(float(y.std() / y.mean()), 3), "coef[1,nl,rows,ent(,kps)]": [round(float(c), 2) for c in coef],
                      "r2": round(float(r2), 3), "p99_resid_frac": round(float(np.percentile(np.abs(y - pred) / y.mean(), 99)), 3)}),
          flush=True)
