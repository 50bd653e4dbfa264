"""Line-level read model of the round-0 forward sweep at S10 (host only, no GPU).

Attributes the forward sweep's PMC fetch excess (FETCH_SIZE x2 over the algorithmic bytes,
DESIGN.md section 5) to its arrays.  For every round-0 block it lists the 128-byte lines each
array occupies (row pointers, perm indices, int16 columns, values, the block record) and the
lines of the input x the perm gather touches, then counts them three ways:
  per_block  every block fetches its own lines (no reuse between blocks),
  xcd_window distinct lines per XCD among the blocks resident at once (G consecutive blocks,
             block b on XCD (b mod G) mod 8 -- the static stride mapping),
  xcd_launch distinct lines per XCD over the whole launch (an L2 that never evicts).
The algorithmic count is the section 8d model (every byte once).

With --chunk K, runs of K consecutive blocks share an XCD (block b on XCD (b // K) mod 8).

  python tools/fwd_traffic_model.py [--N 10000000] [--grid 4096] [--chunk K]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd import synthetic  # noqa: E402

LINE = 128


def lines_of_ranges(start, stop):
    """start/stop byte offsets per block -> (block index, line) pairs of every line touched."""
    a = start // LINE
    b = (stop - 1) // LINE
    n = np.maximum(b - a + 1, 0)
    blk = np.repeat(np.arange(start.size), n)
    off = np.arange(n.sum()) - np.repeat(np.cumsum(n) - n, n)
    return blk, np.repeat(a, n) + off


def count(blk, line, grid, chunk=0):
    xcd = (blk // chunk) % 8 if chunk else (blk % grid) % 8
    win = blk // grid
    per_block = np.unique(blk.astype(np.int64) * (1 << 32) + line).size
    key_w = (win.astype(np.int64) * 8 + xcd) * (1 << 36) + line
    xcd_window = np.unique(key_w).size
    xcd_launch = np.unique(xcd.astype(np.int64) * (1 << 36) + line).size
    return per_block * LINE, xcd_window * LINE, xcd_launch * LINE


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=10_000_000)
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--chunk", type=int, default=0)
    a = ap.parse_args()
    t = time.time()
    S = synthetic.saddle_system(a.N)
    an = cpk.analyze(S["G"], S["B"], -S["C"])
    print(f"analysis {time.time() - t:.1f} s", flush=True)
    L, perm, order = an["L"], an["perm"], an["order"]
    rp, bl, lr = an["round_ptr"], an["blk_lvl"], an["lvl_row"]
    N = perm.size
    rowcnt = np.bincount(L.indices, minlength=N)[order].astype(np.int64)  # forward entries per schedule row
    eptr = np.concatenate([[0], np.cumsum(rowcnt)])
    b0, b1 = rp[0], rp[1]
    r_start = lr[bl[b0:b1]]
    r_stop = lr[bl[b0 + 1:b1 + 1]]
    e_start, e_stop = eptr[r_start], eptr[r_stop]
    nb = b1 - b0
    rows0 = int(r_stop[-1] - r_start[0])
    ent0 = int(e_stop[-1] - e_start[0])
    print(f"round 0: {nb} blocks, {rows0} rows, {ent0} entries (of {N} rows, {eptr[-1]} entries)")
    arrays = {
        "row pointers (u32)": (r_start * 4, r_stop * 4 + 4, 4 * (rows0 + 1)),
        "perm indices (i32)": (r_start * 4, r_stop * 4, 4 * rows0),
        "columns (i16)": (e_start * 2, e_stop * 2, 2 * ent0),
        "values (f64)": (e_start * 8, e_stop * 8, 8 * ent0),
        "block records (32 B)": (np.arange(nb) * 32, np.arange(nb) * 32 + 32, 32 * nb),
    }
    tot = np.zeros(4)
    print(f"{'array':24s} {'algorithmic':>12s} {'per_block':>12s} {'xcd_window':>12s} {'xcd_launch':>12s}  (MB)")
    for name, (s, e, alg) in arrays.items():
        blk, line = lines_of_ranges(np.asarray(s, np.int64), np.asarray(e, np.int64))
        c = count(blk, line, a.grid, a.chunk)
        tot += (alg, *c)
        print(f"{name:24s} {alg / 1e6:12.1f} " + " ".join(f"{v / 1e6:12.1f}" for v in c))
    # the perm gather of the input x (8-byte elements at perm[order[q]])
    q = np.arange(r_start[0], r_stop[-1])
    blk = np.repeat(np.arange(nb), r_stop - r_start)
    line = (perm[order[q]].astype(np.int64) * 8) // LINE
    c = count(blk, line, a.grid, a.chunk)
    alg = 8 * rows0
    tot += (alg, *c)
    print(f"{'x gather (f64, perm)':24s} {alg / 1e6:12.1f} " + " ".join(f"{v / 1e6:12.1f}" for v in c))
    print(f"{'total reads':24s} " + " ".join(f"{v / 1e6:12.1f}" for v in tot))
    print(f"ratio to algorithmic: per_block {tot[1] / tot[0]:.3f}  xcd_window {tot[2] / tot[0]:.3f}  "
          f"xcd_launch {tot[3] / tot[0]:.3f}")


if __name__ == "__main__":
    main()
