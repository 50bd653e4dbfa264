"""Halo and separator exchange volumes of the P-rank plans (host only, no GPU).

    python tools/halo_volumes.py [W] [P]

For the S10 generator with B window +-W (default 4) and P ranks (default 8), prints per rank:
the Kp and Krylov-operator (ac) halo payload kmax, how many values the rank reads from each
source rank, and the separator payload (tsend into kt slots).  DESIGN.md section 7d uses it to
cost a neighbour exchange against the allgather.
"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd import synthetic as syn  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    S = syn.saddle_system(N=10_000_000, window=W)
    t = time.time()
    for r in range(P):
        p = cpk.dist_plan(S["G"], S["B"], -S["C"], S["Q"], S["C"], P, r)
        nl = p["N_loc"]
        for k in ("kp", "ac"):
            col, km = p[f"{k}_col"], p[f"{k}_kmax"]
            g = np.unique(col[col >= nl] - nl)
            src = np.zeros(P, np.int64)
            if len(g):
                # slots per rank: kmax plus the spare slots the plan reserved (0..3)
                ks = next(s for s in range(km, km + 4) if np.all(g % s < km))
                src = np.bincount(g // ks, minlength=P)
            print(f"W{W} rank {r} {k}: N_loc {nl} kmax {km} nsend {len(p[f'{k}_send'])} "
                  f"ghosts {len(g)} per-source {src.tolist()}", flush=True)
        print(f"  nT {p['nT']} kt {p['kt']} tsend {len(p['tsend'])} ({time.time() - t:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
