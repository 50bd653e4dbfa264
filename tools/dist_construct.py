"""Construction of a P-way distributed preconditioner on P simulated ranks (threads of this
process, one GPU, SimComm): wall time, every rank's ptime, and the process's peak host RSS (the
sum over the ranks, as the node's P processes would hold it).  The global analysis is broadcast
from rank 0 (default) or run by every rank (NO_BCAST=1: engine option no_bcast_analysis).

usage: CONFIG=s10|s50 [NO_BCAST=1] python tools/dist_construct.py P"""
import os
import resource
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd.synthetic import nonsym_system, saddle_system  # noqa: E402


def rss_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    cfg = os.environ.get("CONFIG", "s10")
    S = nonsym_system(50_000_000) if cfg == "s50" else saddle_system(10_000_000)
    print(f"{cfg}: system built, peak RSS {rss_gb():.1f} GB", flush=True)
    opts = {"no_bcast_analysis": 1} if os.environ.get("NO_BCAST") else {}
    g = cpk.SimGroup(P)
    t0 = time.time()

    def one(r):
        ctx = cpk.Context(device=0, rank=r, nranks=P, simgroup=g, options=opts)
        try:
            t = time.time()
            M = cpk.opLDL2(S["G"], S["B"], -S["C"], ctx=ctx)
            dt = time.time() - t
            pt = M.ptime
            del M
            return dt, pt
        finally:
            ctx.close()

    with ThreadPoolExecutor(P) as ex:
        res = [f.result() for f in [ex.submit(one, r) for r in range(P)]]
    wall = time.time() - t0
    print({"config": cfg, "P": P, "bcast": not opts, "wall_s": round(wall, 2),
           "rank_s": [round(a, 2) for a, _ in res], "ptime_s": [round(b, 2) for _, b in res],
           "peak_rss_gb_process": round(rss_gb(), 1)}, flush=True)


if __name__ == "__main__":
    main()
