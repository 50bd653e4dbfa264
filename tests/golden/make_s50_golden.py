"""Golden reference of the S50 headline run, from the SERIAL oracle.

On the GPU box the S50 parity test compares against the oracle's OpenMP leg (the serial window
loops take ~10 s per iteration there), with a 10x safety factor on that leg's band.  This script
runs the serial restatement itself once, here on the CPU, with the product's pivot order (the
host analysis is deterministic for any thread count), and records

  * the serial history of cpdqgmres(40) over the bench's truncated run (S50_ITMAX iterations),
    niters and the solved flag;
  * x's norm and a fixed sample of x (every XSTEP-th entry);
  * the serial reference's own band: the largest deviation from it of the same solve with the
    inner products partitioned over 2, 4 and 8 OpenMP threads (each a different summation order
    of every dot product -- the only thing a parallel implementation changes);
  * a hash of the pivot order, so the test can check that the GPU ran the same order.

Run (about an hour on 8 cores, ~45 GB of memory):  python tests/golden/make_s50_golden.py
The output, tests/golden/s50_serial_golden.npz, is data only.
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import cpkrylov_amd as cpk  # noqa: E402  (host-only analysis: no GPU is touched)
from cpkrylov_amd.synthetic import nonsym_system  # noqa: E402
from oracle import oracle as O  # noqa: E402

N = int(os.environ.get("CPK_S50_N", 50_000_000))
ITMAX = int(os.environ.get("CPK_S50_ITMAX", 120))
XSTEP = 5003  # sampled x entries: 0, XSTEP, 2 XSTEP, ...
OPTS = dict(print=False, atol=1.0e-6, rtol=1.0e-6, itmax=ITMAX, residual_update=False, nitref=1,
            force_itref=True, itref_tol=1.0e-8, mem=40)
OUT = os.path.join(HERE, "s50_serial_golden.npz" if N == 50_000_000 else f"s50_serial_golden_{N}.npz")


def log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def solve(S, perm, threads):
    O.set_threads(threads)
    try:
        t = time.perf_counter()
        x, st = O.reg_cpkrylov("dqgmres", S["rhs"], S["Q"], S["B"], S["C"], S["G"], OPTS, perm=perm)
        log(f"oracle threads={threads}: {st['niters']} iterations in {time.perf_counter() - t:.0f} s")
        return x, st
    finally:
        O.set_threads(1)


def main():
    t = time.perf_counter()
    S = nonsym_system(N=N)
    log(f"S50 generated, N={S['N']} ({time.perf_counter() - t:.0f} s)")
    perm = np.ascontiguousarray(cpk.analyze(S["G"], S["B"], -S["C"])["perm"], np.int32)
    log("product pivot order from the host analysis")
    x, st = solve(S, perm, 1)
    h = np.asarray(st["residHistory"])
    sample = np.arange(0, S["N"], XSTEP)
    band_h, band_x = 0.0, 0.0
    legs = {}
    for T in (2, 4, 8):
        xt, stt = solve(S, perm, T)
        ht = np.asarray(stt["residHistory"])
        L = min(len(ht), len(h))
        legs[T] = float(np.max(np.abs(ht[:L] - h[:L])) / h[0])
        band_h = max(band_h, legs[T])
        band_x = max(band_x, float(np.linalg.norm(xt[sample] - x[sample]) / np.linalg.norm(x[sample])))
        assert stt["niters"] == st["niters"], (T, stt["niters"], st["niters"])
    log(f"band over 2/4/8 threads: hist {band_h:.3e} ({legs}) x(sample) {band_x:.3e}")
    np.savez_compressed(OUT, N=np.int64(S["N"]), itmax=np.int64(ITMAX), niters=np.int64(st["niters"]),
                        solved=np.int64(st["solved"]), hist=h, x_norm=np.float64(np.linalg.norm(x)),
                        x_sample_step=np.int64(XSTEP), x_sample=x[sample], band_hist=np.float64(band_h),
                        band_x_sample=np.float64(band_x),
                        band_legs=np.array([legs[2], legs[4], legs[8]]),
                        perm_sha256=np.frombuffer(hashlib.sha256(perm.tobytes()).digest(), np.uint8))
    log(f"wrote {OUT}")


if __name__ == "__main__":
    main()
