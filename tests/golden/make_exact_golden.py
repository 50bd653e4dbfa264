"""Golden references of the headline runs in EXACT mode (engine option exact_dots / the oracle's
orc_set_exact), for tests/test_gpu_scale.py::test_*_exact_*.

In exact mode every inner product is the correctly rounded exact sum of its TwoProd pairs, so
the summation order -- OpenMP threads here, the GPU's grid and rank count there -- changes no
bit, and the oracle given the product's factors runs the device's arithmetic operation for
operation.  The factors come from the product's own host analysis (cpk.analyze: ordering,
symbolic and numeric LDL', no GPU; the device numeric phase reproduces them bit for bit,
test_gpu_factor.py), so the fixture also pins the factorization: the test checks hashes of the
GPU's exported perm, L and D against it.

Recorded: niters, solved, the full history, every XSTEP-th entry of x, a SHA-256 of all of x, and
the hashes of perm / L / D.  The serial restatement (one thread) is what the fixture claims; the
run uses the OpenMP leg for time and checks its first iterations against the serial run.

  python tests/golden/make_exact_golden.py s10   # ~1 minute, ~10 GB
  python tests/golden/make_exact_golden.py s50   # ~15 minutes on 8 cores, ~45 GB
  python tests/golden/make_exact_golden.py w64   # the +-64 window system, ~3 minutes, ~14 GB

Output: tests/golden/{s10,s50,w64}_exact_golden.npz (data only).
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
from cpkrylov_amd.synthetic import nonsym_system, saddle_system  # noqa: E402
from oracle import oracle as O  # noqa: E402

XSTEP = 5003
EXPROG = dict(print=False, atol=1.0e-6, rtol=1.0e-6, itmax=500, residual_update=True, nitref=1, force_itref=True,
              itref_tol=1.0e-8)
CONFIGS = {
    # S10: the bench's converging cpminres (config 4); S50: the bench's truncated cpdqgmres(40)
    "s10": dict(N=10_000_000, gen=saddle_system, method="minres", opts=EXPROG),
    "s50": dict(N=50_000_000, gen=nonsym_system, method="dqgmres", opts=dict(EXPROG, itmax=120, mem=40)),
    # SURVEY 8d's +-64 coupling window at 10 M dofs: the bench's headline system since round 6
    "w64": dict(N=10_000_000, gen=lambda N: saddle_system(N=N, window=64), method="minres", opts=EXPROG),
}
PC = ("nitref", "itref_tol", "force_itref", "residual_update")


def log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def solve(S, Mo, cfg, threads, itmax=None):
    opts = dict(cfg["opts"]) if itmax is None else dict(cfg["opts"], itmax=itmax)
    # the dead residual-update SpMVs of a value object subtract zeros: same bits
    opts["residual_update"] = False
    O.set_threads(threads)
    try:
        t = time.perf_counter()
        with O.exact():
            x, st = O.reg_solve(cfg["method"], S["rhs"], S["Q"], S["B"], S["C"], Mo, opts)
        log(f"oracle exact threads={threads}: {st['niters']} iterations in {time.perf_counter() - t:.0f} s")
        return x, st
    finally:
        O.set_threads(1)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "s10"
    cfg = CONFIGS[which]
    t = time.perf_counter()
    S = cfg["gen"](N=cfg["N"])
    log(f"{which} generated, N={S['N']} ({time.perf_counter() - t:.0f} s)")
    an = cpk.analyze(S["G"], S["B"], -S["C"])
    L, D, perm = an["L"], an["D"], np.ascontiguousarray(an["perm"], np.int32)
    del an
    log(f"product factors from the host analysis: nnz(L) {L.nnz}")
    Mo = O.LDL2(S["G"], S["B"], -S["C"], factors=(L, D, perm))
    Mo.set(**{k: float(cfg["opts"][k]) for k in PC})
    T = min(8, os.cpu_count() or 1)
    # the serial restatement against the OpenMP leg on the first iterations (thread-independence)
    x1, s1 = solve(S, Mo, cfg, 1, itmax=3)
    xT, sT = solve(S, Mo, cfg, T, itmax=3)
    assert np.array_equal(x1, xT) and np.array_equal(s1["residHistory"], sT["residHistory"])
    x, st = solve(S, Mo, cfg, T)
    h = np.asarray(st["residHistory"])
    out = os.path.join(HERE, f"{which}_exact_golden.npz")
    np.savez_compressed(out, N=np.int64(S["N"]), niters=np.int64(st["niters"]), solved=np.int64(st["solved"]),
                        itmax=np.int64(cfg["opts"]["itmax"]), hist=h, x_sample_step=np.int64(XSTEP),
                        x_sample=x[::XSTEP].copy(), x_sha256=sha(x), perm_sha256=sha(perm),
                        L_sha256=sha(L.data), D_sha256=sha(D), nnz_l=np.int64(L.nnz))
    log(f"wrote {out}: niters {st['niters']} solved {st['solved']} h[-1]/h[0] {h[-1] / h[0]:.3e}")


if __name__ == "__main__":
    main()
