"""Construction time of the S10 preconditioner on the GPU box, phase by phase (CPK_TIMING=1
prints the host phases to stderr; this prints the total and a refactorization)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("CPK_TIMING", "1")
import cpkrylov_amd as cpk  # noqa: E402
from cpkrylov_amd.synthetic import saddle_system  # noqa: E402

S = saddle_system(int(os.environ.get("N", "10000000")))
ctx = cpk.Context(device=0)
G, B = cpk.Matrix(S["G"], ctx), cpk.Matrix(S["B"], ctx)
for rep in range(2):
    t = time.perf_counter()
    M = cpk.opLDL2(G, B, -S["C"], ctx=ctx)
    print(f"construction {rep}: {time.perf_counter() - t:.3f} s (ptime {M.ptime:.3f} s)", flush=True)
print(f"refactor: {M.refactor(S['G'], S['B'], -S['C']):.3f} s", flush=True)
