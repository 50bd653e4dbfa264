"""Golden vectors of the CPU oracle on the reference's example systems (committed data).

Runs oracle/ (the C restatement, reverse Cuthill-McKee ordering -- independent of the
product's ordering) with the examples' options (cpk_exprog1.m:79-90, cpk_exprog2.m:69-90)
for every method the examples name (cpk_exprog1.m:67-74, cpk_exprog2.m:69-74) and saves
niters, solved, the histories and x to tests/golden/oracle_<system>_<method>[_<param>].npz.
Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import fixtures as F  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = [("cvxqp1_m", "minres", {}), ("cvxqp1_m", "cg", {}), ("cvxqp1_m", "cglanczos", {}),
         ("cvxqp1_m", "symmlq", {}), ("cvxqp1_m", "dqgmres", {"mem": 2}),
         ("cvxqp2_s", "gmres", {"restart": 100}), ("cvxqp2_s", "gmres", {"restart": 20}),
         ("cvxqp2_s", "dqgmres", {"mem": 100}), ("cvxqp2_s", "dqgmres", {"mem": 20})]


def case_file(name, method, extra):
    tag = "".join(f"_{k}{v}" for k, v in sorted(extra.items()))
    return os.path.join(HERE, f"oracle_{name}_{method}{tag}.npz")


def run(name, method, extra):
    P = F.load(name)
    opts = dict(F.EXPROG_OPTS, **extra)
    x, st = O.reg_cpkrylov(method, P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts, order="rcm")
    return x, st


def main():
    for name, method, extra in CASES:
        x, st = run(name, method, extra)
        out = {"x": x, "niters": np.int64(st["niters"]), "solved": np.int64(st["solved"])}
        for k, v in st.items():
            if k.endswith("History"):
                out[k] = v
        if "status" in st:
            out["status"] = np.array(st["status"])
        np.savez_compressed(case_file(name, method, extra), **out)
        print(name, method, extra, st["niters"], st["solved"])


if __name__ == "__main__":
    main()
