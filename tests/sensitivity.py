"""Sensitivity band of a solve (test infrastructure): the largest deviation of the oracle's
histories (relative to history[0]) and of x (relative to ||x||) when the rhs is perturbed by
random relative amounts of 1e-15.  Rounding differences of any other source -- the GPU's
summation order, MATLAB's MKL -- are of this size, so parity tolerances are expressed in it."""
import functools

import numpy as np

import fixtures as F
from oracle import oracle as O


def _opts(extra):
    return dict(F.EXPROG_OPTS, **extra)


@functools.lru_cache(maxsize=None)
def _band(name, method, extra_items, perm_bytes, trials=4, eps=1e-15):
    P = F.load(name)
    perm = np.frombuffer(perm_bytes, dtype=np.int32)
    opts = _opts(dict(extra_items))
    x1, s1 = O.reg_cpkrylov(method, P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts, perm=perm)
    keys = [k for k in s1 if k.endswith("History")]
    out = {k: 0.0 for k in keys}
    out["x"] = 0.0
    rng = np.random.default_rng(12345)
    for _ in range(trials):
        b = P["rhs"] * (1 + eps * rng.standard_normal(P["rhs"].shape[0]))
        x2, s2 = O.reg_cpkrylov(method, b, P["Q"], P["B"], P["C"], P["G"], opts, perm=perm)
        for k in keys:
            L = min(len(s1[k]), len(s2[k]))
            out[k] = max(out[k], float(np.max(np.abs(s1[k][:L] - s2[k][:L])) / s1[k][0]))
        out["x"] = max(out["x"], float(np.linalg.norm(x1 - x2) / np.linalg.norm(x1)))
    return out


def band(name, method, extra, perm):
    return _band(name, method, tuple(sorted(extra.items())), np.ascontiguousarray(perm, np.int32).tobytes())
