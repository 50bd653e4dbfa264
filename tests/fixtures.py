"""Loads the reference's example systems (tests/golden/*.npz, data only) and cuts the blocks
exactly as the examples do: Q = K(1:n,1:n); G = diag(diag(Q)); A = K(n+1:end,1:n);
C = -K(n+1:end,n+1:end)  (examples/cpk_exprog1.m:59-63, cpk_exprog2.m:61-65), and the
options of the examples (cpk_exprog1.m:79-90, cpk_exprog2.m:69-90)."""
import os

import numpy as np
import scipy.sparse as sp

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

EXPROG_OPTS = dict(print=False, atol=1.0e-6, rtol=1.0e-6, itmax=500,
                   residual_update=True, nitref=1, force_itref=True, itref_tol=1.0e-8)


SYNTHETIC = {"syn_nonsym20k": ("nonsym_system", 20000), "syn_symm20k": ("saddle_system", 20000)}


def _synthetic(name):
    """Small instances of the benchmark generators (cpkrylov_amd/synthetic.py), with the same
    dict layout as the reference fixtures; x_direct from a sparse direct solve."""
    import scipy.sparse.linalg as spl

    from cpkrylov_amd import synthetic
    fn, N = SYNTHETIC[name]
    S = getattr(synthetic, fn)(N=N)
    n, m = S["n"], S["m"]
    K = sp.bmat([[S["Q"], S["B"].T], [S["B"], -S["C"]]]).tocsr()
    K.sort_indices()
    x = spl.spsolve(K.tocsc(), S["rhs"])
    return dict(name=name, n=n, m=m, K=K, Q=S["Q"], G=S["G"], B=S["B"], C=S["C"], rhs=S["rhs"], x_direct=x)


_CACHE = {}


def load(name):
    if name in SYNTHETIC:
        if name not in _CACHE:
            _CACHE[name] = _synthetic(name)
        d = _CACHE[name]
        return {k: (v.copy() if hasattr(v, "copy") else v) for k, v in d.items()}
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    n, m = int(z["n"]), int(z["m"])
    K = sp.csr_matrix((z["K_data"], z["K_indices"], z["K_indptr"]), shape=(n + m, n + m))
    Q = K[:n, :n].tocsr()
    G = sp.diags(Q.diagonal()).tocsr()
    A = K[n:, :n].tocsr()
    Cm = (-K[n:, n:]).tocsr()
    for M in (Q, G, A, Cm):
        M.sort_indices()
    return dict(name=name, n=n, m=m, K=K, Q=Q, G=G, B=A, C=Cm, rhs=z["rhs"].copy(),
                x_direct=z["x_direct"].copy())
