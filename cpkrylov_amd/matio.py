"""MATLAB data files for the example programs (the `.mat` loader).

The reference's example programs start with `load(filename)` of a system from Orban's IPM
collection -- K, rhs and the block sizes nH, nJ, nZ (examples/cpk_exprog1.m:45-49,
cpk_exprog2.m:47-51) -- and cut the constraint-preconditioner blocks out of K
(cpk_exprog1.m:62-67).  `load_mat` reads such a file (MAT v5 through scipy.io; v7.3 files are
HDF5, which scipy does not read -- they raise a clear error) and `saddle_blocks` makes the cut.
Data only: nothing in a file is executed (scipy.io.loadmat builds arrays, it unpickles nothing).
"""
import numpy as np
import scipy.sparse as sp

from ._lib import CPK_ERR_ARGS, CpkError


def load_mat(path):
    """load(filename): the file's variables as a dict -- sparse matrices as CSR (float64),
    dense arrays as float64 ndarrays (column vectors raveled), 1x1 numbers as Python ints when
    integral (the block sizes), else floats.  MATLAB's own class of a scalar is irrelevant here:
    the examples read them as dimensions."""
    import scipy.io as sio
    try:
        raw = sio.loadmat(path, mat_dtype=True)
    except NotImplementedError as e:  # scipy: "Please use HDF reader for matlab v7.3 files"
        raise CpkError(CPK_ERR_ARGS, f"load_mat: {path}: MAT v7.3 (HDF5) files are not supported: {e}") from e
    out = {}
    for k, v in raw.items():
        if k.startswith("__"):
            continue
        if sp.issparse(v):
            out[k] = sp.csr_matrix(v, dtype=np.float64)
            out[k].sort_indices()
        elif isinstance(v, np.ndarray) and v.dtype.kind in "biuf":
            a = np.asarray(v, dtype=np.float64)
            if a.size == 1:
                x = float(a.ravel()[0])
                out[k] = int(x) if x.is_integer() else x
            elif a.ndim == 2 and 1 in a.shape:
                out[k] = a.ravel()
            else:
                out[k] = a
        else:
            out[k] = v
    return out


def saddle_blocks(K, n):
    """The blocks of K = [Q A'; A -C] the examples build (cpk_exprog1.m:62-67, cpk_exprog2.m:61-66):
    Q = K(1:n,1:n), G = diag(Q) (spdiags), A = K(n+1:end,1:n), C = -K(n+1:end,n+1:end).
    Returns (Q, A, C, G) as CSR."""
    K = sp.csr_matrix(K)
    N = K.shape[0]
    if K.shape != (N, N) or not 0 < n <= N:
        raise CpkError(CPK_ERR_ARGS, f"saddle_blocks: K is {K.shape}, n = {n}")
    Q = K[:n, :n].tocsr()
    G = sp.diags(Q.diagonal(), 0, shape=(n, n), format="csr")
    A = K[n:, :n].tocsr()
    C = (-K[n:, n:]).tocsr()
    return Q, A, C, G
