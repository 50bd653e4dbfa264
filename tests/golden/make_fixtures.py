"""Convert the reference's two MATLAB example systems into compact, data-only CSR fixtures.

Source (read as DATA only, never executed): /root/reference/examples/
  cvxqp1_m_2x2_symm_iter10.mat      (used by examples/cpk_exprog1.m:45-49, n = nH, m = nJ)
  cvxqp2_s_3x3_nonsymm_perm_iter10.mat (used by examples/cpk_exprog2.m:47-50, n = nH + nZ, m = nJ)

Each .npz holds K (CSR: K_indptr int64, K_indices int32, K_data f64), rhs (f64), n, m,
and x_direct = K \\ rhs computed here with scipy's SuperLU (the examples' own check,
cpk_exprog1.m:101 / cpk_exprog2.m:100).  The fixtures are loaded with numpy.load
(allow_pickle=False).  Run: python tests/golden/make_fixtures.py
"""
import os
import numpy as np
import scipy.io as sio
import scipy.sparse as sp
import scipy.sparse.linalg as spl

REF = "/root/reference/examples"
OUT = os.path.dirname(os.path.abspath(__file__))

CASES = {
    # name: (mat file, function giving (n, m) from the header scalars)
    "cvxqp1_m": ("cvxqp1_m_2x2_symm_iter10.mat", lambda d: (d["nH"], d["nJ"])),
    "cvxqp2_s": ("cvxqp2_s_3x3_nonsymm_perm_iter10.mat", lambda d: (d["nH"] + d["nZ"], d["nJ"])),
}


def main():
    for name, (fname, dims) in CASES.items():
        d = sio.loadmat(os.path.join(REF, fname), mat_dtype=True)
        hdr = {k: int(d[k][0, 0]) for k in ("n", "nH", "nJ", "nZ")}
        n, m = dims(hdr)
        K = d["K"].tocsr()
        K.sort_indices()
        rhs = np.asarray(d["rhs"], dtype=np.float64).ravel()
        assert K.shape == (n + m, n + m) and rhs.shape == (n + m,)
        x_direct = spl.spsolve(K.tocsc(), rhs)
        np.savez_compressed(
            os.path.join(OUT, f"{name}.npz"),
            K_indptr=K.indptr.astype(np.int64), K_indices=K.indices.astype(np.int32),
            K_data=K.data.astype(np.float64), rhs=rhs, n=np.int64(n), m=np.int64(m),
            x_direct=x_direct, **{f"hdr_{k}": np.int64(v) for k, v in hdr.items()})
        print(name, "N", n + m, "n", n, "m", m, "nnz", K.nnz,
              "resid(K x_direct - rhs)", np.linalg.norm(K @ x_direct - rhs) / np.linalg.norm(rhs))


if __name__ == "__main__":
    main()
