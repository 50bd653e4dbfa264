"""The reference's example programs on the GPU: `cpkrylov_amd.load_mat`
(MAT v5) and the drivers `examples/cpk_exprog1.py` / `cpk_exprog2.py`, which mirror
examples/cpk_exprog1.m:44-104 and cpk_exprog2.m:44-104 -- load, block cut (cpk_exprog1.m:62-67),
reg_cpkrylov with the example options, the comparison with K \\ rhs.

The reference's `.mat` files stay in /root/reference (they do not travel to the GPU box): the CPU
test checks that load_mat reads them to exactly the arrays of the committed data fixtures
(tests/golden/make_fixtures.py), and the GPU test writes the fixture back as a MAT v5 file of the
same variables (K, rhs, n, nH, nJ, nZ) and runs the drivers on it, against the oracle."""
import importlib.util
import os

import numpy as np
import pytest
import scipy.io as sio
import scipy.sparse as sp

import fixtures as F
from oracle import oracle as O
from sensitivity import band

REF = "/root/reference/examples"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = {"cvxqp1_m": "cvxqp1_m_2x2_symm_iter10.mat", "cvxqp2_s": "cvxqp2_s_3x3_nonsymm_perm_iter10.mat"}
FLOOR, SAFETY = 1e-8, 10.0


def _fixture_mat(name, path):
    """The data fixture written back as a MAT v5 file with the reference file's variable names."""
    z = np.load(os.path.join(ROOT, "tests", "golden", f"{name}.npz"), allow_pickle=False)
    n, m = int(z["n"]), int(z["m"])
    K = sp.csr_matrix((z["K_data"], z["K_indices"], z["K_indptr"]), shape=(n + m, n + m))
    hdr = {k: float(z[f"hdr_{k}"]) for k in ("n", "nH", "nJ", "nZ")}
    sio.savemat(path, dict(K=K.tocsc(), rhs=z["rhs"].reshape(-1, 1), **hdr), format="5")
    return K, z["rhs"]


@pytest.mark.parametrize("name", sorted(FILES))
def test_load_mat_reads_the_reference_files(name):
    """load_mat on the reference's own data files = the committed fixtures, bit for bit."""
    import cpkrylov_amd as cpk
    path = os.path.join(REF, FILES[name])
    if not os.path.exists(path):
        pytest.skip("the reference is not in this container")
    d = cpk.load_mat(path)
    z = np.load(os.path.join(ROOT, "tests", "golden", f"{name}.npz"), allow_pickle=False)
    K = d["K"]
    assert sp.isspmatrix_csr(K) and K.dtype == np.float64
    assert np.array_equal(K.indptr, z["K_indptr"]) and np.array_equal(K.indices, z["K_indices"])
    assert np.array_equal(K.data, z["K_data"]) and np.array_equal(d["rhs"], z["rhs"])
    for k in ("n", "nH", "nJ", "nZ"):
        assert d[k] == int(z[f"hdr_{k}"]) and isinstance(d[k], int)


@pytest.mark.parametrize("name", sorted(FILES))
def test_load_mat_roundtrip_and_blocks(name, tmp_path):
    """A MAT v5 file written from the fixture reads back to the same arrays; saddle_blocks makes
    the example's cut (Q, A, C = -K22, G = diag(Q)) exactly as the fixtures' loader does."""
    import cpkrylov_amd as cpk
    p = str(tmp_path / FILES[name])
    K, rhs = _fixture_mat(name, p)
    d = cpk.load_mat(p)
    assert (d["K"] != K).nnz == 0 and np.array_equal(d["rhs"], rhs)
    n = d["nH"] if name == "cvxqp1_m" else d["nH"] + d["nZ"]
    Q, A, C, G = cpk.saddle_blocks(d["K"], n)
    P = F.load(name)
    for a, b in ((Q, P["Q"]), (A, P["B"]), (C, P["C"]), (G, P["G"])):
        assert a.shape == b.shape and (a != b).nnz == 0
    with pytest.raises(cpk.CpkError):
        cpk.saddle_blocks(d["K"], 0)


def _driver(prog):
    spec = importlib.util.spec_from_file_location(prog, os.path.join(ROOT, "examples", f"{prog}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.gpu
@pytest.mark.parametrize("prog,name,method", [("cpk_exprog1", "cvxqp1_m", "minres"), ("cpk_exprog1", "cvxqp1_m", "cg"),
                                              ("cpk_exprog1", "cvxqp1_m", "cglanczos"),
                                              ("cpk_exprog1", "cvxqp1_m", "dqgmres"),
                                              ("cpk_exprog2", "cvxqp2_s", "gmres"),
                                              ("cpk_exprog2", "cvxqp2_s", "dqgmres")])
def test_example_programs_match_oracle(gpu_ctx, prog, name, method, tmp_path, capsys):
    """Each example driver end to end on the GPU (its MAT file, the block cut, reg_cpkrylov, the
    direct-solve comparison, the three printed lines) against the oracle's reg_cpkrylov with the
    product's pivot order: niters and solved equal, histories and x within the sensitivity band,
    and the error against K \\ rhs no worse than the oracle's."""
    path = str(tmp_path / FILES[name])
    _fixture_mat(name, path)
    mod = _driver(prog)
    x, stats, flag, x_direct, relerr = mod.run(path, method, verbose=True)
    out = capsys.readouterr().out
    assert "2-norm relative error in the solution" in out and "iters = " in out and "time (prec setup" in out
    P = F.load(name)
    fname, _, extra = mod.METHODS[method]
    opts = dict(mod.OPTS, **extra)
    perm = stats["M"].export_factors()[2]
    xo, so = O.reg_cpkrylov(method, P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts, perm=perm)
    assert stats["niters"] == so["niters"] and flag["solved"] == so["solved"]
    bd = band(name, method, extra, perm)
    for k in [k for k in so if k.endswith("History")]:
        h0 = so[k][0]
        assert len(stats[k]) == len(so[k])
        assert np.max(np.abs(stats[k] - so[k])) / h0 <= max(FLOOR, SAFETY * bd[k]), k
    assert np.linalg.norm(x - xo) / np.linalg.norm(xo) <= max(FLOOR, SAFETY * bd["x"])
    err_o = float(np.linalg.norm(xo - x_direct) / np.linalg.norm(x_direct))
    assert relerr <= err_o + max(FLOOR, SAFETY * bd["x"]), (relerr, err_o)
