"""The MEX gateway (matlab/cpk_mex.c, SURVEY.md 8b / 8f-4: "MATLAB host code calls HIP through a
thin MEX/C-ABI layer") compiled against a stand-in of the mx API (tests/mex_shim/: MATLAB's array,
error and clean-up rules, plus leak counters) and driven like MATLAB would drive it:

  h = cpk_mex('pc_create', G, B, Cneg); cpk_mex('pc_set', h, opts); y = cpk_mex('pc_apply', h, x)
  [x, y, stats, flag] = cpk_mex('method', @cpminres, b, A, C, h, opts)
  [x, stats, flag] = cpk_mex('reg_solve', @cpgmres, b, A, B, C, G, opts)

(reg_cpkrylov.m:131,163; ops/opLDL2.m:97-115,161-188).  The GPU tests compare with the oracle:
the apply bit for bit given the same factors, the solves bit for bit in exact mode (the gateway's
context is made with CPK_EXACT_DOTS=1).  Every error path -- wrong arguments, a dimension
mismatch, an indefinite preconditioner (CPCGLanczos:IndefiniteError), an unknown method -- must
leave no device matrix, no mxArray and no mxCalloc block behind.  The CPU tests cover the paths
that need no device (argument errors, and a context that cannot be created).
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest
import scipy.sparse as sp

import fixtures as F
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "tests", "mex_shim")
SO = os.path.join(SHIM, "_build", "libcpkmex.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            subprocess.run(["make", "-s", "-C", SHIM], check=True)
        L = C.CDLL(SO)
        vp, sz = C.c_void_p, C.c_size_t
        L.shim_dense.restype = vp
        L.shim_dense.argtypes = [sz, sz, C.POINTER(C.c_double)]
        L.shim_sparse.restype = vp
        L.shim_sparse.argtypes = [sz, sz, C.POINTER(sz), C.POINTER(sz), C.POINTER(C.c_double)]
        for f in ("shim_char", "shim_funchandle"):
            getattr(L, f).restype = vp
            getattr(L, f).argtypes = [C.c_char_p]
        L.shim_scalar.restype = vp
        L.shim_scalar.argtypes = [C.c_double]
        L.shim_struct.restype = vp
        L.shim_struct.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(vp)]
        L.shim_field.restype = vp
        L.shim_field.argtypes = [vp, C.c_char_p]
        L.shim_class.argtypes = [vp]
        L.shim_u64.restype = C.c_uint64
        L.shim_u64.argtypes = [vp]
        L.shim_logical.argtypes = [vp]
        L.shim_destroy.argtypes = [vp]
        L.shim_call.argtypes = [C.c_int, C.POINTER(vp), C.c_int, C.POINTER(vp)]
        L.shim_error_id.restype = C.c_char_p
        L.shim_error_msg.restype = C.c_char_p
        for f in ("shim_live_arrays", "shim_live_calloc", "shim_live_mats", "shim_live_pcs"):
            getattr(L, f).restype = C.c_long
        L.mxGetM.restype = L.mxGetN.restype = sz
        L.mxGetM.argtypes = L.mxGetN.argtypes = [vp]
        L.mxGetPr.restype = C.POINTER(C.c_double)
        L.mxGetPr.argtypes = [vp]
        _lib = L
    return _lib


class MexError(RuntimeError):
    def __init__(self, ident, msg):
        super().__init__(f"{ident}: {msg}")
        self.ident, self.msg = ident, msg


class Mex:
    """MATLAB's side of cpk_mex: converts Python values to mxArrays, calls, converts back, and
    destroys the inputs afterwards (they belong to the caller, as in MATLAB)."""

    def __init__(self):
        self.L = lib()

    def arr(self, v):
        L = self.L
        if isinstance(v, str):
            return L.shim_char(v.encode())
        if isinstance(v, Func):
            return L.shim_funchandle(v.text.encode())
        if isinstance(v, Handle):
            return v.a
        if isinstance(v, dict):
            names = (C.c_char_p * len(v))(*[k.encode() for k in v])
            vals = (C.c_void_p * len(v))(*[self.arr(x) for x in v.values()])
            return L.shim_struct(len(v), names, vals)
        if sp.issparse(v):
            M = sp.csc_matrix(v)
            M.sort_indices()
            self._keep = [np.ascontiguousarray(M.indptr, np.uint64), np.ascontiguousarray(M.indices, np.uint64),
                          np.ascontiguousarray(M.data, np.float64)]
            jc, ir, pr = self._keep
            return L.shim_sparse(M.shape[0], M.shape[1], jc.ctypes.data_as(C.POINTER(C.c_size_t)),
                                 ir.ctypes.data_as(C.POINTER(C.c_size_t)), pr.ctypes.data_as(C.POINTER(C.c_double)))
        if isinstance(v, (int, float, bool, np.floating)):
            return L.shim_scalar(float(v))
        a = np.ascontiguousarray(np.asarray(v, np.float64).reshape(-1))
        return L.shim_dense(a.shape[0], 1, a.ctypes.data_as(C.POINTER(C.c_double)))

    def value(self, a):
        L = self.L
        cls = L.shim_class(a)
        if cls == 5:  # mxUINT64_CLASS: a preconditioner handle (owned by the caller)
            return Handle(a, L.shim_u64(a))
        if cls == 2:
            return bool(L.shim_logical(a))
        if cls == 1:
            return a  # struct: read with field()
        m, n = L.mxGetM(a), L.mxGetN(a)
        return np.ctypeslib.as_array(L.mxGetPr(a), shape=(m * n,)).copy() if m * n else np.zeros(0)

    def field(self, s, name):
        return self.value(self.L.shim_field(s, name.encode()))

    def __call__(self, nlhs, *args):
        L = self.L
        ins = [self.arr(a) for a in args]
        prhs = (C.c_void_p * max(len(ins), 1))(*ins)
        plhs = (C.c_void_p * max(nlhs, 1))()
        rc = L.shim_call(nlhs, plhs, len(ins), prhs)
        for a, v in zip(ins, args):
            if not isinstance(v, Handle):
                L.shim_destroy(a)
        if rc:
            raise MexError(L.shim_error_id().decode(), L.shim_error_msg().decode())
        return [plhs[i] for i in range(nlhs)]

    def live(self):
        L = self.L
        return dict(arrays=L.shim_live_arrays(), calloc=L.shim_live_calloc(), mats=L.shim_live_mats(),
                    pcs=L.shim_live_pcs())


class Func:
    """a function handle; text = what func2str returns for it"""

    def __init__(self, text):
        self.text = text


class Handle:
    def __init__(self, a, value):
        self.a, self.value = a, value


def _expect_error(mex, ident, *args, nlhs=1):
    before = mex.live()
    with pytest.raises(MexError) as e:
        mex(nlhs, *args)
    assert e.value.ident == ident, (e.value.ident, e.value.msg)
    assert mex.live() == before, (mex.live(), before)  # nothing left behind
    return e.value


# ---- CPU: the argument checks and a context that cannot be made (no GPU here) -----------------
def test_mex_argument_errors_leave_nothing():
    mex = Mex()
    P = F.load("cvxqp2_s")
    _expect_error(mex, "cpk:args")  # no command
    _expect_error(mex, "cpk:args", "no_such_command")
    _expect_error(mex, "cpk:args", "pc_create", np.ones(3), P["B"], -P["C"])  # dense, not sparse
    _expect_error(mex, "cpk:args", "pc_create", P["G"])  # missing arguments
    _expect_error(mex, "cpk:args", "pc_apply", 1.0, np.ones(3))  # not a handle
    _expect_error(mex, "cpk:args", "method", Func("@cpnothing"), np.ones(3), P["Q"], P["C"], 1.0, nlhs=4)
    _expect_error(mex, "cpk:args", "method", 3.0, np.ones(3), P["Q"], P["C"], 1.0, nlhs=4)
    assert mex.live()["mats"] == 0 and mex.live()["calloc"] == 0


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present: covered by the GPU tests")
def test_mex_context_failure_frees_temporaries():
    """without a device the context cannot be made: the error surfaces as cpk:error, and the
    matrices converted before it are not leaked"""
    mex = Mex()
    P = F.load("cvxqp2_s")
    e = _expect_error(mex, "cpk:error", "pc_create", P["G"], P["B"], -P["C"])
    assert e.msg


# ---- GPU: the gateway end to end ----------------------------------------------------------------
_MEX = {}


def _gpu_mex():
    """the gateway with its context made in exact mode (the first libcpk call of the process
    through it creates the context from the CPK_* environment)"""
    if "m" not in _MEX:
        mex = Mex()
        P = F.load("cvxqp2_s")
        old = os.environ.get("CPK_EXACT_DOTS")
        os.environ["CPK_EXACT_DOTS"] = "1"
        try:
            h = mex.value(mex(1, "pc_create", P["G"], P["B"], -P["C"])[0])
        finally:
            if old is None:
                del os.environ["CPK_EXACT_DOTS"]
            else:
                os.environ["CPK_EXACT_DOTS"] = old
        mex(0, "pc_destroy", h)
        mex.L.shim_destroy(h.a)
        _MEX["m"] = mex
    return _MEX["m"]


def _factors(P):
    """the product's factors of opLDL2(G, B, -C) (deterministic: what the gateway's handle holds)"""
    import cpkrylov_amd as cpk
    M = cpk.opLDL2(P["G"], P["B"], -P["C"])
    return M.export_factors()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cvxqp1_m", "cvxqp2_s"])
def test_mex_pc_apply_bitexact(name):
    mex = _gpu_mex()
    P = F.load(name)
    live0 = mex.live()
    h = mex.value(mex(1, "pc_create", P["G"], P["B"], -P["C"])[0])
    assert mex.live()["mats"] == 0 and mex.live()["pcs"] == live0["pcs"] + 1
    mex(0, "pc_set", h, dict(nitref=1, force_itref=1, itref_tol=1e-8, residual_update=1))
    z = np.random.default_rng(7).standard_normal(P["n"] + P["m"])
    y = mex.value(mex(1, "pc_apply", h, z)[0])
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=_factors(P))
    Mo.set(nitref=1.0, force_itref=1.0, itref_tol=1e-8)
    assert np.array_equal(y, Mo @ z)
    # Kp * b (opLDL2.divide)
    Kp = sp.bmat([[P["G"], P["B"].T], [P["B"], -P["C"]]]).tocsr()
    xd = mex.value(mex(1, "pc_divide", h, z)[0])
    assert np.allclose(xd, Kp @ z, rtol=1e-13, atol=1e-13 * np.abs(Kp @ z).max())
    # a length mismatch, then the handle is still good
    _expect_error(mex, "cpk:dim", "pc_apply", h, z[:-1])
    assert np.array_equal(mex.value(mex(1, "pc_apply", h, z)[0]), y)
    mex(0, "pc_destroy", h)
    mex.L.shim_destroy(h.a)
    assert mex.live()["pcs"] == live0["pcs"]


@pytest.mark.gpu
@pytest.mark.parametrize("func", ["cpminres", "@cpminres", "pkg.cpminres"])
def test_mex_method_matches_oracle(func):
    """[x, y, stats, flag] = cpk_mex('method', @cpminres, b, A, C, h, opts) on cvxqp1_m (the
    method call of reg_cpkrylov.m:163 with a GPU preconditioner), bit for bit the oracle's exact
    mode; func2str's text forms all name the same method"""
    mex = _gpu_mex()
    P = F.load("cvxqp1_m")
    opts = dict(atol=1e-6, rtol=1e-6, itmax=500)
    h = mex.value(mex(1, "pc_create", P["G"], P["B"], -P["C"])[0])
    mex(0, "pc_set", h, dict(nitref=1, force_itref=1, itref_tol=1e-8))
    b = np.random.default_rng(3).standard_normal(P["n"])
    out = mex(4, "method", Func(func), b, P["Q"], P["C"], h, opts)
    x, y = mex.value(out[0]), mex.value(out[1])
    stats, flag = out[2], out[3]
    hist = mex.field(stats, "residHistory")
    niters = mex.field(stats, "niters")[0]
    solved = mex.field(flag, "solved")
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=_factors(P))
    Mo.set(nitref=1.0, force_itref=1.0, itref_tol=1e-8)
    with O.exact():
        xo, yo, so = O.method("minres", b, P["Q"], P["C"], Mo, opts)
    assert niters == so["niters"] and solved == so["solved"]
    assert np.array_equal(hist, so["residHistory"])
    assert np.array_equal(x, xo) and np.array_equal(y, yo)
    for a in out:
        mex.L.shim_destroy(a)
    mex(0, "pc_destroy", h)
    mex.L.shim_destroy(h.a)
    live = mex.live()
    assert live["mats"] == 0 and live["calloc"] == 0 and live["pcs"] == 0


@pytest.mark.gpu
def test_mex_reg_solve_matches_oracle():
    """[x, stats, flag] = cpk_mex('reg_solve', @cpgmres, b, A, B, C, G, opts) on cvxqp2_s with
    the exprog2 options (restart 20), bit for bit the oracle's reg_cpkrylov in exact mode"""
    mex = _gpu_mex()
    P = F.load("cvxqp2_s")
    opts = dict(F.EXPROG_OPTS, restart=20)
    opts.pop("print")
    out = mex(3, "reg_solve", Func("cpgmres"), P["rhs"], P["Q"], P["B"], P["C"], P["G"], opts)
    x, stats, flag = mex.value(out[0]), out[1], out[2]
    Mo = O.LDL2(P["G"], P["B"], -P["C"], factors=_factors(P))
    Mo.set(**{k: float(opts[k]) for k in ("nitref", "itref_tol", "force_itref", "residual_update")})
    with O.exact():
        xo, so = O.reg_solve("gmres", P["rhs"], P["Q"], P["B"], P["C"], Mo, opts)
    assert mex.field(stats, "niters")[0] == so["niters"]
    assert mex.field(flag, "solved") == so["solved"]
    assert np.array_equal(mex.field(stats, "residHistory"), so["residHistory"])
    assert np.array_equal(x, xo)
    for a in out:
        mex.L.shim_destroy(a)
    assert mex.live()["mats"] == 0 and mex.live()["calloc"] == 0


@pytest.mark.gpu
def test_mex_error_paths_leave_nothing():
    mex = _gpu_mex()
    P = F.load("cvxqp1_m")
    Q2 = F.load("cvxqp2_s")
    # opLDL2.m:61-75: B's columns must match G
    e = _expect_error(mex, "cpk:error", "pc_create", P["G"], Q2["B"], -P["C"])
    assert "imension" in e.msg or "ncompatible" in e.msg, e.msg
    # a right-hand side of the wrong length
    _expect_error(mex, "cpk:dim", "reg_solve", Func("cpminres"), P["rhs"][:-1], P["Q"], P["B"], P["C"], P["G"],
                  dict(itmax=5), nlhs=3)
    # an unknown method after the matrices would have been made
    _expect_error(mex, "cpk:args", "reg_solve", Func("@cpnothing"), P["rhs"], P["Q"], P["B"], P["C"], P["G"],
                  dict(itmax=5), nlhs=3)
    # an indefinite preconditioner: G = -diag(Q) makes <u, M u> negative (cpcglanczos.m:156-160)
    e = _expect_error(mex, "CPCGLanczos:IndefiniteError", "reg_solve", Func("cpcglanczos"), P["rhs"], P["Q"],
                      P["B"], P["C"], -P["G"], dict(itmax=50), nlhs=3)
    assert "beta" in e.msg
    live = mex.live()
    assert live["mats"] == 0 and live["calloc"] == 0 and live["pcs"] == 0
