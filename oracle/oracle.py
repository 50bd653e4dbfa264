"""ctypes front end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It is the checker, never the thing measured or shipped.  See cpk_oracle.h for the scope
and the parity status (pinned by the reference's K\\rhs known answers; MATLAB itself is
unavailable, so iterate-level parity with MATLAB is unpinned).
"""
import ctypes as C
import os
import subprocess

import numpy as np
import scipy.sparse as sp

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libcpk_oracle.so")

METHODS = {"cg": 0, "cglanczos": 1, "minres": 2, "symmlq": 3, "gmres": 4, "dqgmres": 5}
ORDER = {"natural": 0, "given": 1, "rcm": 2}
STATUS = {0: "maximum number of iterations attained",
          1: "residual small compared to initial residual",
          2: "backward error small"}


class _Csr(C.Structure):
    _fields_ = [("nrows", C.c_int64), ("ncols", C.c_int64), ("ptr", C.POINTER(C.c_int64)),
                ("ind", C.POINTER(C.c_int32)), ("val", C.POINTER(C.c_double))]


class _Opts(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("atol", "rtol", "btol", "itmax", "restart", "mem", "print",
                                          "nitref", "itref_tol", "force_itref", "residual_update")] + \
               [("has_" + k, C.c_int) for k in ("atol", "rtol", "btol", "itmax", "restart", "mem", "print",
                                                "nitref", "itref_tol", "force_itref", "residual_update")]


class _Stats(C.Structure):
    _fields_ = [("niters", C.c_int64), ("solved", C.c_int), ("status", C.c_int),
                ("hist", C.POINTER(C.c_double)), ("hist_lq", C.POINTER(C.c_double)),
                ("hist_qr", C.POINTER(C.c_double)), ("hist_cap", C.c_int64), ("hist_len", C.c_int64),
                ("lq_len", C.c_int64), ("qr_len", C.c_int64), ("ptime", C.c_double), ("stime", C.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        P = C.POINTER
        L.orc_ldl2_create.argtypes = [P(_Csr), P(_Csr), P(_Csr), C.c_int, P(C.c_int32), P(C.c_void_p)]
        L.orc_ldl2_create_from_factors.argtypes = [P(_Csr), P(_Csr), P(_Csr), P(C.c_int64), P(C.c_int32),
                                                   P(C.c_double), P(C.c_double), P(C.c_int32), P(C.c_void_p)]
        L.orc_ldl2_destroy.argtypes = [C.c_void_p]
        for nm in ("nitref", "itref_tol", "force_itref", "residual_update", "handle"):
            f = getattr(L, "orc_ldl2_set_" + nm)
            f.argtypes = [C.c_void_p, C.c_double]
        L.orc_ldl2_get_props.argtypes = [C.c_void_p] + [P(C.c_double)] * 4
        L.orc_ldl2_apply.argtypes = [C.c_void_p, P(C.c_double), P(C.c_double)]
        L.orc_ldl2_nnzL.argtypes = [C.c_void_p]
        L.orc_ldl2_nnzL.restype = C.c_int64
        L.orc_ldl2_get_perm.argtypes = [C.c_void_p, P(C.c_int32)]
        L.orc_ldl2_export.argtypes = [C.c_void_p, P(C.c_int64), P(C.c_int32), P(C.c_double), P(C.c_double)]
        L.orc_method.argtypes = [C.c_int, P(C.c_double), P(_Csr), P(_Csr), C.c_void_p, P(_Opts),
                                 P(C.c_double), P(C.c_double), P(_Stats)]
        L.orc_reg_cpkrylov.argtypes = [C.c_int, P(C.c_double), P(_Csr), P(_Csr), P(_Csr), P(_Csr), P(_Opts),
                                       C.c_int, P(C.c_int32), P(C.c_double), P(_Stats), P(C.c_void_p)]
        L.orc_reg_solve.argtypes = [C.c_int, P(C.c_double), P(_Csr), P(_Csr), P(_Csr), C.c_void_p, P(_Opts),
                                    P(C.c_double), P(_Stats)]
        L.orc_symgivens.argtypes = [C.c_double, C.c_double] + [P(C.c_double)] * 3
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_set_exact.argtypes = [C.c_int]
        L.orc_get_exact.restype = C.c_int
        L.orc_xdot.argtypes = [C.c_int64, P(C.c_double), P(C.c_double)]
        L.orc_xdot.restype = C.c_double
        L.orc_xnorm2.argtypes = [C.c_double, C.c_double]
        L.orc_xnorm2.restype = C.c_double
        L.orc_get_threads.restype = C.c_int
        L.orc_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def _ptr(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class _CsrHold:
    """Keeps the numpy arrays of a CSR alive while C holds pointers into them."""

    def __init__(self, M):
        M = sp.csr_matrix(M)
        M.sum_duplicates()
        M.sort_indices()
        self.ptr = np.ascontiguousarray(M.indptr, dtype=np.int64)
        self.ind = np.ascontiguousarray(M.indices, dtype=np.int32)
        self.val = np.ascontiguousarray(M.data, dtype=np.float64)
        self.s = _Csr(M.shape[0], M.shape[1], _ptr(self.ptr, C.c_int64), _ptr(self.ind, C.c_int32),
                      _ptr(self.val, C.c_double))


def _opts(opts):
    o = _Opts()
    for k, v in (opts or {}).items():
        if k == "reorth":  # accepted and ignored, as cpgmres.m:118-120
            continue
        setattr(o, k, float(v))
        setattr(o, "has_" + k, 1)
    return o


def _check(rc):
    if rc != 0:
        raise OracleError(rc, lib().orc_last_error().decode())


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code
        self.msg = msg


class LDL2:
    """opLDL2(A, B, C): Kp = [A B'; B C], M*z solves Kp v = z (ops/opLDL2.m)."""

    def __init__(self, A, B, Cm, order="rcm", perm=None, factors=None):
        self._h = [_CsrHold(A), _CsrHold(B), _CsrHold(Cm)]
        self.n, self.m = A.shape[0], Cm.shape[0]
        h = C.c_void_p()
        if factors is not None:
            Lcsc, D, perm = factors
            Lcsc = sp.csc_matrix(Lcsc)
            Lcsc.sort_indices()
            self._f = (np.ascontiguousarray(Lcsc.indptr, np.int64), np.ascontiguousarray(Lcsc.indices, np.int32),
                       np.ascontiguousarray(Lcsc.data, np.float64), np.ascontiguousarray(D, np.float64),
                       np.ascontiguousarray(perm, np.int32))
            _check(lib().orc_ldl2_create_from_factors(
                C.byref(self._h[0].s), C.byref(self._h[1].s), C.byref(self._h[2].s),
                _ptr(self._f[0], C.c_int64), _ptr(self._f[1], C.c_int32), _ptr(self._f[2], C.c_double),
                _ptr(self._f[3], C.c_double), _ptr(self._f[4], C.c_int32), C.byref(h)))
        else:
            pp = None
            if perm is not None:
                self._perm = np.ascontiguousarray(perm, np.int32)
                pp = _ptr(self._perm, C.c_int32)
                order = "given"
            _check(lib().orc_ldl2_create(C.byref(self._h[0].s), C.byref(self._h[1].s), C.byref(self._h[2].s),
                                         ORDER[order], pp, C.byref(h)))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_ldl2_destroy(self.h)
            self.h = None

    def set(self, **kw):
        for k, v in kw.items():
            getattr(lib(), "orc_ldl2_set_" + k)(self.h, float(v))

    def set_handle(self, on):
        """Opt-in handle semantics of op.Aty / op.Cy (orc_ldl2_set_handle); clears the state."""
        lib().orc_ldl2_set_handle(self.h, C.c_double(1.0 if on else 0.0))

    def props(self):
        v = [C.c_double() for _ in range(4)]
        lib().orc_ldl2_get_props(self.h, *[C.byref(x) for x in v])
        return dict(zip(("nitref", "itref_tol", "force_itref", "residual_update"), [x.value for x in v]))

    def __matmul__(self, z):
        z = np.ascontiguousarray(z, dtype=np.float64)
        y = np.empty_like(z)
        _check(lib().orc_ldl2_apply(self.h, _ptr(z, C.c_double), _ptr(y, C.c_double)))
        return y

    __mul__ = __matmul__

    def nnzL(self):
        return lib().orc_ldl2_nnzL(self.h)

    def factors(self):
        """(L strict lower CSC, D, perm) of the oracle's own factorization."""
        N = self.n + self.m
        nnz = int(self.nnzL())
        Lp = np.empty(N + 1, np.int64)
        Li = np.empty(max(nnz, 1), np.int32)
        Lx = np.empty(max(nnz, 1))
        D = np.empty(N)
        lib().orc_ldl2_export(self.h, _ptr(Lp, C.c_int64), _ptr(Li, C.c_int32), _ptr(Lx, C.c_double),
                              _ptr(D, C.c_double))
        return sp.csc_matrix((Lx[:nnz], Li[:nnz], Lp), shape=(N, N)), D, self.perm()

    def perm(self):
        p = np.empty(self.n + self.m, np.int32)
        lib().orc_ldl2_get_perm(self.h, _ptr(p, C.c_int32))
        return p


def _run(fn, method, hist_cap, *args):
    hist = np.zeros(hist_cap)
    lq = np.zeros(hist_cap)
    qr = np.zeros(hist_cap)
    st = _Stats()
    st.hist, st.hist_lq, st.hist_qr = _ptr(hist, C.c_double), _ptr(lq, C.c_double), _ptr(qr, C.c_double)
    st.hist_cap = hist_cap
    _check(fn(METHODS[method], *args, C.byref(st)))
    stats = {"niters": st.niters, "solved": bool(st.solved)}
    if method == "symmlq":
        stats["cgresidHistory"] = hist[:st.hist_len].copy()
        stats["lqresidHistory"] = lq[:st.lq_len].copy()
        stats["qrresidHistory"] = qr[:st.qr_len].copy()
    else:
        stats["residHistory"] = hist[:st.hist_len].copy()
    if method == "cglanczos":
        stats["status"] = STATUS[st.status]
    return stats, st


def method(name, b, A, Cm, M, opts=None, hist_cap=None):
    """[x, y, stats, flag] = cp<name>(b, A, C, M, opts)"""
    n, m = A.shape[0], Cm.shape[0]
    b = np.ascontiguousarray(b, np.float64)
    hA, hC = _CsrHold(A), _CsrHold(Cm)
    o = _opts(opts)
    x, y = np.zeros(n), np.zeros(m)
    cap = hist_cap or int((opts or {}).get("itmax", n + m)) + 3
    stats, _ = _run(lambda mid, *rest: lib().orc_method(mid, _ptr(b, C.c_double), C.byref(hA.s), C.byref(hC.s),
                                                        M.h, C.byref(o), *rest),
                    name, cap, _ptr(x, C.c_double), _ptr(y, C.c_double))
    return x, y, stats


def reg_cpkrylov(name, b, A, B, Cm, G, opts=None, order="rcm", perm=None, hist_cap=None):
    """[x, stats, flag] = reg_cpkrylov(@cp<name>, b, A, B, C, G, opts)"""
    n, m = A.shape[0], B.shape[0]
    b = np.ascontiguousarray(b, np.float64)
    hs = [_CsrHold(M) for M in (A, B, Cm, G)]
    o = _opts(opts)
    x = np.zeros(n + m)
    pp = None
    if perm is not None:
        perm = np.ascontiguousarray(perm, np.int32)
        pp = _ptr(perm, C.c_int32)
        order = "given"
    cap = hist_cap or int((opts or {}).get("itmax", n + m)) + 3
    stats, st = _run(lambda mid, xp, stp: lib().orc_reg_cpkrylov(
        mid, _ptr(b, C.c_double), *[C.byref(h.s) for h in hs], C.byref(o), ORDER[order], pp, xp, stp, None),
        name, cap, _ptr(x, C.c_double))
    stats["ptime"], stats["stime"] = st.ptime, st.stime
    return x, stats


def reg_solve(name, b, A, B, Cm, M, opts=None, hist_cap=None):
    """reg_cpkrylov's shift + method + recovery with an existing preconditioner M (an LDL2, e.g.
    built from the product's exported factors) -- x (N), stats"""
    n, m = A.shape[0], B.shape[0]
    b = np.ascontiguousarray(b, np.float64)
    hs = [_CsrHold(X) for X in (A, B, Cm)]
    o = _opts(opts)
    x = np.zeros(n + m)
    cap = hist_cap or int((opts or {}).get("itmax", n + m)) + 3
    stats, st = _run(lambda mid, xp, stp: lib().orc_reg_solve(
        mid, _ptr(b, C.c_double), *[C.byref(h.s) for h in hs], M.h, C.byref(o), xp, stp),
        name, cap, _ptr(x, C.c_double))
    return x, stats


def set_threads(t):
    """Threads of the CPU-baseline timing leg (1 = the serial restatement); returns the count
    actually in effect (1 when the oracle was built without OpenMP)."""
    lib().orc_set_threads(int(t))
    return lib().orc_get_threads()


def set_exact(on):
    """Exact inner products (orc_set_exact): every dot / norm the correctly rounded exact sum of
    its TwoProd pairs, norm([a b]) the shared double-double formula -- the values of the
    product's engine option exact_dots.  Returns the previous setting."""
    prev = bool(lib().orc_get_exact())
    lib().orc_set_exact(1 if on else 0)
    return prev


class exact:
    """with oracle.exact(): ... -- exact inner products inside the block"""

    def __init__(self, on=True):
        self.on = on

    def __enter__(self):
        self.prev = set_exact(self.on)
        return self

    def __exit__(self, *exc):
        set_exact(self.prev)


def xdot(a, b):
    """One exact-mode inner product (the correctly rounded sum of the TwoProd pairs)."""
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    return lib().orc_xdot(a.shape[0], _ptr(a, C.c_double), _ptr(b, C.c_double))


def xnorm2(a, b):
    """The exact mode's norm([a b])."""
    return lib().orc_xnorm2(float(a), float(b))


def symgivens(a, b):
    c, s, d = C.c_double(), C.c_double(), C.c_double()
    lib().orc_symgivens(a, b, C.byref(c), C.byref(s), C.byref(d))
    return c.value, s.value, d.value
