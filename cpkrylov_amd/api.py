"""Python host mirror of the cpkrylov interface, running on MI355X through libcpk.

Reference (MATLAB)                                   This module
-------------------------------------------------   ------------------------------------------
[x,stats,flag] = reg_cpkrylov(method,b,A,B,C,G,opts) x, stats, flag = reg_cpkrylov(method, b, A, B, C, G, opts)
   (reg_cpkrylov.m:1)
[x,y,stats,flag] = cpminres(b,A,C,M,opts)            x, y, stats, flag = cpminres(b, A, C, M, opts)
   (kernels/cpminres.m:1; same for cpcg, cpcglanczos, cpsymmlq, cpgmres, cpdqgmres)
M = opLDL2(A,B,C); M.nitref = 1; y = M*z            M = opLDL2(A, B, C); M.nitref = 1; y = M * z
   (ops/opLDL2.m:60, 45-50, 161)
[c,s,d] = SymGivens(a,b)  (util/SymGivens.m:1)       c, s, d = SymGivens(a, b)

`opts` is a dict whose keys behave like MATLAB struct fields (absent = solver default).
`stats` / `flag` are dicts with the reference's field names.  Matrices are scipy.sparse (or
dense numpy) arrays; `A` must be an explicit matrix (a generic linear operator A is not
supported on the device path).  Errors raise CpkError / IndefiniteError.
"""
import ctypes as C
import os

import numpy as np
import scipy.sparse as sp

from . import _lib
from ._lib import CpkError, IndefiniteError, check, lib, make_opts

_P = C.POINTER


def _dptr(a):
    return a.ctypes.data_as(_P(C.c_double))


class Context:
    """One GPU, one HIP stream (and an RCCL communicator when nranks > 1).

    timing_standin=True (diagnostic, cpk_ctx_create_null): rank `rank` of an nranks-way context
    whose collectives are no-ops -- one rank's share of the work, timed on one GPU; its results
    are meaningless."""

    def __init__(self, device=None, rank=0, nranks=1, unique_id=None, simgroup=None, options=None,
                 timing_standin=False):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        h = C.c_void_p()
        if simgroup is not None:  # ranks as threads on one GPU (tests), see cpk_ctx_create_sim
            check(lib.cpk_ctx_create_sim(device, simgroup.h, rank, nranks, C.byref(h)))
        elif timing_standin:
            check(lib.cpk_ctx_create_null(device, rank, nranks, C.byref(h)))
        else:
            uid = None
            if unique_id is not None:
                buf = (C.c_ubyte * 128).from_buffer_copy(bytes(unique_id))
                uid = C.cast(buf, _P(C.c_ubyte))
            check(lib.cpk_ctx_create(device, rank, nranks, uid, C.byref(h)))
        self.h = h
        self.device, self.rank, self.nranks = device, rank, nranks
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def set_option(self, name, value):
        """Engine option of this context (cpk_ctx_set_option); applies to objects created later."""
        if isinstance(value, bool):
            value = "1" if value else "0"
        check(lib.cpk_ctx_set_option(self.h, name.encode(), str(value).encode()))

    def get_option(self, name):
        """The value this context's objects use (sweep: the per-path default unless set)."""
        buf = C.create_string_buffer(256)
        check(lib.cpk_ctx_get_option(self.h, name.encode(), buf, 256))
        return buf.value.decode()

    def options_string(self):
        """Every engine option as "name=value;..." (cpk_ctx_get_options): analyze(options=...)
        and dist_plan(options=...) then plan exactly as this context's preconditioners."""
        buf = C.create_string_buffer(4096)
        check(lib.cpk_ctx_get_options(self.h, buf, 4096))
        return buf.value.decode()

    def info(self):
        """device, rank, nranks, the communicator's kind and rank count (RCCL: ncclCommCount),
        and whether preconditioners built here take the distributed path (cpk_ctx_get_info)."""
        v = (C.c_int64 * 8)()
        check(lib.cpk_ctx_get_info(self.h, v))
        return {"device": v[0], "rank": v[1], "nranks": v[2], "comm": _lib.COMM_KINDS.get(v[3], str(v[3])),
                "comm_ranks": v[4], "distributed": bool(v[5])}

    def synchronize(self):
        check(lib.cpk_ctx_synchronize(self.h))

    def close(self):
        if getattr(self, "h", None):
            lib.cpk_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SimGroup:
    """A group of `nranks` simulated ranks sharing one GPU (one thread per rank)."""

    def __init__(self, nranks):
        h = C.c_void_p()
        check(lib.cpk_simgroup_create(int(nranks), C.byref(h)))
        self.h, self.nranks = h, nranks

    def __del__(self):
        if getattr(self, "h", None):
            lib.cpk_simgroup_destroy(self.h)
            self.h = None


_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx


class engine_options:
    """Context manager: engine options of a context (default: the default context) for the
    duration of a block, restored afterwards -- e.g. `with engine_options(sweep="256,768,64"):`."""

    def __init__(self, ctx=None, **kw):
        self.ctx, self.kw, self.old = ctx, kw, {}

    def __enter__(self):
        self.ctx = self.ctx or default_context()
        for k, v in self.kw.items():
            self.old[k] = self.ctx.get_option(k)
            self.ctx.set_option(k, v)
        return self.ctx

    def __exit__(self, *exc):
        for k, v in self.old.items():
            self.ctx.set_option(k, v)
        return False


def get_unique_id():
    buf = (C.c_ubyte * 128)()
    check(lib.cpk_get_unique_id(buf))
    return bytes(buf)


class Matrix:
    """A sparse matrix handle (host copy + lazily uploaded HBM copy)."""

    def __init__(self, M, ctx=None, host_only=False, csc=False):
        """csc=True hands the matrix over as MATLAB stores it (mxGetJc / mxGetIr / mxGetPr:
        0-based, size_t column pointers and row indices), through cpk_mat_create_csc -- the
        entry the MEX gateway uses (matlab/cpk_mex.c)."""
        if isinstance(M, Matrix):
            raise TypeError("already a Matrix")
        if not sp.issparse(M):
            M = np.asarray(M, dtype=np.float64)
            if M.ndim != 2:
                raise CpkError(_lib.CPK_ERR_ARGS, "matrix expected")
            M = sp.csr_matrix(M)
        self.ctx = None if host_only else (ctx or default_context())
        h = C.c_void_p()
        cx = self.ctx.h if self.ctx else None
        if csc:
            M = sp.csc_matrix(M, dtype=np.float64)
            M.sum_duplicates()
            M.sort_indices()
            self.shape = M.shape
            self._ptr = np.ascontiguousarray(M.indptr, dtype=np.uintp)
            self._ind = np.ascontiguousarray(M.indices, dtype=np.uintp)
            self._val = np.ascontiguousarray(M.data, dtype=np.float64)
            check(lib.cpk_mat_create_csc(cx, M.shape[0], M.shape[1], self._ptr.ctypes.data_as(_P(C.c_size_t)),
                                         self._ind.ctypes.data_as(_P(C.c_size_t)), _dptr(self._val), C.byref(h)))
        else:
            M = sp.csr_matrix(M, dtype=np.float64)
            M.sum_duplicates()
            M.sort_indices()
            self.shape = M.shape
            self._ptr = np.ascontiguousarray(M.indptr, dtype=np.int64)
            self._ind = np.ascontiguousarray(M.indices, dtype=np.int32)
            self._val = np.ascontiguousarray(M.data, dtype=np.float64)
            check(lib.cpk_mat_create_csr(cx, M.shape[0], M.shape[1], self._ptr.ctypes.data_as(_P(C.c_int64)),
                                         self._ind.ctypes.data_as(_P(C.c_int32)), _dptr(self._val), C.byref(h)))
        self.h = h

    def __matmul__(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty(self.shape[0])
        check(lib.cpk_mat_spmv(self.h, _dptr(x), _dptr(y)))
        return y

    def __del__(self):
        if getattr(self, "h", None):
            lib.cpk_mat_destroy(self.h)
            self.h = None


def _as_matrix(M, ctx):
    if isinstance(M, Matrix):
        return M
    if isinstance(M, sp.linalg.LinearOperator):
        raise CpkError(_lib.CPK_ERR_UNSUPPORTED,
                       "A must be an explicit matrix on the device path (generic operators are out of scope)")
    return Matrix(M, ctx)


class opLDL2:
    """Operator for the inverse of [A B'; B C] via its LDL' factorization (ops/opLDL2.m).

    Public properties with the reference's setter semantics (opLDL2.m:45-50, 97-115):
      nitref          = max(0, round(val))          (default 3)
      itref_tol       stored as given (the reference's `sef.itref_tol` typo) (default 1e-8)
      force_itref     anything other than false/true becomes false (default false)
      residual_update stored as given (default false); a functional no-op, as in the reference
    """

    def __init__(self, A, B, Cm, ctx=None, _handle=None, krylov_A=None):
        """krylov_A (optional): the Krylov operator's A, a placement hint for a distributed
        context (cpk_pc_create_hint); ignored on one GPU."""
        self.ctx = ctx or default_context()
        if _handle is not None:
            self.h = _handle
        else:
            mats = [_as_matrix(M, self.ctx) for M in (A, B, Cm)]
            h = C.c_void_p()
            pt = C.c_double()
            if krylov_A is not None:
                ka = _as_matrix(krylov_A, self.ctx)
                check(lib.cpk_pc_create_hint(self.ctx.h, mats[0].h, mats[1].h, mats[2].h, ka.h, C.byref(pt),
                                             C.byref(h)))
            else:
                check(lib.cpk_pc_create(self.ctx.h, mats[0].h, mats[1].h, mats[2].h, C.byref(pt), C.byref(h)))
            self.h = h
            self.ptime = pt.value
        info = _lib.PcInfo()
        check(lib.cpk_pc_get_info(self.h, C.byref(info)))
        self.info = {k: getattr(info, k) for k, _ in _lib.PcInfo._fields_}
        self.nA, self.nC, self.n = info.n, info.m, info.N
        self.shape = (info.N, info.N)

    def refactor(self, A, B, Cm):
        """New values of (A, B, C) with the sparsity this operator was built with: the factors
        of opLDL2(A, B, C) recomputed on the device, symbolic analysis reused (cpk_pc_refactor;
        an IPM outer iteration's rebuild of opLDL2, opLDL2.m:60-92).  Returns the seconds taken."""
        mats = [_as_matrix(M, self.ctx) for M in (A, B, Cm)]
        pt = C.c_double()
        check(lib.cpk_pc_refactor(self.h, mats[0].h, mats[1].h, mats[2].h, C.byref(pt)))
        self.ptime = pt.value
        return pt.value

    # ---- properties --------------------------------------------------------------------------
    def _get(self):
        v = [C.c_double() for _ in range(4)]
        check(lib.cpk_pc_get(self.h, *[C.byref(x) for x in v]))
        return [x.value for x in v]

    def _set(self, **kw):
        check(lib.cpk_pc_set(self.h, C.byref(make_opts(kw))))

    nitref = property(lambda s: s._get()[0], lambda s, v: s._set(nitref=v))
    itref_tol = property(lambda s: s._get()[1], lambda s, v: s._set(itref_tol=v))
    force_itref = property(lambda s: bool(s._get()[2]), lambda s, v: s._set(force_itref=v))
    residual_update = property(lambda s: s._get()[3], lambda s, v: s._set(residual_update=v))

    @property
    def handle_semantics(self):
        """Opt-in (not in the reference): keep op.Aty / op.Cy between applies (cpk_pc_set_handle)."""
        return getattr(self, "_handle", False)

    @handle_semantics.setter
    def handle_semantics(self, on):
        check(lib.cpk_pc_set_handle(self.h, 1 if on else 0))
        self._handle = bool(on)

    # ---- operator surface --------------------------------------------------------------------
    def __mul__(self, z):
        z = np.ascontiguousarray(z, dtype=np.float64).ravel()
        if z.shape[0] != self.n:
            raise CpkError(_lib.CPK_ERR_DIM, "Dimensions do not match")
        y = np.empty(self.n)
        check(lib.cpk_pc_apply(self.h, _dptr(z), _dptr(y)))
        return y

    __matmul__ = __mul__

    def divide(self, b):
        """M \\ b = Kp*b  (opLDL2.divide, opLDL2.m:193-195)."""
        b = np.ascontiguousarray(b, dtype=np.float64).ravel()
        x = np.empty(self.n)
        check(lib.cpk_pc_divide(self.h, _dptr(b), _dptr(x)))
        return x

    def transpose(self):  # opLDL2.m:120-122
        return self

    T = property(transpose)
    ctranspose = transpose

    def to_dense(self):  # double(op), opLDL2.m:138-149
        e = np.zeros(self.n)
        X = np.zeros((self.n, self.n))
        for i in range(self.n):
            e[i] = 1
            X[:, i] = self * e
            e[i] = 0
        return X

    def sep_info(self):
        """Diagnostic: the distributed separator solve's staging (cpk_pc_sep_info)."""
        v = (C.c_int64 * 12)()
        check(lib.cpk_pc_sep_info(self.h, v))
        return dict(zip(("dist", "nT", "nlev", "nrec", "lds", "lds_g", "kt", "tkr", "sched", "fused", "tsweep",
                         "tsweep_rounds"), list(v)))

    def sweep_info(self):
        """Diagnostic: the sweep schedule as launched (cpk_pc_sweep_info)."""
        v = (C.c_int64 * 8)()
        check(lib.cpk_pc_sweep_info(self.h, v))
        return dict(zip(("rounds", "round0_blocks", "upper_blocks", "round0_assigned", "resid_assigned",
                         "bwd_assigned", "persistent", "chain_tasks"), list(v)))

    def local_dofs(self):
        """Global indices of this rank's local vector entries ([x-part; y-part]) and n_loc."""
        nl, ml = C.c_int64(), C.c_int64()
        check(lib.cpk_pc_local_dofs(self.h, C.byref(nl), C.byref(ml), None))
        d = np.empty(nl.value + ml.value, np.int32)
        check(lib.cpk_pc_local_dofs(self.h, C.byref(nl), C.byref(ml), d.ctypes.data_as(_P(C.c_int32))))
        return d, nl.value

    def export_factors(self):
        """(L (CSC, strict lower), D, perm) with P'*Kp*P = L*D*L', perm[k] = original index."""
        N, nnz = self.info["N"], self.info["nnz_l"]
        Lp = np.empty(N + 1, np.int64)
        Li = np.empty(max(nnz, 1), np.int32)
        Lx = np.empty(max(nnz, 1))
        D = np.empty(N)
        perm = np.empty(N, np.int32)
        check(lib.cpk_pc_export(self.h, Lp.ctypes.data_as(_P(C.c_int64)), Li.ctypes.data_as(_P(C.c_int32)),
                                _dptr(Lx), _dptr(D), perm.ctypes.data_as(_P(C.c_int32))))
        L = sp.csc_matrix((Lx[:nnz], Li[:nnz], Lp), shape=(N, N))
        return L, D, perm

    def __del__(self):
        if getattr(self, "h", None):
            lib.cpk_pc_destroy(self.h)
            self.h = None


def _options_spec(ctx, options):
    """The engine-option spec of cpk_analyze: a context's full set (so the analysis plans as that
    context's preconditioner would), then `options` (dict or "name=value;..." string) on top."""
    parts = []
    if ctx is not None:
        parts.append(ctx.options_string())
    if isinstance(options, dict):
        parts.append("".join(f"{k}={('1' if v else '0') if isinstance(v, bool) else v};" for k, v in options.items()))
    elif options:
        parts.append(str(options))
    return ";".join(p.strip(";") for p in parts if p).encode() if parts else None


def analyze(A, B, Cm, ctx=None, options=None):
    """Host-only half of opLDL2(A, B, C) (no GPU): ordering, LDL', sweep schedule.  Engine
    options: the CPK_* environment, then those of `ctx` (if given), then `options`."""
    mats = [M if isinstance(M, Matrix) else Matrix(M, host_only=True) for M in (A, B, Cm)]
    h = C.c_void_p()
    check(lib.cpk_analyze(mats[0].h, mats[1].h, mats[2].h, _options_spec(ctx, options), C.byref(h)))
    try:
        info = _lib.PcInfo()
        check(lib.cpk_analysis_get_info(h, C.byref(info)))
        info = {k: getattr(info, k) for k, _ in _lib.PcInfo._fields_}
        N, nnz = info["N"], info["nnz_l"]
        Lp = np.empty(N + 1, np.int64)
        Li = np.empty(max(nnz, 1), np.int32)
        Lx = np.empty(max(nnz, 1))
        D = np.empty(N)
        perm = np.empty(N, np.int32)
        check(lib.cpk_analysis_export(h, Lp.ctypes.data_as(_P(C.c_int64)), Li.ctypes.data_as(_P(C.c_int32)),
                                      _dptr(Lx), _dptr(D), perm.ctypes.data_as(_P(C.c_int32))))
        nl = C.c_int64()
        check(lib.cpk_analysis_schedule(h, C.byref(nl), None, None, None, None))
        rp = np.empty(info["nrounds"] + 1, np.int64)
        bl = np.empty(info["nblocks"] + 1, np.int64)
        lr = np.empty(nl.value + 1, np.int64)
        order = np.empty(N, np.int32)
        check(lib.cpk_analysis_schedule(h, None, rp.ctypes.data_as(_P(C.c_int64)), bl.ctypes.data_as(_P(C.c_int64)),
                                        lr.ctypes.data_as(_P(C.c_int64)), order.ctypes.data_as(_P(C.c_int32))))
    finally:
        lib.cpk_analysis_destroy(h)
    L = sp.csc_matrix((Lx[:nnz], Li[:nnz], Lp), shape=(N, N))
    return dict(info=info, L=L, D=D, perm=perm, round_ptr=rp, blk_lvl=bl, lvl_row=lr, order=order)


_PLAN_F64 = {"fsub_Lx", "fsub_D", "extra_val", "tf_val", "tb_val", "DT", "kp_val", "ac_val", "ab_val"}
_PLAN_NAMES = ("sizes", "dofs", "node_rank", "T", "fsub_Lp", "fsub_Li", "fsub_Lx", "fsub_D", "fsub_perm",
               "fsub_parent", "fsub_key", "extra_ptr", "extra_col", "extra_key", "extra_val", "tf_ptr", "tf_col",
               "tf_val", "tf_src", "tb_ptr", "tb_col", "tb_val", "DT", "tlev_ptr", "tlev_rows", "tsend", "tdof") + \
    tuple(f"{k}_{a}" for k in ("kp", "ac", "ab") for a in ("ptr", "col", "val", "send"))


def dist_plan(G, B, Cneg, A, Cop, nranks, rank, ctx=None, options=None):
    """Host-only row-block plan of `rank` for opLDL2(G, B, Cneg) and the
    Krylov operator blocks A, Cop: a dict of numpy arrays (see cpk_plan_array in cpk.h).  Engine
    options (split_tol) as in analyze(): pass the distributed context to get exactly the plan its
    preconditioner builds."""
    mats = [Matrix(M, host_only=True) for M in (G, B, Cneg, A, Cop)]
    h = C.c_void_p()
    check(lib.cpk_analyze(mats[0].h, mats[1].h, mats[2].h, _options_spec(ctx, options), C.byref(h)))
    p = C.c_void_p()
    try:
        check(lib.cpk_analysis_plan(h, mats[3].h, mats[4].h, int(nranks), int(rank), C.byref(p)))
    finally:
        lib.cpk_analysis_destroy(h)
    out = {}
    try:
        for nm in _PLAN_NAMES:
            cnt = C.c_int64()
            check(lib.cpk_plan_array(p, nm.encode(), C.byref(cnt), None))
            arr = np.empty(cnt.value, np.float64 if nm in _PLAN_F64 else np.int64)
            check(lib.cpk_plan_array(p, nm.encode(), C.byref(cnt), arr.ctypes.data_as(C.c_void_p)))
            out[nm] = arr
    finally:
        lib.cpk_plan_destroy(p)
    keys = ("P", "rank", "n", "m", "N", "n_loc", "m_loc", "N_loc", "nsub", "nT", "kt", "kp_kmax", "ac_kmax", "ab_kmax")
    out.update({k: int(v) for k, v in zip(keys, out["sizes"])})
    return out


# ---- solvers ----------------------------------------------------------------------------------
_STATUS = {0: "maximum number of iterations attained",
           1: "residual small compared to initial residual",
           2: "backward error small"}


def _hist_cap(method, opts, n, m):
    itmax = (opts or {}).get("itmax", n + m if method in ("gmres", "dqgmres") else n)
    itmax = int(min(max(itmax, 0), 1e8))
    if method == "gmres":
        r = int((opts or {}).get("restart", 50))
        itmax = -(-itmax // max(r, 1)) * max(r, 1)
    return itmax + 4


def _stats_from(method, st, hist, lq, qr):
    stats = {"niters": int(st.niters)}
    if method == "symmlq":
        stats["cgresidHistory"] = hist[:st.hist_len].copy()
        stats["lqresidHistory"] = lq[:st.lq_len].copy()
        stats["qrresidHistory"] = qr[:st.qr_len].copy()
    else:
        stats["residHistory"] = hist[:st.hist_len].copy()
    if method == "cglanczos":
        stats["status"] = _STATUS[st.status]
    stats["loop_ms"] = st.loop_ms
    stats["bytes_moved"] = st.bytes_moved
    return stats, {"solved": bool(st.solved)}


def _new_stats(cap):
    hist, lq, qr = np.zeros(cap), np.zeros(cap), np.zeros(cap)
    st = _lib.Stats()
    st.hist, st.hist_lq, st.hist_qr = _dptr(hist), _dptr(lq), _dptr(qr)
    st.hist_cap = cap
    return st, hist, lq, qr


def _method(name):
    def run(b, A, Cm, M, opts=None):
        if not isinstance(M, opLDL2):
            raise CpkError(_lib.CPK_ERR_ARGS, "M must be an opLDL2 operator")
        ctx = M.ctx
        Am, Cmat = _as_matrix(A, ctx), _as_matrix(Cm, ctx)
        n, m = Am.shape[0], Cmat.shape[0]
        b = np.ascontiguousarray(b, dtype=np.float64).ravel()
        if b.shape[0] != n:
            raise CpkError(_lib.CPK_ERR_DIM, "b must have n entries")
        x, y = np.zeros(n), np.zeros(m)
        st, hist, lq, qr = _new_stats(_hist_cap(name, opts, n, m))
        check(lib.cpk_method_solve(ctx.h, _lib.METHODS[name], _dptr(b), Am.h, Cmat.h, M.h,
                                   C.byref(make_opts(opts)), _dptr(x), _dptr(y), C.byref(st)))
        stats, flag = _stats_from(name, st, hist, lq, qr)
        return x, y, stats, flag

    run.__name__ = "cp" + name
    run._cpk_method = name
    run.__doc__ = f"[x, y, stats, flag] = cp{name}(b, A, C, M, opts)  (kernels/cp{name}.m)"
    return run


cpcg = _method("cg")
cpcglanczos = _method("cglanczos")
cpminres = _method("minres")
cpsymmlq = _method("symmlq")
cpgmres = _method("gmres")
cpdqgmres = _method("dqgmres")


def reg_cpkrylov(method, b, A, B, Cm, G, opts=None, ctx=None):
    """[x, stats, flag] = reg_cpkrylov(method, b, A, B, C, G, opts)   (reg_cpkrylov.m:1-180)."""
    if any(v is None for v in (method, b, A, B, Cm, G)):
        raise CpkError(_lib.CPK_ERR_ARGS, "reg_cpkrylov: not enough inputs")
    name = getattr(method, "_cpk_method", method)
    if name not in _lib.METHODS:
        raise CpkError(_lib.CPK_ERR_ARGS, f"unknown method {method!r}")
    ctx = ctx or default_context()
    mats = [_as_matrix(M, ctx) for M in (A, B, Cm, G)]
    n, m = mats[0].shape[0], mats[1].shape[0]
    b = np.ascontiguousarray(b, dtype=np.float64).ravel()
    if b.shape[0] != n + m:
        raise CpkError(_lib.CPK_ERR_DIM, "b must have n+m entries")
    x = np.zeros(n + m)
    st, hist, lq, qr = _new_stats(_hist_cap(name, opts, n, m))
    Mh = C.c_void_p()
    check(lib.cpk_reg_solve(ctx.h, _lib.METHODS[name], _dptr(b), mats[0].h, mats[1].h, mats[2].h, mats[3].h,
                            C.byref(make_opts(opts)), _dptr(x), C.byref(st), C.byref(Mh)))
    stats, flag = _stats_from(name, st, hist, lq, qr)
    stats["ptime"], stats["stime"] = st.ptime, st.stime
    if Mh:
        stats["M"] = opLDL2(None, None, None, ctx=ctx, _handle=Mh)
    return x, stats, flag


def SymGivens(a, b):
    """[c, s, d] = SymGivens(a, b)  (util/SymGivens.m)."""
    c, s, d = C.c_double(), C.c_double(), C.c_double()
    check(lib.cpk_symgivens(float(a), float(b), C.byref(c), C.byref(s), C.byref(d)))
    return c.value, s.value, d.value
