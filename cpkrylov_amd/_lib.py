"""ctypes binding of libcpk.so (include/cpk.h).

The library is built in-tree (``make -C cpkrylov_amd/csrc`` or ``__graft_entry__.build()``).
There is no fallback: if the shared library is missing, importing this module raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CPK_LIB_PATH") or os.path.join(_HERE, "libcpk.so")  # override: tools/ A/B runs

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libcpk.so not built ({LIB_PATH}); run `make -C cpkrylov_amd/csrc` "
                      "or __graft_entry__.build() -- there is no CPU fallback")

lib = C.CDLL(LIB_PATH)

CPK_OK, CPK_ERR_INDEFINITE, CPK_ERR_DIM, CPK_ERR_ARGS, CPK_ERR_HIP, CPK_ERR_RCCL, CPK_ERR_FACTOR, \
    CPK_ERR_NOMEM, CPK_ERR_UNSUPPORTED = range(9)
COMM_KINDS = {0: "none", 1: "rccl", 2: "sim", 3: "null"}  # CPK_COMM_* (cpk_ctx_get_info)
METHODS = {"cg": 0, "cglanczos": 1, "minres": 2, "symmlq": 3, "gmres": 4, "dqgmres": 5}
_OPT_FIELDS = ("atol", "rtol", "btol", "itmax", "restart", "mem", "print",
               "nitref", "itref_tol", "force_itref", "residual_update")


class Opts(C.Structure):
    _fields_ = [(k, C.c_double) for k in _OPT_FIELDS] + [("has_" + k, C.c_int) for k in _OPT_FIELDS]


class Stats(C.Structure):
    _fields_ = [("niters", C.c_int64), ("solved", C.c_int), ("status", C.c_int),
                ("hist", C.POINTER(C.c_double)), ("hist_lq", C.POINTER(C.c_double)),
                ("hist_qr", C.POINTER(C.c_double)), ("hist_cap", C.c_int64), ("hist_len", C.c_int64),
                ("lq_len", C.c_int64), ("qr_len", C.c_int64), ("ptime", C.c_double), ("stime", C.c_double),
                ("loop_ms", C.c_double), ("bytes_moved", C.c_double)]


class PcInfo(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("n", "m", "N", "nnz_kp", "nnz_l", "nblocks", "nrounds",
                                         "max_block_levels", "depth", "ordering")]


class Profile(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("spmv_ms", "spmv_bytes", "resid_ms", "resid_bytes", "fwd_ms", "fwd_bytes",
                                          "bwd_ms", "bwd_bytes", "apply_ms", "apply_bytes")] + \
               [("fwd_launches", C.c_int64), ("bwd_launches", C.c_int64)] + \
               [("fwd_resid_ms", C.c_double), ("fwd_resid_bytes", C.c_double), ("bwd_dead_store_bytes", C.c_double)]


P = C.POINTER
vp = C.c_void_p
_SIGS = {
    "cpk_last_error": ([], C.c_char_p),
    "cpk_abi_version": ([], C.c_int),
    "cpk_get_unique_id": ([P(C.c_ubyte)], C.c_int),
    "cpk_ctx_create": ([C.c_int, C.c_int, C.c_int, P(C.c_ubyte), P(vp)], C.c_int),
    "cpk_ctx_create_null": ([C.c_int, C.c_int, C.c_int, P(vp)], C.c_int),
    "cpk_ctx_get_info": ([vp, P(C.c_int64)], C.c_int),
    "cpk_ctx_get_options": ([vp, C.c_char_p, C.c_size_t], C.c_int),
    "cpk_ctx_destroy": ([vp], C.c_int),
    "cpk_ctx_synchronize": ([vp], C.c_int),
    "cpk_mat_create_csc": ([vp, C.c_int64, C.c_int64, P(C.c_size_t), P(C.c_size_t), P(C.c_double), P(vp)], C.c_int),
    "cpk_mat_create_csr": ([vp, C.c_int64, C.c_int64, P(C.c_int64), P(C.c_int32), P(C.c_double), P(vp)], C.c_int),
    "cpk_mat_destroy": ([vp], C.c_int),
    "cpk_mat_spmv": ([vp, P(C.c_double), P(C.c_double)], C.c_int),
    "cpk_pc_create": ([vp, vp, vp, vp, P(C.c_double), P(vp)], C.c_int),
    "cpk_pc_create_hint": ([vp, vp, vp, vp, vp, P(C.c_double), P(vp)], C.c_int),
    "cpk_pc_destroy": ([vp], C.c_int),
    "cpk_pc_refactor": ([vp, vp, vp, vp, P(C.c_double)], C.c_int),
    "cpk_pc_set": ([vp, P(Opts)], C.c_int),
    "cpk_pc_get": ([vp] + [P(C.c_double)] * 4, C.c_int),
    "cpk_pc_set_handle": ([vp, C.c_int], C.c_int),
    "cpk_pc_apply": ([vp, P(C.c_double), P(C.c_double)], C.c_int),
    "cpk_pc_apply_device": ([vp, vp, vp], C.c_int),
    "cpk_pc_divide": ([vp, P(C.c_double), P(C.c_double)], C.c_int),
    "cpk_pc_get_info": ([vp, P(PcInfo)], C.c_int),
    "cpk_pc_export": ([vp, P(C.c_int64), P(C.c_int32), P(C.c_double), P(C.c_double), P(C.c_int32)], C.c_int),
    "cpk_analyze": ([vp, vp, vp, C.c_char_p, P(vp)], C.c_int),
    "cpk_analysis_destroy": ([vp], C.c_int),
    "cpk_analysis_get_info": ([vp, P(PcInfo)], C.c_int),
    "cpk_analysis_export": ([vp, P(C.c_int64), P(C.c_int32), P(C.c_double), P(C.c_double), P(C.c_int32)],
                            C.c_int),
    "cpk_analysis_schedule": ([vp, P(C.c_int64), P(C.c_int64), P(C.c_int64), P(C.c_int64), P(C.c_int32)], C.c_int),
    "cpk_analysis_plan": ([vp, vp, vp, C.c_int, C.c_int, P(vp)], C.c_int),
    "cpk_plan_array": ([vp, C.c_char_p, P(C.c_int64), vp], C.c_int),
    "cpk_plan_destroy": ([vp], C.c_int),
    "cpk_simgroup_create": ([C.c_int, P(vp)], C.c_int),
    "cpk_simgroup_destroy": ([vp], C.c_int),
    "cpk_ctx_create_sim": ([C.c_int, vp, C.c_int, C.c_int, P(vp)], C.c_int),
    "cpk_pc_local_dofs": ([vp, P(C.c_int64), P(C.c_int64), P(C.c_int32)], C.c_int),
    "cpk_pc_sep_info": ([vp, P(C.c_int64)], C.c_int),
    "cpk_method_solve": ([vp, C.c_int, P(C.c_double), vp, vp, vp, P(Opts), P(C.c_double), P(C.c_double),
                          P(Stats)], C.c_int),
    "cpk_method_solve_device": ([vp, C.c_int, vp, vp, vp, vp, P(Opts), vp, P(Stats)], C.c_int),
    "cpk_reg_solve": ([vp, C.c_int, P(C.c_double), vp, vp, vp, vp, P(Opts), P(C.c_double), P(Stats), P(vp)],
                      C.c_int),
    "cpk_reg_solve_device": ([vp, C.c_int, vp, vp, vp, vp, vp, P(Opts), vp, P(Stats)], C.c_int),
    "cpk_reg_shift_device": ([vp, vp, vp, vp, vp, vp, vp, vp, P(C.c_int)], C.c_int),
    "cpk_profile_kernels": ([vp, vp, vp, vp, C.c_int, P(Profile)], C.c_int),
    "cpk_debug_pipe_stamps": ([P(C.c_uint64), C.c_int, P(C.c_int)], C.c_int),
    "cpk_debug_blk_cycles": ([P(C.c_uint64), C.c_int64, P(C.c_int64)], C.c_int),
    "cpk_debug_block_model": ([vp, P(C.c_int64), C.c_int64, P(C.c_int64)], C.c_int),
    "cpk_debug_pass_times": ([vp, P(C.c_double)], C.c_int),
    "cpk_ctx_set_option": ([C.c_void_p, C.c_char_p, C.c_char_p], C.c_int),
    "cpk_pc_sweep_info": ([C.c_void_p, P(C.c_int64)], C.c_int),
    "cpk_ctx_get_option": ([C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t], C.c_int),
    "cpk_symgivens": ([C.c_double, C.c_double, P(C.c_double), P(C.c_double), P(C.c_double)], C.c_int),
}
for _name, (_args, _res) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.argtypes = _args
    _f.restype = _res

EXPORTED = tuple(_SIGS)


class CpkError(RuntimeError):
    """An error returned by libcpk (MATLAB `error(...)` in the reference)."""

    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code
        self.identifier = None


class IndefiniteError(CpkError):
    """beta < -100*eps (the reference's `error(...)` / MException('CPCGLanczos:IndefiniteError'))."""


def check(rc):
    if rc != CPK_OK:
        msg = lib.cpk_last_error().decode()
        cls = IndefiniteError if rc == CPK_ERR_INDEFINITE else CpkError
        e = cls(rc, msg)
        if msg.startswith("CPCGLanczos:IndefiniteError"):
            e.identifier = "CPCGLanczos:IndefiniteError"
        raise e


def make_opts(opts):
    o = Opts()
    for k, v in (opts or {}).items():
        if k == "reorth":  # accepted and ignored (cpgmres.m:104,118-120: not implemented)
            continue
        if k not in _OPT_FIELDS:
            continue  # MATLAB ignores unknown struct fields
        setattr(o, k, float(v))
        setattr(o, "has_" + k, 1)
    return o
