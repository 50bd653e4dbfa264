"""cpkrylov_amd -- MI355X-native constraint-preconditioned Krylov solvers (HIP/CDNA4).

Drop-in for the hot path of optimizers/cpkrylov: reg_cpkrylov + cp{cg,cglanczos,minres,
symmlq,gmres,dqgmres} + the opLDL2 preconditioner operator.  See DESIGN.md.
"""
from ._lib import CpkError, IndefiniteError, LIB_PATH  # noqa: F401  (raises if libcpk.so is missing)
from .api import (Context, Matrix, SimGroup, SymGivens, analyze, dist_plan, cpcg, cpcglanczos, cpdqgmres, cpgmres,  # noqa: F401
                  cpminres, cpsymmlq, default_context, engine_options, get_unique_id, opLDL2, reg_cpkrylov)
from .matio import load_mat, saddle_blocks  # noqa: F401

__all__ = ["reg_cpkrylov", "cpcg", "cpcglanczos", "cpminres", "cpsymmlq", "cpgmres", "cpdqgmres", "opLDL2",
           "SymGivens", "Context", "Matrix", "analyze", "CpkError", "IndefiniteError", "get_unique_id",
           "engine_options", "load_mat", "saddle_blocks"]
