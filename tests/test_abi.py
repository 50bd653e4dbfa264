"""The C-ABI library loads and exports every symbol include/cpk.h declares (no GPU calls)."""
import os
import re

import cpkrylov_amd as cpk
from cpkrylov_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "cpk.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(cpk_\w+)\s*\(", src, re.M)))


def test_every_declared_symbol_is_exported():
    names = declared()
    assert len(names) >= 25
    for n in names:
        assert hasattr(_lib.lib, n), n
    assert set(names) == set(_lib.EXPORTED)


def test_abi_version():
    assert _lib.lib.cpk_abi_version() == 3


def test_symgivens_host_entry():
    assert cpk.SymGivens(3.0, 4.0) == (0.6000000000000001, 0.8, 5.0)
    assert cpk.SymGivens(0.0, -2.0) == (0.0, -1.0, 2.0)


def test_no_silent_fallback_without_gpu():
    """On a host without a GPU the device entry points fail loudly."""
    import torch
    if torch.cuda.is_available():
        return
    try:
        cpk.Context(device=0)
    except cpk.CpkError as e:
        assert e.code == _lib.CPK_ERR_HIP
    else:
        raise AssertionError("context creation must fail without a GPU")


def test_multi_rank_context_needs_unique_id():
    """cpk_ctx_create refuses nranks > 1 without an RCCL unique id (checked before any device
    call): there is no environment switch to a peer-less communicator any more; the timing
    stand-in has its own constructor (cpk_ctx_create_null), which refuses nranks == 1."""
    import ctypes as C
    h = C.c_void_p()
    assert _lib.lib.cpk_ctx_create(0, 0, 2, None, C.byref(h)) == _lib.CPK_ERR_ARGS
    assert b"unique_id" in _lib.lib.cpk_last_error()
    assert _lib.lib.cpk_ctx_create_null(0, 0, 1, C.byref(h)) == _lib.CPK_ERR_ARGS
