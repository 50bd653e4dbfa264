"""The host analysis is threaded (nested dissection, symbolic factor, schedule, relabelling, layout
transposes, distributed split) and must not depend on the thread count: every decision is made
from the data alone.  CPU only: the host half of opLDL2 (cpk_analyze) and
the distributed plan (cpk_analysis_plan) at 1, 3 and 8 threads, plus the parallel transpose and
the threaded symbolic factor against their serial loops (tools/micro, compiled here with g++)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import cpkrylov_amd as cpk
from cpkrylov_amd.synthetic import nonsym_system, saddle_system

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cpkrylov_amd", "csrc")


def _with_threads(t, fn):
    old = os.environ.get("CPK_THREADS")
    os.environ["CPK_THREADS"] = str(t)  # host_threads() reads it at every parallel region
    try:
        return fn()
    finally:
        if old is None:
            del os.environ["CPK_THREADS"]
        else:
            os.environ["CPK_THREADS"] = old


@pytest.mark.parametrize("kind", ["saddle", "nonsym"])
def test_analysis_and_plan_independent_of_thread_count(kind):
    S = saddle_system(300000) if kind == "saddle" else nonsym_system(N=200000)
    A = S["Q"]

    def run():
        H = cpk.api.analyze(S["G"], S["B"], -S["C"])
        pl = cpk.api.dist_plan(S["G"], S["B"], -S["C"], A, S["C"], 4, 1)
        return H, pl

    ref_H, ref_pl = _with_threads(8, run)
    for t in (1, 3):
        H, pl = _with_threads(t, run)
        for k in ("perm", "order", "round_ptr", "blk_lvl", "lvl_row", "D"):
            assert np.array_equal(H[k], ref_H[k]), (t, k)
        assert np.array_equal(H["L"].indptr, ref_H["L"].indptr) and np.array_equal(H["L"].indices, ref_H["L"].indices)
        assert np.array_equal(H["L"].data, ref_H["L"].data)
        for k, v in ref_pl.items():
            if isinstance(v, np.ndarray):
                assert np.array_equal(pl[k], v), (t, k)


def _build(tmp_path, name, srcs):
    exe = str(tmp_path / name)
    cmd = ["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", f"-I{CSRC}", f"-I{ROOT}/include",
           "-I/opt/rocm/include", os.path.join(ROOT, "tools", "micro", f"{name}.cpp")] + \
          [os.path.join(CSRC, s) for s in srcs] + ["-lpthread", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=240)
    return exe


def test_parallel_transpose_matches_serial(tmp_path):
    exe = _build(tmp_path, "transpose_check", ["hostsparse.cpp", "ordering.cpp"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "0 mismatches" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_threaded_symbolic_matches_serial(tmp_path, threads):
    exe = _build(tmp_path, "sym_check", ["factor.cpp", "ordering.cpp", "hostsparse.cpp"])
    S = saddle_system(200000)
    H = cpk.api.analyze(S["G"], S["B"], -S["C"])
    import scipy.sparse as sp
    Kp = sp.bmat([[S["G"], S["B"].T], [S["B"], -S["C"]]]).tocsr()
    Kp.sort_indices()
    d = tmp_path / "sys"
    d.mkdir()
    Kp.indptr.astype(np.int64).tofile(d / "ptr.bin")
    Kp.indices.astype(np.int32).tofile(d / "ind.bin")
    Kp.data.astype(np.float64).tofile(d / "val.bin")
    H["perm"].astype(np.int32).tofile(d / "perm.bin")
    env = dict(os.environ, CPK_THREADS=str(threads))
    r = subprocess.run([exe, str(d)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "identical" in r.stdout, r.stdout + r.stderr
