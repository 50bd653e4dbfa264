"""Every `<file>.m:N` / `<file>.m:N-M` citation in the product, oracle, tests and docs points at
lines that exist in the cited reference file.  The file lengths are recorded here as data (the
reference is not present on the GPU box); when /root/reference is present they are checked too."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

# line counts of the reference's MATLAB sources (lines, the last one unterminated counted)
LENGTHS = {
    "SymGivens.m": 29, "opLDL2.m": 199, "reg_cpkrylov.m": 180, "cpdqgmres.m": 282, "cpminres.m": 254,
    "cpsymmlq.m": 369, "cpcg.m": 195, "cpgmres.m": 271, "cpcglanczos.m": 326, "cpk_exprog2.m": 117,
    "cpk_exprog1.m": 118, "cpk_path_setup.m": 11,
}

SCAN_DIRS = ("cpkrylov_amd", "oracle", "include", "tests", "matlab", "tools")
SCAN_FILES = ("DESIGN.md", "INTEGRATION.md", "README.md", "bench.py", "__graft_entry__.py")
EXTS = (".py", ".c", ".h", ".cpp", ".hpp", ".hip", ".md", ".m")
# `file.m:12-34,56` and the continuation form `file.m:12, 56-60`
CITE = re.compile(r"([A-Za-z0-9_]+\.m):(\d+(?:-\d+)?(?:\s*,\s*\d+(?:-\d+)?)*)")


def _files():
    for d in SCAN_DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            if "__pycache__" in dp or "_build" in dp:
                continue
            for f in fs:
                if f.endswith(EXTS) and f != "test_citations.py":
                    yield os.path.join(dp, f)
    for f in SCAN_FILES:
        p = os.path.join(ROOT, f)
        if os.path.exists(p):
            yield p


def _citations():
    out = []
    for path in _files():
        with open(path, errors="replace") as fh:
            for ln, line in enumerate(fh, 1):
                for m in CITE.finditer(line):
                    fname = m.group(1)
                    for part in m.group(2).split(","):
                        part = part.strip()
                        lo, _, hi = part.partition("-")
                        out.append((os.path.relpath(path, ROOT), ln, fname, int(lo), int(hi or lo)))
    return out


def test_lengths_match_reference():
    if not os.path.isdir(REF):
        pytest.skip("reference not present")
    for dp, _, fs in os.walk(REF):
        for f in fs:
            if f.endswith(".m"):
                with open(os.path.join(dp, f), errors="replace") as fh:
                    n = sum(1 for _ in fh)
                assert LENGTHS.get(f) == n, (f, n)


def test_citations_in_range():
    cites = _citations()
    assert len(cites) > 100  # the scan finds the citations
    bad = [c for c in cites if c[2] in LENGTHS and not (1 <= c[3] <= c[4] <= LENGTHS[c[2]])]
    unknown = sorted({c[2] for c in cites if c[2] not in LENGTHS})
    assert not bad, "\n".join(f"{p}:{ln}: {f}:{a}-{b} (file has {LENGTHS[f]} lines)" for p, ln, f, a, b in bad)
    assert not unknown, unknown
