"""Writes Kp and the product's pivot order for a system to a directory and runs sym_check
(threaded symbolic LDL' vs the serial loop).  Usage: sym_check.py <system> [N]"""
import os
import subprocess
import sys
import tempfile

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cpkrylov_amd as cpk  # noqa: E402

name = sys.argv[1]
if name.startswith("syn"):
    from cpkrylov_amd.synthetic import nonsym_system, saddle_system
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    S = (nonsym_system if "nonsym" in name else saddle_system)(N=N)
    G, B, C = S["G"], S["B"], S["C"]
else:
    import fixtures as F
    P = F.load(name)
    G, B, C = P["G"], P["B"], P["C"]
H = cpk.analyze(G, B, -C)
Kp = sp.bmat([[G, B.T], [B, -C]]).tocsr()
Kp.sort_indices()
with tempfile.TemporaryDirectory() as d:
    Kp.indptr.astype(np.int64).tofile(os.path.join(d, "ptr.bin"))
    Kp.indices.astype(np.int32).tofile(os.path.join(d, "ind.bin"))
    Kp.data.astype(np.float64).tofile(os.path.join(d, "val.bin"))
    H["perm"].astype(np.int32).tofile(os.path.join(d, "perm.bin"))
    sys.exit(subprocess.run([os.path.join(ROOT, "build", "sym_check"), d]).returncode)
