#!/usr/bin/env python3
"""Host-only timing of the native iteration evaluation (tk_solver_evaluate: compressed solve
+ residual + orthogonality) at the C2 shape d = 8, K = 50 on this machine's CPU, with records
from the CPU stand-in device (n = 200: the k-sized work does not depend on n).
usage: python tools/host_eval_bench.py [tol] [C2|C4]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tensorkrylov.jl_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import tkamd  # noqa: E402
import _fake_device as FD  # noqa: E402

tol = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-9
cfg = sys.argv[2] if len(sys.argv) > 2 else "C2"
d, n, K = (8, 200, 50) if cfg == "C2" else (10, 200, 50)
cls, inst = ("Laplace", "SymInstance") if cfg == "C2" else ("ConvDiff", "NonSymInstance")
csc = tkamd.assemble_matrix(n, cls)
b = [np.random.default_rng(1000 + s).random(n) for s in range(d)]
b = [x / np.linalg.norm(x) for x in b]
A = tkamd.KroneckerMatrix(inst, [csc] * d, cls)
td = tkamd.TensorArnoldi(A, K, backend=FD.backend)
td.orthonormalize_first(b)
T = tkamd.compressed.IterationTables(A, K, tol, d)
sv = tkamd.compressed.NativeSolver(td.method, d, K, inst == "SymInstance", 1.0, T)
f = FD.FakeDecomposition(td, b)
sv.apply(-1, f.init())
for j in range(K):
    sv.apply(j, f.step(j))
tot = 0.0
for k in range(2, K + 1):
    best = 1e9
    for r in range(3):
        t0 = time.perf_counter()
        for i in range(20):
            sv.evaluate(k)
        best = min(best, (time.perf_counter() - t0) / 20)
    tot += best
    if k in (2, 10, 20, 30, 40, 50):
        print("k=%d t=%d evaluate %.1f us" % (k, T.rank[k - 1], best * 1e6))
print("mean over k=2..%d: %.1f us per iteration (one thread)" % (K, 1e6 * tot / (K - 1)))
