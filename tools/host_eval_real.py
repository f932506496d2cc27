#!/usr/bin/env python3
"""Host-only timing of the native iteration evaluation (tk_solver_evaluate) on the bench
configurations' REAL compressed data: records of a C4 / C1 / C2-shaped run produced by the
CPU stand-in device at the config's own n (the spectral scale of H_s sets the Pade scaling of
the nonsymmetric exponentials), exp-sum tables of the config.  Prints per-k times and the mean.
usage: python tools/host_eval_real.py C4|C1|C2 [d_cap]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tensorkrylov.jl_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import tkamd  # noqa: E402
import _fake_device as FD  # noqa: E402

CFG = {"C1": (4, 1 << 18, "Laplace", "SymInstance"), "C2": (8, 1 << 20, "Laplace", "SymInstance"),
       "C4": (10, 1 << 17, "ConvDiff", "NonSymInstance")}
cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
d, n, cls, inst = CFG[cfg]
K = 50
csc = tkamd.assemble_matrix(n, cls)
b = [np.random.default_rng(1000 + s).random(n) for s in range(d)]
b = [x / np.linalg.norm(x) for x in b]
A = tkamd.KroneckerMatrix(inst, [csc] * d, cls)
td = tkamd.TensorArnoldi(A, K, backend=FD.backend)
td.orthonormalize_first(b)
T = tkamd.compressed.IterationTables(A, K, 1e-9, d)
sv = tkamd.compressed.NativeSolver(td.method, d, K, inst == "SymInstance", kron := 1.0, T)
cache = os.path.join("/tmp", "host_eval_real_%s.npy" % cfg)
if os.path.exists(cache):
    recs = np.load(cache)
else:
    f = FD.FakeDecomposition(td, b)
    recs = np.stack([f.init()] + [f.step(j) for j in range(K)])
    np.save(cache, recs)
sv.apply(-1, recs[0])
for j in range(K):
    sv.apply(j, recs[j + 1])
tot, out = 0.0, []
for k in range(2, K + 1):
    best = 1e9
    for r in range(3):
        t0 = time.perf_counter()
        for i in range(3):
            try:
                sv.evaluate(k)
            except Exception:   # noqa: BLE001  (a breakdown still costs its evaluation)
                pass
        best = min(best, (time.perf_counter() - t0) / 3)
    tot += best
    if k in (2, 10, 20, 30, 40, 45, 50):
        out.append("k=%d %.0fus" % (k, best * 1e6))
print(cfg, "t=%d" % T.rank[K - 1], " ".join(out), "mean %.1f us per iteration (one thread)" % (1e6 * tot / (K - 1)))
