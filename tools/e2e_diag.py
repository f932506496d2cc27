import os, sys, time, json
import numpy as np
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tensorkrylov.jl_amd"))
import tkamd
ctx = tkamd.Context(0)
d, n, K = 4, 1 << 18, 50
csc = tkamd.assemble_matrix(n, "Laplace")
b = [np.random.default_rng(1000 + s).random(n) for s in range(d)]
b = [x / np.linalg.norm(x) for x in b]
A = tkamd.KroneckerMatrix("SymInstance", [csc] * d, "Laplace")
for mode in ("deferred", "rows", "deferred"):
    os.environ["TKHIP_GRAM"] = mode
    conv = tkamd.ConvergenceData(K)
    t0 = time.perf_counter()
    tkamd.tensorkrylov(conv, A, b, 1e-9, K, "TensorArnoldi", ctx=ctx)
    t1 = time.perf_counter()
    print(mode, "total %.4f" % (t1 - t0), {k: round(v, 5) for k, v in conv.timing.items()}, flush=True)
