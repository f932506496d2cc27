#!/usr/bin/env python3
"""Profile the end-to-end tkamd.tensorkrylov loop (device steps + host compressed side)
on a bench configuration: cProfile top entries and the wall time per iteration.
usage: python tools/e2e_profile.py [C2] [pipelined:1|0]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorkrylov.jl_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import tkamd  # noqa: E402
from bench import CONFIGS  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
pipe = (sys.argv[2] if len(sys.argv) > 2 else "1") == "1"
d, n, cls, method, K, inst = CONFIGS[cfg]
ctx = tkamd.Context(0)
csc = tkamd.assemble_matrix(n, cls)
b = [np.random.default_rng(1000 + s).random(n) for s in range(d)]
b = [x / np.linalg.norm(x) for x in b]
A = tkamd.KroneckerMatrix(inst, [csc] * d, cls)
for rep in range(2):
    conv = tkamd.ConvergenceData(K)
    pr = cProfile.Profile()
    pr.enable()
    t0 = time.perf_counter()
    tkamd.tensorkrylov(conv, A, b, 1e-9, K, method, ctx=ctx, pipelined=pipe)
    el = time.perf_counter() - t0
    pr.disable()
    print("rep %d: %d iterations, %.3f s, %.3f ms/iteration" % (rep, conv.niterations, el, 1e3 * el / conv.niterations))
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
ctx.close()
