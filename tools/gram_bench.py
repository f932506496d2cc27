#!/usr/bin/env python3
"""Time tk_decomp_gram (the MFMA SYRK of one factor's basis) at the C2 factor size, n = 2^20,
k = 50, on the library TKHIP_LIB points at (A/B of k_gram variants)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tensorkrylov.jl_amd"))
import tkamd  # noqa: E402
from tkamd import _lib as L  # noqa: E402

n, K = 1 << 20, 50
ctx = tkamd.Context(0)
A = tkamd.DeviceMatrix(ctx, tkamd.assemble_matrix(n, "Laplace"))
b = np.random.default_rng(1000).random(n)
dev = tkamd.DeviceDecomposition(ctx, L.TK_ARNOLDI, 1, 0, [A], [b / np.linalg.norm(b)], K)
dev.init(False)
dev.sweep(0, K)
dev.gram(0, K, want=False)
ctx.sync()
ctx.timing(1)
for _ in range(20):
    dev.gram(0, K, want=False)
ctx.sync()
ms, cnt = ctx.timing_read(L.T_GRAM)
us = 1e3 * ms / cnt
print("%s gram n=%d k=%d: %.1f us  %.2f TB/s" % (os.environ.get("TKHIP_LIB", "tree").split("/")[-1], n, K, us,
                                                  8.0 * n * K / (us * 1e-6) / 1e12))
dev.close()
A.close()
ctx.close()
