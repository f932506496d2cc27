#!/usr/bin/env python3
"""Do two one-sweep Arnoldi sweeps on two streams (two contexts on one GPU) overlap each
other's launch drains and reduce latencies?  Times F factors (n each, K steps) as one
decomposition on one stream against two decompositions of F/2 factors on two streams,
enqueued together (diagnostic for a factor-group-per-stream launch model).
usage: stream_probe.py F LOG2N"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tensorkrylov.jl_amd"))
import tkamd  # noqa: E402
from tkamd import _lib as L  # noqa: E402


def main():
    F, n, K = int(sys.argv[1]), 1 << int(sys.argv[2]), 50
    csc = tkamd.assemble_matrix(n, "Laplace")
    bs = [(lambda v: v / np.linalg.norm(v))(np.random.default_rng(1000 + s).random(n)) for s in range(F)]
    ca, cb = tkamd.Context(0), tkamd.Context(0)
    Aa, Ab = tkamd.DeviceMatrix(ca, csc), tkamd.DeviceMatrix(cb, csc)
    one = tkamd.DeviceDecomposition(ca, L.TK_ARNOLDI, F, 0, [Aa] * F, bs, K)
    h = F // 2
    da = tkamd.DeviceDecomposition(ca, L.TK_ARNOLDI, h, 0, [Aa] * h, bs[:h], K)
    db = tkamd.DeviceDecomposition(cb, L.TK_ARNOLDI, F - h, 0, [Ab] * (F - h), bs[h:], K)

    def run(devs, reps):
        for dv in devs:
            dv.init(False)
            dv.sweep(0, K)
            dv.flush(False)
        ca.sync()
        cb.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            for dv in devs:
                dv.init(False)
                dv.sweep(0, K)
                dv.flush(False)
        ca.sync()
        cb.sync()
        return (time.perf_counter() - t0) / reps

    for rep in range(2):
        t1 = run([one], 5)
        t2 = run([da, db], 5)
        ts = run([da], 5) + run([db], 5)
        print("F=%d n=2^%s: one stream %.3f ms, two streams together %.3f ms (%.3f x), the halves one after the other %.3f ms"
              % (F, sys.argv[2], 1e3 * t1, 1e3 * t2, t1 / t2, 1e3 * ts), flush=True)
    for x in (one, da, db, Aa, Ab):
        x.close()
    ca.close()
    cb.close()


if __name__ == "__main__":
    main()
