"""ctypes wrapper of oracle/tk_ref.c -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/ and by bench.py's cpu_baseline leg (never by the product).
The shared object is built by __graft_entry__.build_oracle() into oracle/_build/.
"""
import ctypes
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libtkref.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            import subprocess
            import sys
            sys.path.insert(0, os.path.dirname(_HERE))
            import __graft_entry__
            __graft_entry__.build_oracle()
        L = ctypes.CDLL(_SO)
        D = ctypes.POINTER(ctypes.c_double)
        I64 = ctypes.POINTER(ctypes.c_int64)
        L.tkref_matvec.argtypes = [ctypes.c_int64, I64, I64, D, D, D]
        L.tkref_init.argtypes = [ctypes.c_int64, D, D]
        L.tkref_arnoldi_step.argtypes = [ctypes.c_int64, I64, I64, D, D, ctypes.c_int64, D,
                                         ctypes.c_int64, ctypes.c_int, D]
        L.tkref_lanczos_step.argtypes = [ctypes.c_int64, I64, I64, D, D, ctypes.c_int64, ctypes.c_int,
                                         ctypes.c_double, D, D, D]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _i(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


class RefFactor:
    """One factor's Arnoldi/Lanczos state in the C oracle; V is Fortran-ordered so
    V[:, j] is contiguous like Julia's column-major storage."""

    def __init__(self, csc, b, kmax):
        self.colptr = np.ascontiguousarray(csc[0], dtype=np.int64)
        self.rowval = np.ascontiguousarray(csc[1], dtype=np.int64)
        self.nz = np.ascontiguousarray(csc[2], dtype=np.float64)
        self.n = len(self.colptr) - 1
        self.V = np.zeros((self.n, kmax + 1), order="F")
        self.H = np.zeros((kmax + 2, kmax + 1), order="F")
        self.w = np.zeros(self.n)
        b = np.ascontiguousarray(b, dtype=np.float64)
        lib().tkref_init(self.n, _d(b), _d(self.V))
        self.beta = 0.0

    def matvec(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.n)
        lib().tkref_matvec(self.n, _i(self.colptr), _i(self.rowval), _d(self.nz), _d(x), _d(y))
        return y

    def arnoldi_step(self, j):
        lib().tkref_arnoldi_step(self.n, _i(self.colptr), _i(self.rowval), _d(self.nz), _d(self.V),
                                 self.n, _d(self.H), self.H.shape[0], int(j), _d(self.w))

    def lanczos_step(self, j):
        a = ctypes.c_double()
        bt = ctypes.c_double()
        lib().tkref_lanczos_step(self.n, _i(self.colptr), _i(self.rowval), _d(self.nz), _d(self.V),
                                 self.n, int(j), self.beta, _d(self.w), ctypes.byref(a), ctypes.byref(bt))
        self.H[j, j] = a.value
        self.H[j + 1, j] = bt.value
        self.H[j, j + 1] = bt.value
        self.beta = bt.value
        return a.value, bt.value


def baseline(csc, n, d, K, seconds=15.0):
    """CPU baseline for bench.py: the C restatement's full K-step Arnoldi (MGS2) sweep,
    1 thread, on the benchmark's factors (b_s ~ U(0,1), seed 1000+s, as on the GPU) one
    after another -- cycling through them again if time is left -- until about `seconds`
    of CPU work; the mean sweep time times d is the time of one K-iteration solve."""
    sweeps = []
    s = 0
    t_start = time.perf_counter()
    while True:
        rng = np.random.default_rng(1000 + (s % d))
        b = rng.random(n)
        b /= np.linalg.norm(b)
        f = RefFactor(csc, b, K)
        t0 = time.perf_counter()
        for j in range(K):
            f.arnoldi_step(j)
        sweeps.append(time.perf_counter() - t0)
        del f
        s += 1
        if time.perf_counter() - t_start >= seconds or s >= 4 * d:
            break
    per_iter = d * float(np.mean(sweeps)) / K
    return {"value": round(1.0 / per_iter, 4), "unit": "iterations/s", "cores": 1, "kind": "port",
            "sample": "oracle/tk_ref.c MGS2 Arnoldi, full K=%d sweeps of %d factor(s) of the workload "
                      "(n=%d; d=%d), %.1f s of CPU work, mean sweep x d" % (K, len(sweeps), n, d,
                                                                         float(np.sum(sweeps)))}
