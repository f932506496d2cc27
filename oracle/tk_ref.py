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
        L.tkref_arnoldi_sweep_omp.argtypes = [ctypes.c_int64, I64, I64, D, D, ctypes.c_int64, D,
                                              ctypes.c_int64, ctypes.c_int, D, ctypes.c_int, D]
        L.tkref_max_threads.restype = ctypes.c_int
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


class CFactor:
    """tk_oracle.Factor's interface (1-based k, V, H) over RefFactor, so that
    tk_oracle.tensorkrylov(..., factor=CFactor) steps its factors in the C restatement:
    the MGS2 step of src/orthogonal_bases.jl:15-37 and the TTR step of :39-67 in the
    reference's operation order, compiled (the full-size n = 2^20 driver tests)."""

    def __init__(self, csc, b, kmax):
        self._f = RefFactor(csc, b, kmax)
        self.V = self._f.V                 # n x (kmax+1), column-major
        self.H = self._f.H                 # (kmax+2) x (kmax+1)

    def arnoldi_mgs(self, k):
        self._f.arnoldi_step(k - 1)

    def lanczos_ttr(self, k):
        self._f.lanczos_step(k - 1)

    def lanczos_reorth(self, k, force=None):
        raise NotImplementedError("LanczosReorth: use tk_oracle.Factor")


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


def csc_to_csr(csc):
    """Row-major copy of a CSC matrix with every row's columns ascending (the order the CSC
    scatter adds them in)."""
    colptr, rowval, nz = (np.asarray(a) for a in csc)
    n = len(colptr) - 1
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(colptr))
    order = np.lexsort((cols, rowval))
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(rowval, minlength=n), out=rowptr[1:])
    return rowptr, np.ascontiguousarray(cols[order]), np.ascontiguousarray(nz[order], dtype=np.float64)


def arnoldi_sweep_omp(csr, b, K, threads=None, V=None, H=None):
    """K-step MGS2 sweep with rows split over `threads` OpenMP threads (all-cores baseline);
    returns V (n x K+1, Fortran order) and H ((K+2) x (K+1))."""
    L = lib()
    rowptr, colind, val = csr
    n = len(rowptr) - 1
    threads = threads or L.tkref_max_threads()
    if V is None:
        V = np.zeros((n, K + 1), order="F")
    if H is None:
        H = np.zeros((K + 2, K + 1), order="F")
    b = np.ascontiguousarray(b, dtype=np.float64)
    L.tkref_init(n, _d(b), _d(V))
    w = np.zeros(n)
    part = np.zeros(2 * 8 * threads)
    L.tkref_arnoldi_sweep_omp(n, _i(rowptr), _i(colind), _d(val), _d(V), n, _d(H), H.shape[0], int(K),
                              _d(w), int(threads), _d(part))
    return V, H


def cpu_info():
    """Host CPU model and the core count visible to this process."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": avail}


def baseline_all_cores(csc, n, d, K, seconds=10.0, threads=None):
    """All-cores CPU baseline: the MGS2 sweep with rows over OpenMP threads (threads =
    OMP_NUM_THREADS / the OpenMP default), same factors and sampling rule as baseline()."""
    threads = threads or lib().tkref_max_threads()
    csr = csc_to_csr(csc)
    V = np.zeros((n, K + 1), order="F")
    H = np.zeros((K + 2, K + 1), order="F")
    sweeps = []
    s = 0
    t_start = time.perf_counter()
    while True:
        rng = np.random.default_rng(1000 + (s % d))
        b = rng.random(n)
        b /= np.linalg.norm(b)
        t0 = time.perf_counter()
        arnoldi_sweep_omp(csr, b, K, threads, V, H)
        sweeps.append(time.perf_counter() - t0)
        s += 1
        if time.perf_counter() - t_start >= seconds or s >= 4 * d:
            break
    per_iter = d * float(np.mean(sweeps)) / K
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"value": round(1.0 / per_iter, 4), "unit": "iterations/s", "cores": int(threads), "kind": "port",
            "sample": "oracle/tk_ref.c MGS2 Arnoldi, rows over %d OpenMP threads, full K=%d sweeps of %d "
                      "factor(s) of the workload (n=%d; d=%d), %.1f s, mean sweep x d"
                      % (threads, K, len(sweeps), n, d, float(np.sum(sweeps))),
            # the thread count is the process's CPU share, not the machine: the GPU box sets
            # OMP_NUM_THREADS (16 per GPU) although the host shows all of its CPUs
            "cores_cap": ("OMP_NUM_THREADS=%s: the CPU share given to this job; the host has %s CPUs "
                          "(not all used)" % (omp, os.cpu_count())) if omp else None}
