"""Device objects owning libtkhip handles: context, coefficient matrix, decomposition.

These wrap include/tk.h one to one; the Julia glue (julia/TensorKrylovHIP.jl) binds
the same entry points with ccall.
"""
import ctypes

import numpy as np

from . import _lib as L


class Context:
    """tk_ctx: one HIP device + one stream (+ optional RCCL communicator)."""

    def __init__(self, device=0):
        self._lib = L.lib()
        h = ctypes.c_void_p()
        L.check(self._lib.tk_ctx_create(int(device), ctypes.byref(h)))
        self.h = h
        self.device = device
        self.nranks = 1
        self.rank = 0

    def sync(self):
        L.check(self._lib.tk_ctx_sync(self.h))

    def init_comm(self, uid, nranks, rank):
        assert len(uid) == 128
        L.check(self._lib.tk_comm_init(self.h, uid, int(nranks), int(rank)))
        self.nranks, self.rank = nranks, rank

    def init_comm_test(self, key, nranks, rank):
        """Test build only (tests/_build/libtkhip_test.so, loaded through TKHIP_LIB): join an
        nranks-wide job of processes sharing ONE GPU through the shared-memory stand-in for
        RCCL (tk_comm_init_test) -- RCCL refuses several ranks on one device."""
        fn = getattr(self._lib, "tk_comm_init_test", None)
        if fn is None:
            raise L.TKError("tk_comm_init_test: %s is not the test build" % L.LIB_PATH)
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.check(fn(self.h, key.encode(), int(nranks), int(rank)))
        self.nranks, self.rank = nranks, rank

    def allreduce_host(self, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        L.check(self._lib.tk_comm_allreduce_host(self.h, L.dptr(arr), arr.size))
        return arr

    def comm_count(self):
        """Ranks of the communicator as RCCL reports them (ncclCommCount); 0 without one."""
        n = ctypes.c_int()
        L.check(self._lib.tk_comm_count(self.h, ctypes.byref(n)))
        return n.value

    def timing(self, level):
        L.check(self._lib.tk_timing_enable(self.h, int(level)))

    def timing_read(self, cls):
        ms = ctypes.c_double()
        cnt = ctypes.c_long()
        L.check(self._lib.tk_timing_read(self.h, int(cls), ctypes.byref(ms), ctypes.byref(cnt)))
        return ms.value, cnt.value

    def close(self):
        if getattr(self, "h", None):
            self._lib.tk_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def unique_id():
    buf = ctypes.create_string_buffer(128)
    L.check(L.lib().tk_comm_unique_id(buf))
    return buf.raw


class DeviceMatrix:
    """tk_mat: A_s on the device as CSR (from Julia-style CSC)."""

    def __init__(self, ctx, csc, one_based=False):
        colptr, rowval, nzval = (np.ascontiguousarray(csc[0], dtype=np.int64),
                                 np.ascontiguousarray(csc[1], dtype=np.int64),
                                 np.ascontiguousarray(csc[2], dtype=np.float64))
        self.ctx = ctx
        self.n = len(colptr) - 1
        h = ctypes.c_void_p()
        L.check(ctx._lib.tk_matrix_from_csc(ctx.h, self.n, L.i64ptr(colptr), L.i64ptr(rowval),
                                            L.dptr(nzval), 1 if one_based else 0, ctypes.byref(h)))
        self.h = h

    @property
    def format(self):
        """0 = CSR, k > 0 = DIA with k diagonals."""
        return int(self.ctx._lib.tk_matrix_format(self.h))

    def matvec(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty(self.n)
        L.check(self.ctx._lib.tk_matvec(self.h, L.dptr(x), L.dptr(y)))
        return y

    def close(self):
        if getattr(self, "h", None):
            self.ctx._lib.tk_matrix_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceDecomposition:
    """tk_decomp: this rank's factors s = first .. first+nf-1 of a d_total-factor
    tensor decomposition, with device-resident V_s (n x kmax+1), b_s and work vectors."""

    def __init__(self, ctx, method, d_total, first, mats, bs, kmax, track_all_gram=False, n=None):
        """mats may be empty (a rank of a job with more ranks than factors: it only takes part
        in the records exchange); n is then required.  track_all_gram: True/1 = Gram rows of
        every factor in the records, 2 = factor 0's rows per step, False/0 = the library's
        choice (tk_decomp_create)."""
        self.ctx = ctx
        self.method = method
        self.d_total = d_total
        self.first = first
        self.nf = len(mats)
        self.n = mats[0].n if mats else int(n)
        self.kmax = kmax
        self.layout = L.RecordLayout(kmax)
        self.m = self.layout.m
        self._bs = [np.ascontiguousarray(b, dtype=np.float64) for b in bs]
        MatArr = ctypes.c_void_p * self.nf
        BArr = ctypes.POINTER(ctypes.c_double) * self.nf
        marr = MatArr(*[m.h.value for m in mats])
        barr = BArr(*[L.dptr(b) for b in self._bs])
        h = ctypes.c_void_p()
        L.check(ctx._lib.tk_decomp_create(ctx.h, int(method), int(d_total), int(first), self.nf, marr,
                                          barr, int(self.n), int(kmax), int(track_all_gram),
                                          ctypes.byref(h)))
        self.h = h
        self._mats = mats

    @property
    def arnoldi_sweeps(self):
        """Sweeps over V per Arnoldi step (1: delayed-reorthogonalization CGS2 on banded
        A_s, 2: CGS2); TensorLanczos 1 for the one-sweep TTR on banded A_s, else 0;
        LanczosReorth 0 (tk_decomp_arnoldi_sweeps)."""
        return int(self.ctx._lib.tk_decomp_arnoldi_sweeps(self.h))

    @property
    def exchange_signalled(self):
        """Records exchange triggered by a signal word, not an event (tk_decomp_exchange_signalled)."""
        return bool(self.ctx._lib.tk_decomp_exchange_signalled(self.h))

    @property
    def next_step(self):
        """The next step index the device accepts (tk_decomp_next_step): steps below it are
        enqueued, possibly by a driver that ran ahead of the records read so far."""
        return int(self.ctx._lib.tk_decomp_next_step(self.h))

    @property
    def matrix_reads(self):
        """Reads of A_s's bytes per step of all local factors (tk_decomp_matrix_reads): 1 when
        factors sharing one A_s read it once for all, else the local factor count."""
        return int(self.ctx._lib.tk_decomp_matrix_reads(self.h))

    @property
    def factor_groups(self):
        """Streams the one-sweep Arnoldi step's launches use (tk_decomp_factor_groups)."""
        return int(self.ctx._lib.tk_decomp_factor_groups(self.h))

    @property
    def single_columns(self):
        """V_s in single-column tiles (tk_decomp_single_columns): the Gram-free one-sweep
        TensorLanczos; paired columns otherwise."""
        return bool(self.ctx._lib.tk_decomp_single_columns(self.h))

    @property
    def gram_deferred(self):
        """Factor 0's Gram comes from one SYRK (gram()) rather than per-step record rows
        (tk_decomp_gram_deferred)."""
        return bool(self.ctx._lib.tk_decomp_gram_deferred(self.h))

    def gram(self, f, k, want=True):
        """G = V_f[:, :k]' V_f[:, :k] of local factor f on MFMA (tk_decomp_gram); want=False
        leaves it on the device."""
        G = np.zeros((k, k)) if want else None
        L.check(self.ctx._lib.tk_decomp_gram(self.h, int(f), int(k), L.dptr(G)))
        return G.T.copy() if want else None

    def set_replica(self, on=True):
        """This rank's factors are replicas of another rank's (tk_decomp_set_replica): same
        steps, zero rows sent into the records all-reduce."""
        L.check(self.ctx._lib.tk_decomp_set_replica(self.h, 1 if on else 0))

    def _rec(self):
        return np.zeros((self.d_total, self.m))

    def init(self, want=True):
        r = self._rec() if want else None
        L.check(self.ctx._lib.tk_decomp_init(self.h, L.dptr(r)))
        return r

    def step(self, j, want=True):
        r = self._rec() if want else None
        L.check(self.ctx._lib.tk_decomp_step(self.h, int(j), L.dptr(r)))
        return r

    def step_async(self, j):
        """Enqueue step j; its record stays on the device (records(j+1, j+2))."""
        L.check(self.ctx._lib.tk_decomp_step(self.h, int(j), None))

    def sweep(self, j0, j1):
        L.check(self.ctx._lib.tk_decomp_sweep(self.h, int(j0), int(j1)))

    def flush(self, want=True):
        r = self._rec() if want else None
        L.check(self.ctx._lib.tk_decomp_flush(self.h, L.dptr(r)))
        return r

    def records(self, s0, s1):
        out = np.zeros((s1 - s0, self.d_total, self.m))
        L.check(self.ctx._lib.tk_decomp_records(self.h, int(s0), int(s1), L.dptr(out)))
        return out

    def basis(self, f, c0, nc):
        out = np.zeros((nc, self.n))          # column-major n x nc == row-major nc x n
        L.check(self.ctx._lib.tk_decomp_get_basis(self.h, int(f), int(c0), int(nc), L.dptr(out)))
        return out.T

    def basis_mul(self, k, Ys, want=True):
        """X_s = V_s[:, :k] @ Y_s for the local factors (Ys: list of k x t arrays)."""
        if self.nf == 0 or Ys[0].shape[1] == 0:
            # (still the flush, and its record exchange, every rank makes); an empty term slice
            self.flush(False)
            if not want:
                return None
            return [np.zeros((self.n, 0)) for _ in Ys] if self.nf else []
        t = Ys[0].shape[1]
        Y = np.ascontiguousarray(np.stack([np.asarray(y, dtype=np.float64).T for y in Ys]))  # [nf][t][k]
        X = np.zeros((self.nf, t, self.n)) if want else None
        L.check(self.ctx._lib.tk_decomp_basis_mul(self.h, int(k), int(t), L.dptr(Y), L.dptr(X)))
        if not want:
            return None
        return [X[f].T.copy() for f in range(self.nf)]

    def close(self):
        if getattr(self, "h", None):
            self.ctx._lib.tk_decomp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
