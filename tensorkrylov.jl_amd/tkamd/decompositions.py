"""TensorArnoldi / TensorLanczos / TensorLanczosReorth backed by libtkhip.

Mirrors src/decompositions.jl:120-176 and the fan-out orthonormalize!(td, b) /
orthonormalize!(td, k) of src/orthogonal_bases.jl:142-180.  The n-length state
(V_s, b_s, work vectors) lives on the device; the host keeps only what the
reference's driver reads on the host: H_s (k x k minors and H_s[k+1,k]), btilde_s,
and factor 1's Gram rows for orthogonality_data.  H is updated from the per-step
records with the reference's bookkeeping (update_subdiagonals!, the LanczosReorth
zeroing of H[1:k-2, k]).
"""
import numpy as np

from . import _lib as L
from .device import Context, DeviceDecomposition, DeviceMatrix


class Partition:
    """Contiguous factor blocks over ranks: the first d % N ranks own
    ceil(d/N) factors, the rest floor(d/N).

    With more ranks than factors (N > d) and term_split (default; TKHIP_TERM_SPLIT=0 turns
    it off), rank r >= d holds a REPLICA of factor r % d instead of idling: it runs the same
    steps (sending zero rows into the records all-reduce, tk_decomp_set_replica) and at
    convergence the ranks holding factor s split the t exponential-sum terms of
    X_s = V_s Y_s between them (terms(t); src/tensor_krylov_method.jl:10-34 and
    basis_tensor_mul!, src/utils.jl:478-488).  Without term_split those ranks own nothing."""

    def __init__(self, d, nranks=1, rank=0, term_split=None):
        import os
        self.d, self.nranks, self.rank = d, nranks, rank
        if term_split is None:
            term_split = os.environ.get("TKHIP_TERM_SPLIT", "1") != "0"
        self.term_split = bool(term_split) and nranks > d
        q, r = divmod(d, nranks)
        self.sizes = [q + (1 if i < r else 0) for i in range(nranks)]
        self.starts = [sum(self.sizes[:i]) for i in range(nranks)]
        if self.term_split:
            self.sizes = [1] * nranks
            self.starts = [i % d for i in range(nranks)]

    @property
    def first(self):
        return self.starts[self.rank]

    @property
    def nf(self):
        return self.sizes[self.rank]

    @property
    def replica(self):
        """True when another rank owns this rank's factors (their records come from there)."""
        return self.term_split and self.rank >= self.d

    def local(self):
        return range(self.first, self.first + self.nf)

    def terms(self, t):
        """This rank's contiguous slice [c0, c1) of the t exponential-sum terms (columns of
        Y_s / X_s): all of them unless term_split, else the ranks holding the same factor
        (ranks s, s + d, s + 2d, ...) take near-equal consecutive slices (possibly empty)."""
        if not self.term_split:
            return 0, t
        s, g = self.rank % self.d, self.rank // self.d
        groups = len(range(s, self.nranks, self.d))
        q, r = divmod(t, groups)
        c0 = g * q + min(g, r)
        return c0, c0 + q + (1 if g < r else 0)


class TensorDecomposition:
    method = None
    name = None

    def __init__(self, A, nmax, ctx=None, partition=None, track_all_gram=False, backend=None):
        self.A = A
        self.d = len(A)
        self.n = A.dimensions()[0]
        self.kmax = nmax
        self.part = partition or Partition(self.d)
        self.layout = L.RecordLayout(nmax)
        KP, KC = nmax + 2, nmax + 1
        self.H = np.zeros((self.d, KP, KC))
        self.btilde = np.zeros((self.d, KC))
        self.gram = {}
        self.loss = np.zeros((self.d, KC))
        self.reorth = np.zeros((self.d, KC), dtype=bool)
        self.track_all_gram = track_all_gram
        self.ctx = ctx
        self._backend = backend
        self.dev = None
        self._issued = {}

    # -------------------------------------------------------------- device setup
    def _attach(self, b):
        if self._backend is not None:           # injected (tests of the host logic only)
            self.dev = self._backend(self, b)
            if self.part.replica:
                self.dev.set_replica()
            return
        if self.ctx is None:
            self.ctx = Context(0)
        mats = {}
        dmats = []
        for s in self.part.local():
            key = id(self.A[s])
            if key not in mats:                 # factors sharing A_s share its device CSR
                mats[key] = DeviceMatrix(self.ctx, self.A[s])
            dmats.append(mats[key])
        self._dmats = list(mats.values())
        self.dev = DeviceDecomposition(self.ctx, self.method, self.d, self.part.first, dmats,
                                       [b[s] for s in self.part.local()], self.kmax,
                                       track_all_gram=self.track_all_gram, n=len(b[0]))
        if self.part.replica:
            self.dev.set_replica()

    # -------------------------------------------------------------- records -> host mirror
    def _apply_gram(self, rec):
        lay = self.layout
        for s in range(self.d):
            c = int(round(rec[s, lay.col]))
            if c < 0:
                continue
            self.btilde[s, c] = rec[s, lay.bt]
            if rec[s, lay.tracked] > 0:
                G = self.gram.setdefault(s, np.zeros((self.kmax + 1, self.kmax + 1)))
                G[c, :c + 1] = rec[s, lay.gram:lay.gram + c + 1]

    def _apply_step(self, j, rec):
        raise NotImplementedError

    # -------------------------------------------------------------- reference API
    def orthonormalize_first(self, b):
        """orthonormalize!(td, b) (src/orthogonal_bases.jl:142-160): V[:,1] = b/|b|,
        then step 1 for every factor."""
        self._attach(b)
        r0 = self.dev.init()
        self._apply_gram(r0)
        self.first_records = [(-1, r0)]          # for a native driver taking over (tk_solver)
        self.orthonormalize(1)
        self.first_records.append((0, self._last_rec))

    def orthonormalize(self, k):
        """orthonormalize!(td, k) (src/orthogonal_bases.jl:162-180), k 1-based."""
        self.issue(k)
        self.collect(k)

    def issue(self, k):
        """Enqueue step k on the device without waiting (the driver overlaps it with the
        host's compressed solve of step k-1).  Columns <= k-1 of V, H and b~ are not
        touched by step k, so results are the same as with orthonormalize(k)."""
        j = k - 1
        if j < getattr(self.dev, "next_step", 0):
            # already enqueued (the native loop, tk_solver_run, issues steps ahead of the
            # records it reads): its record waits on the device for collect()
            return
        if hasattr(self.dev, "step_async"):
            self.dev.step_async(j)
        else:
            self._issued[j] = self.dev.step(j)

    def collect(self, k):
        """Records of an issued step k -> the host mirror of H, b~ and the Gram rows."""
        j = k - 1
        rec = self._issued.pop(j, None)
        if rec is None:
            rec = self.dev.records(j + 1, j + 2)[0]
        self._apply_step(j, rec)
        self._apply_gram(rec)
        self._last_rec = rec

    def flush(self):
        rec = self.dev.flush()
        self._apply_gram(rec)

    def subdiagonal(self, k):
        return [self.H[s, k, k - 1] for s in range(self.d)]

    def minors(self, k):
        """compute_minors (src/utils.jl:490-498): H_s[1:k,1:k] for every factor."""
        return [self.H[s, :k, :k].copy() for s in range(self.d)]

    def orthogonality_loss(self, s, k):
        from .compressed import orthogonality_loss_from_gram
        if s not in self.gram and s == 0 and getattr(self.dev, "gram_deferred", False):
            # no Gram rows in the records: one SYRK of the basis (tk_decomp_gram)
            return orthogonality_loss_from_gram(self.dev.gram(0, k), k)
        return orthogonality_loss_from_gram(self.gram[s], k)

    def basis(self, s, k):
        """V_s[:, 1:k] (local factor s only)."""
        f = s - self.part.first
        assert 0 <= f < self.part.nf, "factor %d is not owned by this rank" % s
        return self.dev.basis(f, 0, k)

    def close(self):
        if self.dev is not None and hasattr(self.dev, "close"):
            self.dev.close()
        for m in getattr(self, "_dmats", []):
            m.close()


class TensorArnoldi(TensorDecomposition):
    """src/decompositions.jl:120-137 -- MGS steps (src/orthogonal_bases.jl:15-37)."""
    method = L.TK_ARNOLDI
    name = "TensorArnoldi"

    def _apply_step(self, j, rec):
        for s in range(self.d):
            self.H[s, :j + 2, j] = rec[s, :j + 2]


class TensorLanczos(TensorDecomposition):
    """src/decompositions.jl:140-157 -- TTR steps (src/orthogonal_bases.jl:39-67)."""
    method = L.TK_LANCZOS
    name = "TensorLanczos"

    def _apply_step(self, j, rec):
        for s in range(self.d):
            alpha, beta = rec[s, j], rec[s, j + 1]
            self.H[s, j, j] = alpha                      # :50
            self.H[s, j + 1, j] = beta                   # update_subdiagonals! (decompositions.jl:180-186)
            self.H[s, j, j + 1] = beta


class TensorLanczosReorth(TensorDecomposition):
    """src/decompositions.jl:159-176 -- TTR + loss check + MGS redo
    (src/orthogonal_bases.jl:98-139)."""
    method = L.TK_LANCZOS_REORTH
    name = "TensorLanczosReorth"

    def _apply_step(self, j, rec):
        lay = self.layout
        for s in range(self.d):
            self.loss[s, j] = rec[s, lay.loss]
            if rec[s, lay.flag] > 0:
                self.reorth[s, j] = True
                self.H[s, :j + 2, j] = rec[s, :j + 2]    # MGS column (:125)
                beta = self.H[s, j + 1, j]               # :127
                self.H[s, :max(j - 1, 0), j] = 0.0       # H[1:k-2, k] .= 0 (:129)
            else:
                self.H[s, j, j] = rec[s, j]
                beta = rec[s, j + 1]
            self.H[s, j + 1, j] = beta                   # update_subdiagonals! (:137)
            self.H[s, j, j + 1] = beta


METHODS = {"TensorArnoldi": TensorArnoldi, "TensorLanczos": TensorLanczos,
           "TensorLanczosReorth": TensorLanczosReorth}


# ------------------------------------------------------------------ single-matrix drivers
class Decomposition:
    """Result of arnoldi_algorithm / lanczos_algorithm: the reference's Arnoldi / Lanczos
    structs (src/decompositions.jl:28-110) with host copies of V and H."""

    def __init__(self, A, V, H, loss=None):
        self.A, self.V, self.H = A, V, H
        self.loss = loss


def _single(cls, A, b, nmax, ctx, backend):
    from .structures import KroneckerMatrix, SymInstance, as_csc
    csc = as_csc(A)
    td = cls(KroneckerMatrix(SymInstance, [csc]), nmax, ctx=ctx, track_all_gram=True, backend=backend)
    return td, csc


def arnoldi_algorithm(A, b, k, ctx=None, backend=None):
    """arnoldi_algorithm(A, b, k) (src/orthogonal_bases.jl:182-195): k Arnoldi steps from
    V[:,1] = b/|b|; V is n x (k+1), H is (k+1) x k."""
    td, csc = _single(TensorArnoldi, A, b, k, ctx, backend)
    try:
        td.orthonormalize_first([b])
        for j in range(2, k + 1):
            td.orthonormalize(j)
        td.flush()
        return Decomposition(csc, td.basis(0, k + 1), td.H[0, :k + 1, :k].copy())
    finally:
        td.close()


def lanczos_algorithm(A, b, k, reorth=False, ctx=None, backend=None):
    """lanczos_algorithm(A, b, k[, LanczosReorth]) (src/orthogonal_bases.jl:198-229): k-1
    three-term steps; V is n x k, H is k x k (H[k,k] is left 0 as in the reference)."""
    if k < 2:
        raise ValueError("lanczos_algorithm needs k >= 2")
    cls = TensorLanczosReorth if reorth else TensorLanczos
    td, csc = _single(cls, A, b, k - 1, ctx, backend)
    try:
        td.orthonormalize_first([b])
        for j in range(2, k):
            td.orthonormalize(j)
        td.flush()
        H = td.H[0, :k, :k].copy()
        H[k - 1, k - 1] = 0.0
        return Decomposition(csc, td.basis(0, k), H, td.loss[0, :k - 1].copy() if reorth else None)
    finally:
        td.close()


def orthogonality_loss(V, k):
    """norm(V[:,1:k]'V[:,1:k] - I) (src/orthogonal_bases.jl:250-257)."""
    Vk = np.asarray(V)[:, :k]
    return float(np.linalg.norm(Vk.T @ Vk - np.eye(k)))


def isorthonormal(x, k, tol=1e-8):
    """isorthonormal(V | decomposition | tensor decomposition, k) (src/orthogonal_bases.jl:
    259-284).  A TensorDecomposition is checked through the device Gram rows of every factor
    it tracks (all factors when built with track_all_gram=True)."""
    if isinstance(x, Decomposition):
        return orthogonality_loss(x.V, k) < tol
    if isinstance(x, TensorDecomposition):
        if not x.gram:
            raise ValueError("no Gram rows tracked for this decomposition")
        return all(x.orthogonality_loss(s, k) < tol for s in x.gram)
    return orthogonality_loss(x, k) < tol
