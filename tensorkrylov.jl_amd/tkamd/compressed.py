"""Compressed-side (k-sized) host numerics of tensorkrylov!.

Restates, vectorized, the reference's per-iteration host work on the projected
system (none of it touches n-length data):
  * SpectralData / update_data!            src/eigenvalues.jl:247-370
  * ApproximationData / compute_rank! /
    exponential_sum_parameters!            src/approximation.jl:6-175
  * solve_compressed_system                src/tensor_krylov_method.jl:10-34,
                                           src/utils.jl:501-523
  * residualnorm! / compressed_residual /
    MVnorm / tensorinnerprod               src/utils.jl:132-443 (Lemma 3.4)
Differences from the reference are performance-only: the coefficient tables are loaded
once (the reference re-reads the CSV every iteration, src/approximation.jl:162-163);
the compressed solve and the residual run in native host code (libtkhip, tk_host.cpp):
exp(gamma_j * Symmetric(H)) for all t terms comes from ONE eigendecomposition
(exp(gH) = Q exp(g L) Q'); the O(d^3 t^2) masked products become leave-one-out /
leave-two-out elementwise products.  Exact-arithmetic results are identical.
"""
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))


class CompressedNormBreakdown(Exception):
    """src/utils.jl:7-14: the compressed squared residual came out negative."""

    def __init__(self, r_comp):
        super().__init__("compressed norm breakdown: r_comp = %r" % r_comp)
        self.r_comp = r_comp


# ------------------------------------------------------------------ spectral data

def laplace_eigenvalue(n, k, j):
    """src/eigenvalues.jl:247-256: eigenvalue j of the k x k minor of the n-point Laplacian."""
    h = 1.0 / (n + 1)
    return 4 * (1.0 / (h * h)) * math.sin(j * math.pi * (1.0 / (2 * (k + 1)))) ** 2


class SpectralData:
    """SpectralData{matT,T,U} (src/eigenvalues.jl:268-284) with update_data!
    (:353-370).  lambda_min/max/kappa of d * A_s[1:k,1:k]."""

    def __init__(self, A, nmax):
        self.A = A
        self.symmetric = A.symmetric
        self.lmin = np.full(nmax, np.inf)
        self.lmax = np.full(nmax, np.inf)
        self.kappa = np.full(nmax, np.inf)
        self.k = 1
        self._dense = None

    def _minor(self, k):
        from .structures import csc_leading_block
        return csc_leading_block(self.A[0], k)

    def update(self, d):
        self.k += 1
        k = self.k
        cls = self.A.matrixclass
        n = self.A.dimensions()[0]
        if self.symmetric:
            if cls in ("Laplace", "LaplaceDense"):
                lo = laplace_eigenvalue(n, k, 1) * d              # analytic_eigenvalues :258-265
                hi = laplace_eigenvalue(n, k, k) * d
            else:
                ev = np.linalg.eigvalsh(self._minor(k))           # :337
                lo, hi = ev.min() * d, ev.max() * d
            self.lmin[k - 1], self.lmax[k - 1] = lo, hi
            self.kappa[k - 1] = hi * (1.0 / lo)                   # :360
        else:
            ev = np.linalg.eigvals(self._minor(k))                # :344-350
            if np.all(ev.imag == 0):
                ev = ev.real
            self.lmin[k - 1] = float(np.min(ev)) * d

    def current(self):
        k = self.k
        return self.lmin[k - 1], self.lmax[k - 1], self.kappa[k - 1]


# ------------------------------------------------------------------ exp-sum approximation

class ExpSumTables:
    """coefficients_data (packed by data/pack_tables.py), loaded once."""

    _cache = None

    def __init__(self, path=None):
        path = path or os.path.join(_HERE, "data", "expsum_tables.npz")
        z = np.load(path, allow_pickle=False)
        self.R = np.asarray(z["R"])
        self.err = np.asarray(z["err"])
        self._z = z
        self._coef = {}

    @classmethod
    def default(cls):
        if cls._cache is None:
            cls._cache = cls()
        return cls._cache

    def coefficients(self, rank, digit, order):
        key = "xk%02d.%d_%d" % (rank, digit, order)         # 1_xk{t:02d}.{digit}_{order}
        if key not in self._coef:
            v = np.asarray(self._z[key])
            self._coef[key] = (v[rank:2 * rank].copy(), v[:rank].copy())   # alpha, omega
        return self._coef[key]


def parse_condition(kappa):
    """src/approximation.jl:109-116."""
    order = int(math.floor(math.log10(kappa)))
    digit = int(math.floor(kappa / (10.0 ** order)))
    return order, digit


class ApproximationData:
    """ApproximationData{T,U} (src/approximation.jl:6-30): rank t and (alpha, omega)
    with 1/x ~ sum_j omega_j exp(-alpha_j x)."""

    def __init__(self, tol, symmetric, tables=None):
        self.tol = tol
        self.symmetric = symmetric
        self.tables = tables if tables is not None or not symmetric else ExpSumTables.default()
        self.rank = 0
        self.alpha = np.zeros(1)
        self.omega = np.zeros(1)
        self.first_digit = 0
        self.condition_order = 0

    def update(self, spectral):
        lmin, _, kappa = spectral.current()
        if self.symmetric:
            # compute_rank! (:65-84) + exponential_sum_parameters! (:119-147)
            order, digit = parse_condition(kappa)
            R = self.tables.R
            while True:
                rows = np.nonzero(R == digit * 10.0 ** order)[0]
                if len(rows):
                    break
                digit += 1
                if digit > 100:
                    raise ValueError("condition number %r beyond the coefficient tables" % kappa)
            errs = self.tables.err[rows[0]]
            ok = np.nonzero(self.tol >= errs)[0]
            if len(ok) == 0:
                raise ValueError("no tabulated rank reaches tol=%g at kappa=%g" % (self.tol, kappa))
            self.rank = int(ok.min()) + 1
            self.first_digit, self.condition_order = digit, order
            self.alpha, self.omega = self.tables.coefficients(self.rank, digit, order)
        else:
            # compute_rank!(::NonSym) (:86-107) + closed form (:150-158)
            rank = 1
            while 2.75 * (1.0 / lmin) * math.exp(-math.pi * math.sqrt(rank / 2)) > self.tol:
                rank += 1
            self.rank = rank
            h = math.pi * (1.0 / math.sqrt(rank))
            js = np.arange(-rank, rank + 1, dtype=np.float64)
            self.alpha = np.log(np.exp(js * h) + np.sqrt(1 + np.exp(2 * js * h)))
            self.omega = h * (1.0 / np.sqrt(1 + np.exp(-2 * js * h)))


# ------------------------------------------------------------------ compressed solve
# Both functions run in libtkhip's host code (csrc/tk_host.cpp); they need no GPU.

def solve_compressed_system(H1, btilde, approx, lmin, symmetric):
    """y = sum_j omega_j/lmin * exp(-alpha_j/lmin * first(H)) btilde_s, as the Kruskal
    tensor (lambda, [Y_s]) of src/tensor_krylov_method.jl:10-34.  first(H) is
    Symmetric(H_1, :L) for SymInstance (src/tensor_struct.jl:259).  -> tk_compressed_solve"""
    import ctypes
    from . import _lib as L
    k = H1.shape[0]
    d = len(btilde)
    alpha = np.ascontiguousarray(approx.alpha, dtype=np.float64)
    omega = np.ascontiguousarray(approx.omega, dtype=np.float64)
    t = len(alpha)
    Hc = np.ascontiguousarray(np.asarray(H1, dtype=np.float64).T)        # column-major k x k
    B = np.ascontiguousarray(np.stack([np.asarray(b, dtype=np.float64)[:k] for b in btilde]))
    lam = np.empty(t)
    Y = np.empty((d, t, k))                                              # [s][j][i] = column-major k x t
    L.check(L.lib().tk_compressed_solve(d, k, L.dptr(Hc), 1 if symmetric else 0, L.dptr(B), t,
                                        L.dptr(alpha), L.dptr(omega), ctypes.c_double(lmin),
                                        L.dptr(lam), L.dptr(Y)))
    return lam, [Y[s].T for s in range(d)]


def residualnorm(Hs, lam, Ys, k, subdiag, btilde, b_norm):
    """residualnorm! + compressed_residual (src/utils.jl:371-443).
    Hs: d k x k minors (full), Ys: d k x t, subdiag[s] = H_s[k+1, k].
    Returns (r_comp, r_norm); raises CompressedNormBreakdown when r_comp < 0.
    -> tk_residualnorm"""
    import ctypes
    from . import _lib as L
    d = len(Ys)
    t = len(lam)
    H = np.ascontiguousarray(np.stack([np.asarray(h, dtype=np.float64)[:k, :k].T for h in Hs]))
    Y = np.ascontiguousarray(np.stack([np.asarray(y, dtype=np.float64).T for y in Ys]))
    B = np.ascontiguousarray(np.stack([np.asarray(b, dtype=np.float64)[:k] for b in btilde]))
    lamc = np.ascontiguousarray(lam, dtype=np.float64)
    sub = np.ascontiguousarray(subdiag, dtype=np.float64)
    rc = ctypes.c_double()
    rn = ctypes.c_double()
    st = L.lib().tk_residualnorm(d, k, t, L.dptr(H), L.dptr(lamc), L.dptr(Y), L.dptr(sub), L.dptr(B),
                                 ctypes.c_double(b_norm), ctypes.byref(rc), ctypes.byref(rn))
    if st == L.TK_BREAKDOWN:
        raise CompressedNormBreakdown(rc.value)
    L.check(st)
    return rc.value, rn.value


def orthogonality_loss_from_gram(G, k):
    """norm(V[:,1:k]'V[:,1:k] - I) (src/orthogonal_bases.jl:250-257) from the lower
    Gram rows G[c, 0..c] kept by the device."""
    Gk = np.tril(G[:k, :k])
    D = Gk + np.tril(Gk, -1).T - np.eye(k)
    return float(np.linalg.norm(D))


def orthogonality_losses_from_gram(G):
    """[norm(V[:,1:k]'V[:,1:k] - I) for k = 1..K] (src/orthogonal_bases.jl:250-257) from one
    Gram matrix G = V[:,1:K]'V[:,1:K] (lower triangle used): the squared loss grows by column
    k's diagonal and twice its off-diagonal squares (tk_orthogonality_losses -- the sum the
    native loop applies to the Gram it reads itself, so both give the same bits)."""
    from . import _lib as L
    G = np.asarray(G, dtype=np.float64)
    K = G.shape[0]
    Gc = np.ascontiguousarray(G.T)          # column-major G: lower triangle (i >= j) at j*K + i
    out = np.zeros(K)
    L.check(L.lib().tk_orthogonality_losses(K, L.dptr(Gc), L.dptr(out)))
    return out


# ------------------------------------------------------------------ native iteration driver

class IterationTables:
    """SpectralData / ApproximationData for every iteration k = 2..nmax, computed up front:
    they depend on A and tol only (src/eigenvalues.jl:353-370, src/approximation.jl:65-175),
    so the native driver (tk_solver) gets them per k.  If the approximation data run out at
    some k (kappa beyond the coefficient tables), `error` holds the exception the reference
    would raise at that iteration and rank[k-1:] = 0."""

    def __init__(self, A, nmax, tol, d=None):
        d = len(A) if d is None else d
        spectral = SpectralData(A, nmax)
        approx = ApproximationData(tol, A.symmetric)
        self.lmin = np.zeros(nmax)
        self.rank = np.zeros(nmax, dtype=np.int32)
        al, om = [], []
        self.error = None
        self.error_k = None
        for k in range(2, nmax + 1):
            spectral.update(d)
            try:
                approx.update(spectral)
            except ValueError as e:
                self.error, self.error_k = e, k
                break
            self.lmin[k - 1] = spectral.lmin[k - 1]
            self.rank[k - 1] = len(approx.alpha)
            al.append(np.asarray(approx.alpha, dtype=np.float64))
            om.append(np.asarray(approx.omega, dtype=np.float64))
        self.alpha = np.ascontiguousarray(np.concatenate(al) if al else np.zeros(1))
        self.omega = np.ascontiguousarray(np.concatenate(om) if om else np.zeros(1))


class NativeSolver:
    """tk_solver: the per-iteration host work of tensorkrylov! in native code (csrc/
    tk_solver.cpp) -- record bookkeeping, compressed solve, residual, orthogonality of V_1 --
    and the pipelined loop over a device decomposition with iterations evaluated on a pool
    of host threads."""

    def __init__(self, method, d, kmax, symmetric, b_norm, tables):
        import ctypes
        from . import _lib as L
        self._L = L
        self.d, self.kmax = d, kmax
        self.tables = tables
        h = ctypes.c_void_p()
        rank = np.ascontiguousarray(tables.rank, dtype=np.int32)
        self._rank = rank
        L.check(L.lib().tk_solver_create(int(method), int(d), int(kmax), 1 if symmetric else 0,
                                         ctypes.c_double(b_norm), L.dptr(tables.lmin),
                                         rank.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                         L.dptr(tables.alpha), L.dptr(tables.omega), ctypes.byref(h)))
        self.h = h
        self.split = None          # (nranks, rank) once the evaluations are split (share)

    def overlay(self, first, nf, records):
        """Emulation only: rows of factors outside [first, first+nf) come from `records`
        ([kmax+2][d][m], a full run's) whenever records are applied (tk_solver_overlay)."""
        self._ov = None if records is None else np.ascontiguousarray(records, dtype=np.float64)
        self._L.check(self._L.lib().tk_solver_overlay(self.h, int(first), int(nf),
                                                      None if records is None else self._L.dptr(self._ov)))

    def apply(self, j, rec):
        rec = np.ascontiguousarray(rec, dtype=np.float64)
        self._L.check(self._L.lib().tk_solver_apply(self.h, int(j), self._L.dptr(rec)))

    def evaluate(self, k):
        """(r_comp, r_norm, relative residual, orthogonality loss) of iteration k; raises
        CompressedNormBreakdown like residualnorm!."""
        out = np.zeros(4)
        st = self._L.lib().tk_solver_evaluate(self.h, int(k), self._L.dptr(out))
        if st == self._L.TK_BREAKDOWN:
            raise CompressedNormBreakdown(out[0])
        self._L.check(st)
        return tuple(float(x) for x in out)

    def solution(self, k):
        t = int(self.tables.rank[k - 1])
        lam = np.zeros(t)
        Y = np.zeros((self.d, t, k))
        self._L.check(self._L.lib().tk_solver_solution(self.h, int(k), self._L.dptr(lam), self._L.dptr(Y)))
        return lam, [Y[s].T.copy() for s in range(self.d)]

    def state(self):
        KP, KC = self.kmax + 2, self.kmax + 1
        H = np.zeros((self.d, KP, KC))
        bt = np.zeros((self.d, KC))
        G = np.zeros((KC, KC))
        self._L.check(self._L.lib().tk_solver_state(self.h, self._L.dptr(H), self._L.dptr(bt),
                                                    self._L.dptr(G)))
        return H, bt, G

    def share(self, key, nranks, rank):
        """Split the evaluations over the ranks of this node (tk_solver_share): rank
        k % nranks evaluates iteration k, the others read its result from a shared-memory
        mailbox.  Collective (same key on every rank)."""
        self._L.check(self._L.lib().tk_solver_share(self.h, key.encode(), int(nranks), int(rank)))
        self.split = (int(nranks), int(rank)) if nranks > 1 else None

    def share_emulated(self, nranks, rank, results):
        """Emulation (bench.py --emulate-ranks): the split on one rank, the other ranks' results
        from a full run's `results` ([kmax][6], results())."""
        self._tab = np.ascontiguousarray(results, dtype=np.float64)
        assert self._tab.shape == (self.kmax, 6)
        self._L.check(self._L.lib().tk_solver_share_emulated(self.h, int(nranks), int(rank), self._L.dptr(self._tab)))
        self.split = (int(nranks), int(rank)) if nranks > 1 else None

    def evaluate_shared(self, k):
        """evaluate(k) under the split: owner evaluates and posts, the others read."""
        out = np.zeros(4)
        st = self._L.lib().tk_solver_evaluate_shared(self.h, int(k), self._L.dptr(out))
        if st == self._L.TK_BREAKDOWN:
            raise CompressedNormBreakdown(out[0])
        self._L.check(st)
        return tuple(float(x) for x in out)

    def owns(self, k):
        sp = getattr(self, "split", None)
        return sp is None or k % sp[0] == sp[1]

    def results(self):
        """Per iteration of the last run: [kmax][6] = r_comp, r_norm, relres, orthogonality,
        status, evaluation us on this rank (-1: evaluated by another rank); NaN rows where the
        run consumed nothing (tk_solver_results)."""
        out = np.zeros((self.kmax, 6))
        self._L.check(self._L.lib().tk_solver_results(self.h, self._L.dptr(out)))
        return out

    def prepare(self, nthreads):
        """Start the evaluation threads now (setup), not inside the loop (tk_solver_prepare)."""
        self._L.check(self._L.lib().tk_solver_prepare(self.h, int(nthreads)))

    def run(self, dev, tol, kfirst=2, depth=2, nthreads=4):
        """Pipelined loop k = kfirst..kmax on a DeviceDecomposition.  Returns (outcome,
        k_end, relres, projres, orth) with outcome 0 / 1 / 2 as tk_solver_run."""
        import ctypes
        L = self._L
        rel = np.zeros(self.kmax)
        proj = np.zeros(self.kmax)
        orth = np.zeros(self.kmax)
        k_end = ctypes.c_int()
        outcome = ctypes.c_int()
        L.check(L.lib().tk_solver_run(self.h, dev.h, ctypes.c_double(tol), int(kfirst), int(depth),
                                      int(nthreads), L.dptr(rel), L.dptr(proj), L.dptr(orth),
                                      ctypes.byref(k_end), ctypes.byref(outcome)))
        return outcome.value, k_end.value, rel, proj, orth

    def close(self):
        if getattr(self, "h", None):
            self._L.lib().tk_solver_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
