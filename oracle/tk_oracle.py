"""CPU restatement of thbake/TensorKrylov.jl (reference v0.1.0) -- TEST INFRASTRUCTURE ONLY.

This module is the parity ORACLE.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it, and only as the checker -- the product path
(tensorkrylov.jl_amd/) never imports, links or calls anything under oracle/.

It restates, in plain NumPy with explicit loops in the reference's operation order,
the reference's algorithm for the hot path and for the host-side compressed solve
that the driver needs to produce the reference's observable outputs
(ConvergenceData).  Every function cites the reference file:line it follows
(paths relative to the reference repository root).

Pinning: this restatement is checked in tests/test_oracle.py
against
  * the reference's recorded convergence histories (experiments/data/
    reproduction_data/{laplace_new,nonsym_new}, decoded to tests/golden/
    reproduction.json by tests/golden/make_golden.py),
  * the Lanczos known-answer test test/eigenvalues.jl:32,
  * the residual KAT test/utils.jl:188-227,
  * the orthonormality properties test/decompositions.jl:4-56.
The reference's arithmetic lives in Julia 1.9.3 SparseArrays / OpenBLAS 0.3.21 /
LAPACK (not in the reference tree, not available here); dot/nrm2 summation orders are
therefore not reproducible bit for bit and parity is tolerance-based.
"""
import math
import os

import numpy as np

EPS = np.finfo(np.float64).eps

# --------------------------------------------------------------------------------------
# Matrix gallery  (src/tensor_struct.jl:48-79)
# --------------------------------------------------------------------------------------


def _laplace_coeff(n):
    # h = inv(n + 1); inv(h^2)  (src/tensor_struct.jl:50-51); Julia literal h^2 == h*h
    h = 1.0 / (n + 1)
    return 1.0 / (h * h), h


def laplace_dense(n):
    """assemble_matrix(n, LaplaceDense): inv(h^2) * SymTridiagonal(2ones(n), -ones(n))
    (src/tensor_struct.jl:48-55)."""
    c, _ = _laplace_coeff(n)
    A = np.zeros((n, n))
    i = np.arange(n)
    A[i, i] = c * 2.0
    A[i[:-1], i[:-1] + 1] = c * -1.0
    A[i[:-1] + 1, i[:-1]] = c * -1.0
    return A


def convdiff_dense(n, c_conv=10.0):
    """assemble_matrix(n, ConvDiff, c=10): L + (c*inv(4h)) .* diagm(-1=>1, 0=>3, 1=>-5, 2=>1)
    (src/tensor_struct.jl:60-68); entries added in fp64 exactly as sparse `+` does."""
    ch, h = _laplace_coeff(n)
    cc = c_conv * (1.0 / (4 * h))
    L = laplace_dense(n)
    C = np.zeros((n, n))
    i = np.arange(n)
    C[i[1:], i[1:] - 1] = cc * 1.0
    C[i, i] = cc * 3.0
    C[i[:-1], i[:-1] + 1] = cc * -5.0
    C[i[:-2], i[:-2] + 2] = cc * 1.0
    return L + C


def dense_to_csc(A):
    """sparse(A) storage: column pointers, sorted row indices, values (0-based)."""
    n = A.shape[1]
    colptr = [0]
    rowval = []
    nzval = []
    for j in range(n):
        rows = np.nonzero(A[:, j])[0]
        rowval.extend(rows.tolist())
        nzval.extend(A[rows, j].tolist())
        colptr.append(len(rowval))
    return (np.array(colptr, dtype=np.int64), np.array(rowval, dtype=np.int64),
            np.array(nzval, dtype=np.float64))


def gallery_csc(n, cls):
    if cls == "Laplace":
        return dense_to_csc(laplace_dense(n))
    if cls == "ConvDiff":
        return dense_to_csc(convdiff_dense(n))
    raise ValueError(cls)


def csc_matvec(csc, x):
    """mul!(y, A::SparseMatrixCSC, x): Julia 1.9 SparseArrays `_spmatmul!` -- y zeroed, then
    for each column j, y[rowval[p]] += nzval[p] * x[j] (no FMA).  Used at
    src/orthogonal_bases.jl:20,45,103."""
    colptr, rowval, nzval = csc
    n = len(colptr) - 1
    y = np.zeros(n)
    for j in range(n):
        xj = x[j]
        for p in range(colptr[j], colptr[j + 1]):
            y[rowval[p]] = y[rowval[p]] + nzval[p] * xj
    return y


def csc_matvec_fast(csc, x):
    """Same arithmetic as csc_matvec for matrices whose rows receive contributions in
    ascending column order (always true for a CSC scatter): row sums in column order,
    computed per nonzero 'layer' so it is vectorized.  Bitwise equal to csc_matvec."""
    colptr, rowval, nzval = csc
    n = len(colptr) - 1
    cols = np.repeat(np.arange(n), np.diff(colptr))
    order = np.lexsort((cols, rowval))           # row-major, ascending column inside a row
    r, c, v = rowval[order], cols[order], nzval[order]
    prod = v * x[c]
    y = np.zeros(n)
    # position of each entry within its row
    start = np.searchsorted(r, np.arange(n))
    pos = np.arange(len(r)) - start[r]
    for layer in range(int(pos.max()) + 1 if len(pos) else 0):
        m = pos == layer
        y[r[m]] = y[r[m]] + prod[m]
    return y


# --------------------------------------------------------------------------------------
# Per-factor Krylov steps  (src/orthogonal_bases.jl, src/decompositions.jl)
# --------------------------------------------------------------------------------------


class Factor:
    """One factor's decomposition state: A (CSC), V (n x kmax+1), H ((kmax+1)^2),
    beta / v (Lanczos state).  Mirrors Arnoldi/Lanczos/LanczosReorth of
    src/decompositions.jl:28-110 with storage capped at kmax+1 columns (the reference
    allocates n+1, src/decompositions.jl:130-131, infeasible beyond small n)."""

    def __init__(self, csc, b, kmax, matvec=csc_matvec_fast):
        self.csc = csc
        self.n = len(b)
        self.V = np.zeros((self.n, kmax + 1))
        self.H = np.zeros((kmax + 1, kmax + 1))
        self.beta = 0.0
        self.matvec = matvec
        # initialize_decomp!: V[:, 1] = inv(norm(b)) .* b  (src/decompositions.jl:112-118)
        self.V[:, 0] = (1.0 / np.linalg.norm(b)) * b

    # ---- a1: orthonormalize!(::Decomposition, k, ::MGS)  src/orthogonal_bases.jl:15-37
    def arnoldi_mgs(self, k):
        """1-based k as in the reference: uses V[:, k], writes H[1:k+1, k], V[:, k+1]."""
        V, H = self.V, self.H
        v = self.matvec(self.csc, V[:, k - 1])                         # :20
        for i in range(k):                                              # :22-26
            H[i, k - 1] = np.dot(v, V[:, i])
            v = v - H[i, k - 1] * V[:, i]
        for i in range(k):                                              # :28-33
            H[i, k - 1] += np.dot(v, V[:, i])
            v = v - np.dot(v, V[:, i]) * V[:, i]
        H[k, k - 1] = np.linalg.norm(v)                                 # :35
        V[:, k] = v * (1.0 / H[k, k - 1])                               # :36

    # ---- a2: orthonormalize!(::Lanczos, k, ::TTR)  src/orthogonal_bases.jl:39-67
    def _ttr(self, k):
        V, H = self.V, self.H
        # Lanczos(A, V, H, k): beta = H[k-1, k], v = V[:, k-1]  (src/decompositions.jl:76-83);
        # for k == 1 the (A, V, H, b) constructor sets beta = 0, v = 0 (:64-74)
        if k == 1:
            beta_prev, vprev = 0.0, np.zeros(self.n)
        else:
            beta_prev, vprev = H[k - 2, k - 1], V[:, k - 2]
        u = self.matvec(self.csc, V[:, k - 1])                          # :45
        u = u - beta_prev * vprev                                       # :47
        H[k - 1, k - 1] = np.dot(u, V[:, k - 1])                        # :50
        v = u - H[k - 1, k - 1] * V[:, k - 1]                           # :53
        beta = np.linalg.norm(v)                                        # :56
        V[:, k] = np.zeros(self.n) if beta == 0.0 else (1.0 / beta) * v  # :59
        return beta

    def lanczos_ttr(self, k):
        beta = self._ttr(k)
        self._update_subdiagonals(k, beta)                              # :65
        self.beta = beta

    # ---- a3: orthonormalize!(::LanczosReorth, k, ::TTR)  src/orthogonal_bases.jl:98-139
    def lanczos_reorth(self, k, force=None):
        """force=True/False overrides the loss > sqrt(eps) decision (tests use it to
        follow the device's decisions, which are rounding-sensitive near the threshold)."""
        beta = self._ttr(k)                                             # :100-117
        loss = orthogonality_loss(self.V, k + 1)                        # :119
        reorth = loss > math.sqrt(EPS) if force is None else bool(force)   # :123
        if reorth:
            self.arnoldi_mgs(k)                                         # :125
            beta = self.H[k, k - 1]                                     # :127
            self.H[0:max(k - 2, 0), k - 1] = 0.0                        # :129
        self._update_subdiagonals(k, beta)                              # :137
        self.beta = beta
        return loss, reorth

    def _update_subdiagonals(self, k, beta):
        # update_subdiagonals!(H, k, beta)  src/decompositions.jl:180-186
        self.H[k, k - 1] = beta
        self.H[k - 1, k] = beta


def orthogonality_loss(V, k):
    """norm(V[:,1:k]' V[:,1:k] - I)  (src/orthogonal_bases.jl:231-257)."""
    Vk = V[:, :k]
    G = Vk.T @ Vk
    return float(np.linalg.norm(G - np.eye(k)))


def arnoldi_algorithm(A_csc, b, k):
    """src/orthogonal_bases.jl:182-196: k MGS steps on zeros(n, k+1)."""
    f = Factor(A_csc, b, k)
    for j in range(1, k + 1):
        f.arnoldi_mgs(j)
    return f


def lanczos_algorithm(A_csc, b, k, reorth=False):
    """src/orthogonal_bases.jl:199-229: k-1 TTR steps on zeros(n, k)."""
    f = Factor(A_csc, b, k)
    for j in range(1, k):
        if reorth:
            f.lanczos_reorth(j)
        else:
            f.lanczos_ttr(j)
    return f


# --------------------------------------------------------------------------------------
# Sturm-sequence helpers for the KAT  (src/eigenvalues.jl:33-76)
# --------------------------------------------------------------------------------------


def next_coefficients(polys, j, gamma, beta):
    """next_coefficients!  (src/eigenvalues.jl:55-76); polys is a 1-based-like list."""
    p1 = list(polys[j - 1])
    a = [1.0] * (j + 1)
    a[0] = gamma * p1[0]
    for i in range(1, j):
        a[i] = gamma * p1[i] - p1[i - 1]
    a[j] = -p1[j - 1]
    p2 = polys[j - 2]
    for i in range(j - 1):
        a[i] -= beta ** 2 * p2[i]
    polys.append(a)


def evalpoly(x, coeffs):
    r = 0.0
    for c in reversed(coeffs):
        r = r * x + c
    return r


def sign_changes(x, polys):
    """src/eigenvalues.jl:33-53."""
    cnt = 0
    cur = evalpoly(x, polys[0])
    for p in polys[1:]:
        e = evalpoly(x, p)
        if e * cur < 0.0:
            cur = e
            cnt += 1
    return cnt


# --------------------------------------------------------------------------------------
# Spectral data  (src/eigenvalues.jl:247-370)
# --------------------------------------------------------------------------------------


def laplace_eigenvalue(n, k, j):
    """src/eigenvalues.jl:247-256."""
    h = 1.0 / (n + 1)
    return 4 * (1.0 / (h * h)) * math.sin(j * math.pi * (1.0 / (2 * (k + 1)))) ** 2


def analytic_eigenvalues(d, n, k):
    """src/eigenvalues.jl:258-265."""
    return laplace_eigenvalue(n, k, 1) * d, laplace_eigenvalue(n, k, k) * d


def spectral_update(cls, symmetric, d, n, k, A_dense_minor=None):
    """update_data!(::SpectralData, d, class) at iteration k (src/eigenvalues.jl:353-370).
    Returns (lambda_min, lambda_max, kappa) -- lambda_max/kappa are inf for NonSym."""
    if symmetric:
        if cls == "Laplace":
            lmin, lmax = analytic_eigenvalues(d, n, k)                 # :335
        else:
            ev = np.linalg.eigvalsh(A_dense_minor)                      # :337
            lmin, lmax = ev.min() * d, ev.max() * d
        return lmin, lmax, lmax * (1.0 / lmin)                          # :360
    ev = np.linalg.eigvals(A_dense_minor)                               # :344-350
    if np.all(ev.imag == 0):
        ev = ev.real
    return float(np.min(ev)) * d, math.inf, math.inf


# --------------------------------------------------------------------------------------
# Exponential-sum approximation  (src/approximation.jl)
# --------------------------------------------------------------------------------------


class ExpSumTables:
    """The coefficients_data tables.  Reads the packed .npz the product ships (data
    only); the lookup logic below is restated independently of the product."""

    def __init__(self, path=None):
        if path is None:
            here = os.path.dirname(os.path.abspath(__file__))
            path = os.path.join(here, "..", "tensorkrylov.jl_amd", "tkamd", "data", "expsum_tables.npz")
        z = np.load(path, allow_pickle=False)
        self.R = z["R"]
        self.err = z["err"]
        self._z = z

    def coeffs(self, rank, first_digit, order):
        # filename "1_xk" + %02d rank + "." + digit + "_" + order  (src/approximation.jl:128-134)
        key = "xk%02d.%d_%d" % (rank, first_digit, order)
        v = self._z[key]
        return v[rank:2 * rank].copy(), v[:rank].copy()          # alpha, omega  (:144-145)


def parse_condition(kappa):
    """src/approximation.jl:109-116."""
    order = int(math.floor(math.log10(kappa)))
    digit = int(math.floor(kappa / (10.0 ** order)))
    return order, digit


def sym_expsum(tables, kappa, tol):
    """compute_rank!(::SymInstance) + exponential_sum_parameters! (src/approximation.jl:65-84,
    :119-147).  Returns (rank, alpha, omega)."""
    order, digit = parse_condition(kappa)
    while True:
        rows = np.nonzero(tables.R == digit * 10.0 ** order)[0]      # getclosestrow :56-63
        if len(rows):
            break
        digit += 1                                                    # :71-76
    errs = tables.err[rows[0]]
    ranks = [t + 1 for t in range(63) if tol >= errs[t]]              # :79-81
    rank = min(ranks)
    alpha, omega = tables.coeffs(rank, digit, order)
    return rank, alpha, omega


def nonsym_expsum(lmin, tol):
    """compute_rank!(::NonSymInstance) + closed-form sinc quadrature
    (src/approximation.jl:86-107, :150-158).  t = 2*rank + 1 terms."""
    def bound(r):
        return 2.75 * (1.0 / lmin) * math.exp(-math.pi * math.sqrt(r / 2))
    rank = 1
    while bound(rank) > tol:
        rank += 1
    h = math.pi * (1.0 / math.sqrt(rank))
    js = range(-rank, rank + 1)
    alpha = np.array([math.log(math.exp(j * h) + math.sqrt(1 + math.exp(2 * j * h))) for j in js])
    omega = np.array([h * (1.0 / math.sqrt(1 + math.exp(-2 * j * h))) for j in js])
    return rank, alpha, omega


# --------------------------------------------------------------------------------------
# Compressed solve  (src/tensor_krylov_method.jl:10-34, src/utils.jl:501-523)
# --------------------------------------------------------------------------------------


def _expm(M):
    import scipy.linalg
    return scipy.linalg.expm(M)


def solve_compressed_system(H1, btilde, alpha, omega, lmin, symmetric):
    """Y_s[:, j] = exp(-alpha_j/lmin * first(H)) * btilde_s; lambda = omega / lmin.
    first(H) = Symmetric(H_1, :L) for SymInstance (src/tensor_struct.jl:259), dense
    Matrix for NonSymInstance (:260).  exp(Symmetric) via eigen; exp(Matrix) Pade."""
    k = H1.shape[0]
    t = len(omega)
    lam_inv = 1.0 / lmin
    lam = lam_inv * omega
    Y = [np.ones((k, t)) for _ in btilde]
    if symmetric:
        L = np.tril(H1)
        S = L + np.tril(L, -1).T
    for j in range(t):
        gamma = -alpha[j] * lam_inv
        if symmetric:
            w, Q = np.linalg.eigh(gamma * S)
            E = (Q * np.exp(w)) @ Q.T
        else:
            E = _expm(gamma * H1)
        for s, b in enumerate(btilde):
            Y[s][:, j] = E @ b
    return lam, Y


# --------------------------------------------------------------------------------------
# Residual norm, Lemma 3.4  (src/utils.jl:132-443) -- faithful mask loops
# --------------------------------------------------------------------------------------


class CompressedNormBreakdown(Exception):
    """src/utils.jl:7-14."""


def _lower_syrk(M):
    return np.tril(M.T @ M)


def squared_tensor_entries(Y_masked, Gamma):
    """src/utils.jl:206-226."""
    t = Gamma.shape[0]
    value = 0.0
    for k in range(t):
        value += Gamma[k, k] * np.prod([Y[k, k] for Y in Y_masked])
        for i in range(k + 1, t):
            value += 2 * Gamma[i, k] * np.prod([Y[i, k] for Y in Y_masked])
    return value


def mvnorm(lam_lower, Ly, X, Lz, d, t):
    """MVnorm (src/utils.jl:255-324)."""
    total = 0.0
    for s in range(d):
        for r in range(d):
            for j in range(t):
                for i in range(j, t):
                    a = np.prod([Ly[q][i, j] for q in range(d) if q != s and q != r])
                    b = 1.0 if s == r else X[s][i, j] * X[r][j, i]
                    g = Lz[s][i, j] if s == r else 1.0
                    val = lam_lower[i, j] * a * b * g
                    total += val if i == j else 2 * val
    return total


def residualnorm(Hs, lam, Y, k, subdiag, btilde, b_norm):
    """residualnorm! + compressed_residual (src/utils.jl:371-443).  Hs are k x k minors
    (full, both triangles), Y the k x t factor matrices.  Returns (r_comp, r_norm)."""
    d = len(Y)
    t = len(lam)
    Ly = [_lower_syrk(Ys) for Ys in Y]                           # compute_lower_triangles! :186-194
    Lam = np.tril(np.outer(lam, lam))                            # compute_lower_outer! :132-144
    res = 0.0
    for s in range(d):
        Gamma = np.tril(np.outer(Y[s][k - 1, :], Y[s][k - 1, :])) * Lam   # cp_tensor_coefficients :146-164
        y2 = squared_tensor_entries([Ly[q] for q in range(d) if q != s], Gamma)
        res += subdiag[s] ** 2 * y2
    # compressed_residual :371-399
    Z = [Hs[s] @ Y[s] for s in range(d)]                         # matrix_vector :229-253
    X = [Y[s].T @ Z[s] for s in range(d)]
    Lz = [_lower_syrk(Zs) for Zs in Z]
    hy_norm = mvnorm(Lam, Ly, X, Lz, d, t)
    hy_b = 0.0                                                   # tensorinnerprod :332-369
    for s in range(d):
        for i in range(t):
            hy_b += lam[i] * Z[s][0, i] * np.prod([Y[q][0, i] for q in range(d) if q != s])
    hy_b *= b_norm
    bnorm2 = np.prod([np.dot(b, b) for b in btilde])             # kronproddot
    r_comp = hy_norm - 2 * hy_b + bnorm2
    if r_comp < 0.0:
        raise CompressedNormBreakdown(r_comp)
    return r_comp, math.sqrt(res + r_comp)


# --------------------------------------------------------------------------------------
# Driver  (src/tensor_krylov_method.jl:36-125, src/system.jl:65-83)
# --------------------------------------------------------------------------------------


class ConvergenceData:
    """src/convergence.jl:3-23."""

    def __init__(self, nmax):
        self.niterations = nmax
        self.iterations = list(range(1, nmax + 1))
        self.relative_residual_norm = [1.0] * nmax
        self.projected_residual_norm = [1.0] * nmax
        self.orthogonality_data = [1.0] * nmax

    def resize(self, k):
        for name in ("iterations", "relative_residual_norm", "projected_residual_norm",
                     "orthogonality_data"):
            setattr(self, name, getattr(self, name)[:k])


def tensorkrylov(A_cscs, b, tol, nmax, method, cls, symmetric, tables=None,
                 A_dense=None, step_hook=None, factor=None, threads=1):
    """tensorkrylov!  (src/tensor_krylov_method.jl:36-125).
    method in {"TensorArnoldi", "TensorLanczos", "TensorLanczosReorth"}.
    factor: the per-factor state class (default Factor, NumPy); tk_ref.CFactor steps the
    factors in the C restatement instead (full-size tests: same MGS2 order, compiled).
    threads > 1 steps the factors concurrently (independent per factor, so the same
    results; useful only with CFactor, whose C calls release the GIL).
    Returns (ConvergenceData, x or None, factors)."""
    d = len(A_cscs)
    n = len(b[0])
    conv = ConvergenceData(nmax)
    b_norm = math.sqrt(np.prod([np.dot(bs, bs) for bs in b]))    # kronprodnorm
    factor = factor or Factor
    fs = [factor(A_cscs[s], b[s], nmax) for s in range(d)]
    step = {"TensorArnoldi": factor.arnoldi_mgs, "TensorLanczos": factor.lanczos_ttr,
            "TensorLanczosReorth": factor.lanczos_reorth}[method]
    for f in fs:                                                  # orthonormalize!(td, b) :53
        step(f, 1)
    btilde = [np.zeros(n) for _ in range(d)]
    for s in range(d):                                            # initialize_compressed_rhs :55
        btilde[s][0] = np.dot(fs[s].V[:, 0], b[s])
    if tables is None and symmetric:
        tables = ExpSumTables()
    r_norm = math.inf
    x = None
    pool = None
    if threads > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(threads)
    for k in range(2, nmax + 1):                                  # :63
        if pool is not None:
            list(pool.map(lambda f: step(f, k), fs))              # :66
        else:
            for f in fs:
                step(f, k)                                        # :66
        for s in range(d):                                        # update_rhs! :71
            btilde[s][k - 1] = np.dot(fs[s].V[:, k - 1], b[s])
        minor = None if A_dense is None else A_dense[:k, :k]
        lmin, lmax, kappa = spectral_update(cls, symmetric, d, n, k, minor)   # :72
        if symmetric:                                             # :73
            rank, alpha, omega = sym_expsum(tables, kappa, tol)
        else:
            rank, alpha, omega = nonsym_expsum(lmin, tol)
        Hs = [f.H[:k, :k].copy() for f in fs]
        bt = [bs[:k].copy() for bs in btilde]
        lam, Y = solve_compressed_system(Hs[0], bt, alpha, omega, lmin, symmetric)  # :76
        subdiag = [f.H[k, k - 1] for f in fs]                     # :79
        try:
            r_comp, r_norm = residualnorm(Hs, lam, Y, k, subdiag, bt, b_norm)      # :83
        except CompressedNormBreakdown:                           # :85-96
            conv.niterations = k - 1
            conv.resize(k - 1)
            return conv, None, fs
        rel = r_norm / b_norm                                     # :99
        conv.relative_residual_norm[k - 1] = rel
        conv.projected_residual_norm[k - 1] = r_comp
        conv.orthogonality_data[k - 1] = orthogonality_loss(fs[0].V, k)   # :103
        if step_hook is not None:
            step_hook(k, fs, btilde, rel)
        if rel < tol:                                             # :108-118
            # deviation: X sized by ncomponents(y), not approxdata.rank
            x = (lam.copy(), [fs[s].V[:, :k] @ Y[s] for s in range(d)])
            return conv, x, fs
    return conv, x, fs


def normalize_rhs(b):
    """LinearAlgebra.normalize!(::KronProd)  src/utils.jl:446-454 (via src/system.jl:33-37)."""
    return [bs * (1.0 / np.linalg.norm(bs)) for bs in b]
