"""Host-side tensor structures mirroring the reference's API surface.

KroneckerMatrix / KruskalTensor / TensorizedSystem / ConvergenceData / random_rhs /
assemble_matrix follow src/tensor_struct.jl, src/system.jl and src/convergence.jl of
thbake/TensorKrylov.jl (file:line cited per object).  These are small host containers;
the n-length arithmetic lives on the device (tkamd.device).
"""
import math

import numpy as np

SymInstance = "SymInstance"        # src/tensor_struct.jl:83-85
NonSymInstance = "NonSymInstance"

# MatrixGallery (src/tensor_struct.jl:18-23) -- names used as class tags
Laplace = "Laplace"
LaplaceDense = "LaplaceDense"
ConvDiff = "ConvDiff"
RandSparseSPD = "RandSparseSPD"    # build-defined generator for config C3


def _lap_coeff(n):
    # h = inv(n + 1); inv(h^2) with Julia's literal h^2 == h*h (src/tensor_struct.jl:50-51)
    h = 1.0 / (n + 1)
    return 1.0 / (h * h), h


def assemble_matrix(n, cls, c=10.0, seed=42, nnz_row=15):
    """assemble_matrix(n, class) (src/tensor_struct.jl:48-68) as 0-based CSC arrays
    (colptr, rowval, nzval), entries bit-identical to the reference's SparseMatrixCSC."""
    n = int(n)
    ch, h = _lap_coeff(n)
    if cls in (Laplace, LaplaceDense):
        # inv(h^2) * SymTridiagonal(2ones(n), -ones(n))
        j = np.arange(n)
        rows = np.stack([j - 1, j, j + 1], axis=1)
        vals = np.tile(np.array([ch * -1.0, ch * 2.0, ch * -1.0]), (n, 1))
        keep = (rows >= 0) & (rows < n)
        return _pack(rows, vals, keep, n)
    if cls == ConvDiff:
        # L + (c*inv(4h)) .* diagm(-1 => 1, 0 => 3, 1 => -5, 2 => 1)   (src/tensor_struct.jl:60-68)
        cc = c * (1.0 / (4 * h))
        j = np.arange(n)
        rows = np.stack([j - 2, j - 1, j, j + 1], axis=1)
        vals = np.tile(np.array([cc * 1.0, ch * -1.0 + cc * -5.0, ch * 2.0 + cc * 3.0,
                                 ch * -1.0 + cc * 1.0]), (n, 1))
        keep = (rows >= 0) & (rows < n)
        return _pack(rows, vals, keep, n)
    if cls == RandSparseSPD:
        return rand_sparse_spd(n, seed=seed, nnz_row=nnz_row)
    raise ValueError("unsupported matrix class %r" % (cls,))


def _pack(rows, vals, keep, n):
    counts = keep.sum(axis=1)
    colptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=colptr[1:])
    return colptr, rows[keep].astype(np.int64), vals[keep].astype(np.float64)


def rand_sparse_spd(n, seed=42, nnz_row=15):
    """Config C3 generator (defined by this build; BASELINE.json configs[3]
    "nnz/row ~ 15"): each row draws (nnz_row-1)//2 random off-diagonal columns with
    U(-1,0) values; A = (B + B')/2 doubles them, so with the diagonal a row holds
    ~nnz_row entries (14.99 at n = 2^19; duplicate draws are summed).  Diagonal =
    sum |offdiag| + 1 (SPD by strict diagonal dominance).  Returns CSC (0-based)."""
    rng = np.random.default_rng(seed)
    k = (nnz_row - 1) // 2
    r = np.repeat(np.arange(n, dtype=np.int64), k)
    c = rng.integers(0, n - 1, size=n * k, dtype=np.int64)
    c = c + (c >= r)                        # skip the diagonal
    v = -rng.random(n * k)
    # B + B' as COO, halved, duplicates summed
    rr = np.concatenate([r, c])
    cc = np.concatenate([c, r])
    vv = np.concatenate([v, v]) * 0.5
    key = cc * n + rr                       # column-major order
    order = np.argsort(key, kind="stable")
    key, vv = key[order], vv[order]
    uniq, start = np.unique(key, return_index=True)
    sums = np.add.reduceat(vv, start)
    cols, rows = uniq // n, uniq % n
    diag = np.zeros(n)
    np.add.at(diag, rows, np.abs(sums))
    diag += 1.0
    rows = np.concatenate([rows, np.arange(n)])
    cols = np.concatenate([cols, np.arange(n)])
    vals = np.concatenate([sums, diag])
    order = np.lexsort((rows, cols))
    rows, cols, vals = rows[order], cols[order], vals[order]
    colptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(colptr, cols + 1, 1)
    np.cumsum(colptr, out=colptr)
    return colptr, rows.astype(np.int64), vals


def as_csc(A):
    """0-based (colptr, rowval, nzval) of a CSC triple, a scipy.sparse matrix or a dense
    array (explicit zeros of a dense input are dropped, as sparse() does in Julia)."""
    if isinstance(A, tuple) and len(A) == 3:
        return (np.ascontiguousarray(A[0], dtype=np.int64), np.ascontiguousarray(A[1], dtype=np.int64),
                np.ascontiguousarray(A[2], dtype=np.float64))
    if hasattr(A, "tocsc"):
        S = A.tocsc()
        S.sort_indices()
        return (S.indptr.astype(np.int64), S.indices.astype(np.int64), S.data.astype(np.float64))
    D = np.asarray(A, dtype=np.float64)
    if D.ndim != 2 or D.shape[0] != D.shape[1]:
        raise ValueError("A must be square")
    n = D.shape[0]
    colptr = np.zeros(n + 1, dtype=np.int64)
    rows, vals = [], []
    for j in range(n):
        nzr = np.nonzero(D[:, j])[0]
        rows.append(nzr)
        vals.append(D[nzr, j])
        colptr[j + 1] = colptr[j] + len(nzr)
    return colptr, np.concatenate(rows).astype(np.int64), np.concatenate(vals)


def csc_leading_block(csc, k):
    """Dense A[1:k, 1:k] of a CSC matrix (for spectral data of non-Laplace classes,
    src/eigenvalues.jl:337,344-350)."""
    colptr, rowval, nzval = csc
    M = np.zeros((k, k))
    for j in range(k):
        p0, p1 = colptr[j], colptr[j + 1]
        rows = rowval[p0:p1]
        m = rows < k
        M[rows[m], j] = nzval[p0:p1][m]
    return M


class KroneckerMatrix:
    """KroneckerMatrix{matT, U} (src/tensor_struct.jl:168-231): the d coefficient
    matrices A_s of the Kronecker sum, an Instance tag and a MatrixGallery class.
    Like the reference's KroneckerMatrix{U}(d, n, class) the gallery constructor
    stores ONE matrix object d times."""

    def __init__(self, instance, mats, matrixclass=None):
        self.instance = instance
        self.M = list(mats)
        self.matrixclass = matrixclass

    @classmethod
    def gallery(cls, instance, d, n, matrixclass, **kw):
        A = assemble_matrix(n, matrixclass, **kw)
        return cls(instance, [A] * d, matrixclass)

    def __len__(self):
        return len(self.M)

    def __getitem__(self, s):
        return self.M[s]

    def dimensions(self):
        return [len(A[0]) - 1 for A in self.M]

    @property
    def symmetric(self):
        return self.instance == SymInstance


class KruskalTensor:
    """KruskalTensor{T} (src/tensor_struct.jl:283-316): lambda, factor matrices."""

    def __init__(self, lam, fmat):
        self.lam = np.asarray(lam, dtype=np.float64)
        self.fmat = list(fmat)

    def ncomponents(self):
        return len(self.lam)

    def ndims(self):
        return len(self.fmat)

    def size(self):
        """Base.size (src/tensor_struct.jl:323): the row count of every factor matrix."""
        return tuple(int(np.asarray(F).shape[0]) for F in self.fmat)

    def redistribute(self, mode):
        """redistribute!(x, mode) (src/tensor_struct.jl:325-333): column j of factor `mode`
        (0-based here) scaled by lambda[j], in place (lambda itself is left as it is)."""
        F = np.array(self.fmat[mode], dtype=np.float64)
        for j in range(self.ncomponents()):
            F[:, j] = self.lam[j] * F[:, j]
        self.fmat[mode] = F


def kroneckervectorize(x):
    """kroneckervectorize(x) (src/tensor_struct.jl:361-384): the length prod(size(x))
    vector sum_i x_d[:, i] kron ... kron (lambda_i x_1[:, i]) -- vec of the Kruskal tensor with
    the first mode running fastest.  Like the reference it first calls redistribute!(x, 1),
    so x's first factor is left scaled by lambda (call it once per tensor)."""
    x.redistribute(0)
    N = int(np.prod(x.size()))
    vecx = np.zeros(N)
    for i in range(x.ncomponents()):
        tmp = np.asarray(x.fmat[-1])[:, i]
        for j in range(x.ndims() - 2, -1, -1):
            tmp = np.kron(tmp, np.asarray(x.fmat[j])[:, i])
        vecx += tmp
    return vecx


def kronecker_sum_matvec(A, v):
    """(sum_s I kron .. kron A_s kron .. kron I) v for the Kronecker-sum operator of
    KroneckerMatrix A (the system the reference solves, src/system.jl:15-43), with v in
    kroneckervectorize's ordering: A_s acts on mode s, mode 1 fastest.  Small sizes only
    (test use: the explicit residual of a solution)."""
    import scipy.sparse as sp
    dims = A.dimensions()
    X = np.asarray(v, dtype=np.float64).reshape(dims[::-1])   # axes (d, ..., 1): mode s on axis d-1-s
    out = np.zeros_like(X)
    for s in range(len(dims)):
        colptr, rowval, nzval = A[s]
        M = sp.csc_matrix((nzval, rowval, colptr), shape=(dims[s], dims[s]))
        ax = len(dims) - 1 - s
        Xs = np.moveaxis(X, ax, 0).reshape(dims[s], -1)
        out += np.moveaxis((M @ Xs).reshape(np.moveaxis(X, ax, 0).shape), 0, ax)
    return out.ravel()


def random_rhs(d, n, rng=None):
    """random_rhs (src/system.jl:5-11): ONE rand(n) vector shared by all d slots."""
    rng = np.random.default_rng() if rng is None else rng
    bs = rng.random(n)
    return [bs for _ in range(d)]


def normalize_rhs(b):
    """LinearAlgebra.normalize!(::KronProd) (src/utils.jl:446-454): rhs[i] *= inv(norm)."""
    return [bs * (1.0 / np.linalg.norm(bs)) for bs in b]


def kronprodnorm(b):
    """src/tensor_struct.jl:271-281."""
    return math.sqrt(float(np.prod([np.dot(bs, bs) for bs in b])))


class TensorizedSystem:
    """TensorizedSystem{U} (src/system.jl:15-43); normalizes b by default."""

    def __init__(self, A, b, normalize=True):
        assert len(A) == len(b)
        assert all(dim == len(bs) for dim, bs in zip(A.dimensions(), b))
        self.d = len(A)
        self.n = A.dimensions()[0]
        self.A = A
        self.b = normalize_rhs(b) if normalize else [np.asarray(bs, dtype=np.float64) for bs in b]


class ConvergenceData:
    """ConvergenceData{T} (src/convergence.jl:3-32)."""

    def __init__(self, nmax):
        self.niterations = nmax
        self.iterations = np.arange(1, nmax + 1)
        self.relative_residual_norm = np.ones(nmax)
        self.projected_residual_norm = np.ones(nmax)
        self.orthogonality_data = np.ones(nmax)

    def resize(self, k):
        self.iterations = self.iterations[:k]
        self.relative_residual_norm = self.relative_residual_norm[:k]
        self.projected_residual_norm = self.projected_residual_norm[:k]
        self.orthogonality_data = self.orthogonality_data[:k]

    def __repr__(self):
        return ("Convergence data:\nComputations ran for %d iterations.\n"
                "Achieved relative residual norm: %s" %
                (self.niterations, self.relative_residual_norm[self.niterations - 1]))
