"""CPU tests of the product's host side (no GPU): gallery, compressed-side numerics,
record bookkeeping, partitioning, the C-ABI library's exports, and the whole
tensorkrylov driver loop over a CPU stand-in device (tests/_fake_device.py)."""
import math
import os
import re
import subprocess

import numpy as np
import pytest

import tkamd
from oracle import tk_oracle as O
from tkamd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ gallery
@pytest.mark.parametrize("n", [1, 2, 3, 200, 257, 1000])
@pytest.mark.parametrize("cls", ["Laplace", "ConvDiff"])
def test_gallery_bit_identical_to_reference_assembly(n, cls):
    a = tkamd.assemble_matrix(n, cls)
    A = O.laplace_dense(n) if cls == "Laplace" else O.convdiff_dense(n)
    o = O.dense_to_csc(A)
    for x, y in zip(a, o):
        assert np.array_equal(x, y)


def test_rand_sparse_spd_generator():
    colptr, rowval, nz = tkamd.assemble_matrix(4000, "RandSparseSPD")
    n = 4000
    A = np.zeros((n, n))
    for j in range(n):
        A[rowval[colptr[j]:colptr[j + 1]], j] = nz[colptr[j]:colptr[j + 1]]
    assert np.array_equal(A, A.T)
    off = np.abs(A).sum(axis=1) - np.abs(np.diag(A))
    assert np.all(np.diag(A) > off)                     # strictly diagonally dominant -> SPD
    assert 14.5 <= len(nz) / n <= 15.0                  # 7 draws + transpose + diagonal ~ 15/row
    assert np.all(np.diff(colptr) > 0)
    # rows sorted within columns (CSC invariant)
    for j in range(0, n, 97):
        assert np.all(np.diff(rowval[colptr[j]:colptr[j + 1]]) > 0)


# ------------------------------------------------------------------ compressed side
@pytest.mark.parametrize("d,k,t", [(2, 4, 3), (3, 5, 4), (5, 7, 6), (4, 6, 1), (6, 3, 5)])
def test_residual_vectorized_matches_reference_loops(d, k, t):
    rng = np.random.default_rng(100 * d + k)
    Hs = [rng.standard_normal((k, k)) for _ in range(d)]
    Ys = [0.3 * rng.standard_normal((k, t)) for _ in range(d)]
    lam = rng.random(t)
    sub = list(rng.random(d))
    bt = [rng.standard_normal(k) for _ in range(d)]
    try:
        ro = O.residualnorm(Hs, lam, Ys, k, sub, bt, 1.3)
    except O.CompressedNormBreakdown:
        ro = None
    try:
        rp = tkamd.residualnorm(Hs, lam, Ys, k, sub, bt, 1.3)
    except tkamd.CompressedNormBreakdown:
        rp = None
    if ro is None:
        assert rp is None
    else:
        assert math.isclose(ro[0], rp[0], rel_tol=1e-12, abs_tol=1e-14)
        assert math.isclose(ro[1], rp[1], rel_tol=1e-12)


def test_compressed_breakdown_raised():
    # a residual whose compressed part is negative must raise (src/utils.jl:395)
    k, t = 3, 2
    Hs = [np.zeros((k, k))]
    Ys = [np.zeros((k, t))]
    bt = [np.zeros(k)]
    Ys[0][0, :] = 1.0
    Hs[0][:] = np.eye(k)
    with pytest.raises(tkamd.CompressedNormBreakdown):
        # Hy_norm = 0 here is impossible; use b_norm large so -2<Hy,b> dominates
        tkamd.residualnorm(Hs, np.array([1.0, 1.0]), Ys, k, [0.0], bt, 10.0)


@pytest.mark.parametrize("sym", [True, False])
def test_compressed_solve_matches_reference(sym):
    rng = np.random.default_rng(5)
    k = 9
    H = O.laplace_dense(20)[:k, :k] if sym else O.convdiff_dense(20)[:k, :k]
    bt = [rng.random(k) for _ in range(3)]
    if sym:
        rank, al, om = O.sym_expsum(O.ExpSumTables(), 437.0, 1e-9)
    else:
        rank, al, om = O.nonsym_expsum(3000.0, 1e-9)
    ap = tkamd.ApproximationData(1e-9, sym)
    ap.alpha, ap.omega = al, om
    l1, Y1 = O.solve_compressed_system(H, bt, al, om, 7.5, sym)
    l2, Y2 = tkamd.solve_compressed_system(H, bt, ap, 7.5, sym)
    assert np.allclose(l1, l2, rtol=1e-15, atol=0)
    scale = max(np.abs(y).max() for y in Y1)
    assert max(np.abs(a - b).max() for a, b in zip(Y1, Y2)) <= 1e-12 * scale


@pytest.mark.parametrize("kappa", [1.5, 2.0, 9.99, 10.0, 123.4, 999.0, 1054.2, 16534.0, 3.3e7])
@pytest.mark.parametrize("tol", [1e-9, 1e-6, 1e-12])
def test_expsum_rank_and_coefficients(kappa, tol):
    class S:
        def current(self):
            return 1.0, kappa, kappa
    ap = tkamd.ApproximationData(tol, True)
    try:
        rank, al, om = O.sym_expsum(O.ExpSumTables(), kappa, tol)
    except ValueError:
        with pytest.raises(ValueError):
            ap.update(S())
        return
    ap.update(S())
    assert ap.rank == rank
    assert np.array_equal(ap.alpha, al) and np.array_equal(ap.omega, om)


@pytest.mark.parametrize("lmin", [1.0, 37.0, 4e4, 2e5])
def test_nonsym_expsum(lmin):
    class S:
        def current(self):
            return lmin, math.inf, math.inf
    ap = tkamd.ApproximationData(1e-9, False)
    ap.update(S())
    rank, al, om = O.nonsym_expsum(lmin, 1e-9)
    assert ap.rank == rank and len(ap.alpha) == 2 * rank + 1
    assert np.allclose(ap.alpha, al, rtol=1e-15) and np.allclose(ap.omega, om, rtol=1e-15)


def test_spectral_data_laplace_and_convdiff():
    for cls, inst in (("Laplace", tkamd.SymInstance), ("ConvDiff", tkamd.NonSymInstance)):
        d, n = 4, 120
        A = tkamd.KroneckerMatrix.gallery(inst, d, n, cls)
        sp = tkamd.SpectralData(A, 30)
        dense = O.laplace_dense(n) if cls == "Laplace" else O.convdiff_dense(n)
        for k in range(2, 30):
            sp.update(d)
            ref = O.spectral_update(cls, inst == tkamd.SymInstance, d, n, k, dense[:k, :k])
            assert math.isclose(sp.lmin[k - 1], ref[0], rel_tol=1e-12)
            if inst == tkamd.SymInstance:
                assert math.isclose(sp.kappa[k - 1], ref[2], rel_tol=1e-12)


# ------------------------------------------------------------------ partition / records
@pytest.mark.parametrize("d,N", [(8, 1), (8, 2), (8, 8), (10, 8), (5, 8), (4, 3)])
def test_partition(d, N):
    parts = [tkamd.Partition(d, N, r) for r in range(N)]
    owned = [s for p in parts if not p.replica for s in p.local()]   # (replicas: N > d)
    assert owned == list(range(d))
    assert max(p.nf for p in parts) - min(p.nf for p in parts) <= 1


def test_reorth_record_bookkeeping():
    """LanczosReorth H mirror: MGS column, H[1:k-2,k] = 0, update_subdiagonals!."""
    K = 6
    td = tkamd.TensorLanczosReorth(tkamd.KroneckerMatrix(tkamd.SymInstance, [tkamd.assemble_matrix(10, 'Laplace')]), K)
    lay = td.layout
    rec = np.zeros((1, lay.m))
    j = 4
    rec[0, :j + 2] = np.arange(1, j + 3, dtype=float)   # MGS column 1..6
    rec[0, lay.flag] = 1.0
    rec[0, lay.loss] = 1e-7
    td._apply_step(j, rec)
    col = td.H[0, :, j]
    assert np.all(col[:j - 1] == 0.0)                   # rows 0..j-2 zeroed
    assert col[j - 1] == j and col[j] == j + 1          # MGS values kept
    assert col[j + 1] == j + 2 and td.H[0, j, j + 1] == j + 2


# ------------------------------------------------------------------ C ABI library
def _header_symbols():
    hdr = open(os.path.join(ROOT, "include", "tk.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return set(re.findall(r"\b(tk_[a-z_0-9]+)\s*\(", hdr))


def test_library_exports_every_declared_symbol():
    lib = os.path.join(ROOT, "tensorkrylov.jl_amd", "tkamd", "libtkhip.so")
    assert os.path.exists(lib), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (tk_[a-z_0-9]+)$", out, flags=re.M))
    declared = _header_symbols()
    assert declared == set(L.EXPORTS)
    assert declared <= exported, declared - exported
    # C linkage only: no mangled tk entry points leak from the ABI
    assert not [s for s in exported if s.startswith("_Z")]


def test_library_loads_and_fails_loudly_without_gpu():
    lib = L.lib()
    assert lib.tk_version() == 100
    assert lib.tk_record_len(50) == 110
    # (torch is deliberately not imported here: it bundles its own HIP runtime, and
    # loading it after libtkhip would put two runtimes in one process -- DESIGN.md)
    try:
        tkamd.Context(0).close()
    except tkamd.TKError as e:
        assert "no HIP device" in str(e) or "gfx950" in str(e)
    # null handles are rejected with a status, never a crash
    assert lib.tk_decomp_step(None, 0, None) != 0
    assert b"NULL" in lib.tk_last_error()


# ------------------------------------------------------------------ whole driver, CPU device stand-in
@pytest.mark.parametrize("method,cls,sym,d,K", [("TensorArnoldi", "Laplace", True, 3, 30),
                                                  ("TensorLanczosReorth", "Laplace", True, 3, 30),
                                                  ("TensorLanczos", "Laplace", True, 2, 20),
                                                  ("TensorArnoldi", "ConvDiff", False, 3, 15)])
def test_driver_host_logic_matches_oracle(method, cls, sym, d, K):
    from _fake_device import backend
    n = 200
    rng = np.random.default_rng(12345)
    b = tkamd.normalize_rhs(tkamd.random_rhs(d, n, rng))
    inst = tkamd.SymInstance if sym else tkamd.NonSymInstance
    A = tkamd.KroneckerMatrix.gallery(inst, d, n, cls)
    conv = tkamd.ConvergenceData(K)
    tkamd.tensorkrylov(conv, A, b, 1e-9, K, method, backend=backend)
    dense = O.laplace_dense(n) if cls == "Laplace" else O.convdiff_dense(n)
    conv_o, _, _ = O.tensorkrylov([O.dense_to_csc(dense)] * d, b, 1e-9, K, method, cls, sym, A_dense=dense)
    assert conv.niterations == conv_o.niterations
    ref = np.array(conv_o.relative_residual_norm)
    assert np.abs(conv.relative_residual_norm - ref).max() <= 1e-12 * ref.max()
    assert np.allclose(conv.orthogonality_data[1:], conv_o.orthogonality_data[1:], rtol=1e-6, atol=1e-15)


@pytest.mark.parametrize("method,cls,sym,d,K,tol", [("TensorArnoldi", "Laplace", True, 4, 40, 1e-9),
                                                      ("TensorLanczosReorth", "Laplace", True, 3, 30, 1e-9),
                                                      ("TensorLanczos", "Laplace", True, 3, 25, 1e-9),
                                                      ("TensorArnoldi", "ConvDiff", False, 3, 15, 1e-9),
                                                      ("TensorArnoldi", "Laplace", True, 2, 40, 1e-6)])
def test_native_iteration_driver_matches_python_loop(method, cls, sym, d, K, tol):
    """tk_solver (native record bookkeeping + compressed solve + residual + orthogonality)
    against the Python mirror of the reference's loop on the same records: the host mirror
    of H and b~ bit for bit, the trajectories to rounding, the same stopping iteration and
    the same solution factors."""
    from _fake_device import backend
    n = 200
    rng = np.random.default_rng(99)
    b = [x / np.linalg.norm(x) for x in (rng.random(n) for _ in range(d))]
    inst = tkamd.SymInstance if sym else tkamd.NonSymInstance
    A = tkamd.KroneckerMatrix.gallery(inst, d, n, cls)
    out = []
    for native in (False, True):
        conv = tkamd.ConvergenceData(K)
        x = tkamd.tensorkrylov(conv, A, [v.copy() for v in b], tol, K, method, backend=backend,
                               native=native, keep_decomposition=True)
        out.append((conv, x))
    (cp, xp), (cn, xn) = out
    assert cp.niterations == cn.niterations
    kk = cp.niterations
    assert np.array_equal(cp.decomposition.H[:, :kk + 1, :kk], cn.decomposition.H[:, :kk + 1, :kk])
    assert np.array_equal(cp.decomposition.btilde[:, :kk], cn.decomposition.btilde[:, :kk])
    ref = cp.relative_residual_norm
    assert np.abs(cn.relative_residual_norm - ref).max() <= 1e-12 * ref.max()
    assert np.allclose(cn.projected_residual_norm, cp.projected_residual_norm, rtol=1e-9, atol=1e-12)
    assert np.allclose(cn.orthogonality_data, cp.orthogonality_data, rtol=1e-9, atol=1e-15)
    assert (xp is None) == (xn is None)
    if xp is not None:
        assert np.allclose(xn.lam, xp.lam, rtol=1e-15)
        for a_, b_ in zip(xn.fmat, xp.fmat):
            assert np.abs(a_ - b_).max() <= 1e-12 * max(1.0, np.abs(b_).max())


def test_native_iteration_tables_match_python_updates():
    """IterationTables (spectral bounds and exp-sum data per k, computed up front) equal the
    per-iteration updates of the Python loop."""
    d, n, K = 3, 300, 30
    A = tkamd.KroneckerMatrix.gallery(tkamd.SymInstance, d, n, tkamd.Laplace)
    T = tkamd.compressed.IterationTables(A, K, 1e-9, d)
    spec = tkamd.SpectralData(A, K)
    apx = tkamd.ApproximationData(1e-9, True)
    off = 0
    for k in range(2, K + 1):
        spec.update(d)
        apx.update(spec)
        t = len(apx.alpha)
        assert T.rank[k - 1] == t and T.lmin[k - 1] == spec.lmin[k - 1]
        assert np.array_equal(T.alpha[off:off + t], apx.alpha) and np.array_equal(T.omega[off:off + t], apx.omega)
        off += t


# ------------------------------------------------------------------ single-matrix drivers (a12)
def test_single_matrix_drivers_host_logic():
    """arnoldi_algorithm / lanczos_algorithm / isorthonormal (src/orthogonal_bases.jl:182-284)
    over the CPU stand-in: shapes and H/V follow the reference structs; test/decompositions.jl:4-19
    properties."""
    from _fake_device import backend
    n, k = 300, 40
    A = O.laplace_dense(n)
    b = np.random.default_rng(7).random(n)
    ar = tkamd.arnoldi_algorithm(A, b, k, backend=backend)
    assert ar.V.shape == (n, k + 1) and ar.H.shape == (k + 1, k)
    f = O.Factor(O.dense_to_csc(A), b, k)
    for j in range(1, k + 1):
        f.arnoldi_mgs(j)
    assert np.array_equal(ar.H, f.H[:k + 1, :k]) and np.array_equal(ar.V, f.V[:, :k + 1])
    assert tkamd.isorthonormal(ar, k)
    la = tkamd.lanczos_algorithm(A, b, k, backend=backend)
    assert la.V.shape == (n, k) and la.H.shape == (k, k) and la.H[k - 1, k - 1] == 0.0
    assert tkamd.isorthonormal(la, k - 1)
    assert np.all(np.linalg.eigvalsh(la.H[:k - 1, :k - 1]) > 0)
    assert not tkamd.isorthonormal(np.ones((n, 3)), 3)


def test_as_csc_inputs():
    A = O.convdiff_dense(50)
    ref = O.dense_to_csc(A)
    import scipy.sparse as sp
    for x in (tkamd.as_csc(A), tkamd.as_csc(sp.csr_matrix(A)), tkamd.as_csc(ref)):
        for u, v in zip(x, ref):
            assert np.array_equal(u, v)


def test_handles_destroyed_in_any_order_without_gpu():
    """Destroy entry points accept NULL and never crash (the refcounted order-independence
    itself is exercised on the GPU by test_gpu_parity's session teardown)."""
    lib = L.lib()
    assert lib.tk_decomp_destroy(None) == 0
    assert lib.tk_matrix_destroy(None) == 0
    assert lib.tk_ctx_destroy(None) == 0


# ------------------------------------------------------------------ native compressed side edge cases
@pytest.mark.parametrize("k", [1, 2, 5, 60, 150])
@pytest.mark.parametrize("scale", [1e-4, 0.3, 3.0, 40.0])
def test_native_compressed_solve_sym_and_nonsym(k, scale):
    """tk_compressed_solve vs eigh / scipy expm across sizes and norms that select every
    Pade degree (3, 5, 7, 9, 13) and the scaling-and-squaring branch."""
    import scipy.linalg
    rng = np.random.default_rng(k)
    d, t = 3, 4
    M = rng.standard_normal((k, k))
    M /= np.linalg.norm(M, 1)                     # ||g H||_1 <= 2 * scale: degree set by scale
    bt = [rng.standard_normal(k) for _ in range(d)]

    class Ap:
        alpha = np.linspace(0.1, 2.0, t)
        omega = np.linspace(1.0, 0.2, t)
    lmin = 1.0 / scale
    for sym in (True, False):
        H = (M + M.T) / 2 if sym else M
        lam, Ys = tkamd.solve_compressed_system(H, bt, Ap, lmin, sym)
        assert np.allclose(lam, Ap.omega / lmin, rtol=1e-15)
        for j in range(t):
            g = -Ap.alpha[j] / lmin
            if sym:
                w, Q = np.linalg.eigh(np.tril(H) + np.tril(H, -1).T)
                E = (Q * np.exp(g * w)) @ Q.T
            else:
                E = scipy.linalg.expm(g * H)
            for s in range(d):
                ref = E @ bt[s]
                assert np.abs(Ys[s][:, j] - ref).max() <= 1e-11 * max(1.0, np.abs(ref).max())


def test_native_eigensolver_degenerate_spectrum():
    """Repeated eigenvalues (identity blocks, the Laplace minors' symmetry) and a diagonal
    matrix: exp(gS) b is still exact to rounding."""
    k = 40
    S = np.kron(np.eye(4), O.laplace_dense(10)[:10, :10] / 1e4)     # 4 repeated copies
    bt = [np.random.default_rng(3).standard_normal(k)]

    class Ap:
        alpha = np.array([0.5])
        omega = np.array([1.0])
    lam, Ys = tkamd.solve_compressed_system(S, bt, Ap, 1.0, True)
    w, Q = np.linalg.eigh(S)
    ref = (Q * np.exp(-0.5 * w)) @ Q.T @ bt[0]
    assert np.abs(Ys[0][:, 0] - ref).max() <= 1e-13
    D = np.diag(np.arange(1.0, k + 1))
    lam, Ys = tkamd.solve_compressed_system(D, bt, Ap, 1.0, True)
    assert np.abs(Ys[0][:, 0] - np.exp(-0.5 * np.arange(1.0, k + 1)) * bt[0]).max() <= 1e-15


def test_native_residual_breakdown_status():
    """tk_residualnorm returns TK_BREAKDOWN with r_comp set (the reference throws
    CompressedNormBreakdown, src/utils.jl:395)."""
    import ctypes
    lib = L.lib()
    d, k, t = 1, 3, 2
    H = np.eye(k).T.copy()
    Y = np.zeros((d, t, k))
    Y[0, :, 0] = 1.0
    lam = np.ones(t)
    B = np.zeros((d, k))
    rc, rn = ctypes.c_double(), ctypes.c_double()
    st = lib.tk_residualnorm(d, k, t, L.dptr(H), L.dptr(lam), L.dptr(Y), L.dptr(np.zeros(d)), L.dptr(B),
                             ctypes.c_double(10.0), ctypes.byref(rc), ctypes.byref(rn))
    assert st == L.TK_BREAKDOWN and rc.value < 0
    assert lib.tk_residualnorm(0, k, t, None, None, None, None, None, 1.0, None, None) == 1   # TK_ERR_ARG


def test_kroneckervectorize_and_kronecker_sum():
    """kroneckervectorize (src/tensor_struct.jl:361-384): vec of the Kruskal tensor, mode 1
    fastest, with redistribute!(x, 1) applied to x first; the Kronecker-sum operator
    (sum_s I kron .. A_s .. kron I) against explicit kron products."""
    import scipy.sparse as sp
    rng = np.random.default_rng(1)
    dims, t = (4, 3, 5), 2
    F = [rng.standard_normal((n, t)) for n in dims]
    lam = rng.standard_normal(t)
    x = tkamd.KruskalTensor(lam, [f.copy() for f in F])
    assert x.size() == dims
    v = tkamd.kroneckervectorize(x)
    T = np.einsum("r,ir,jr,kr->ijk", lam, *F)
    assert np.abs(v - T.ravel(order="F")).max() <= 1e-14
    assert np.allclose(x.fmat[0], F[0] * lam)            # redistribute!(x, 1) happened
    csc = [tkamd.assemble_matrix(n, "ConvDiff") for n in dims]
    A = tkamd.KroneckerMatrix(tkamd.NonSymInstance, csc, tkamd.ConvDiff)
    M = [sp.csc_matrix((c[2], c[1], c[0]), shape=(n, n)).toarray() for c, n in zip(csc, dims)]
    I3 = [np.eye(n) for n in dims]
    K = (np.kron(np.kron(I3[2], I3[1]), M[0]) + np.kron(np.kron(I3[2], M[1]), I3[0])
         + np.kron(np.kron(M[2], I3[1]), I3[0]))
    assert np.abs(K @ v - tkamd.kronecker_sum_matvec(A, v)).max() <= 1e-14 * np.abs(K @ v).max()


@pytest.mark.parametrize("cls,method,tol", [("Laplace", "TensorLanczos", 1e-2), ("ConvDiff", "TensorArnoldi", 0.3)])
def test_solution_host_logic(cls, method, tol):
    """The driver's solution output over the CPU stand-in device: the returned KruskalTensor
    equals the oracle's x, vec(x) solves the Kronecker-sum system to the reported relative
    residual, and X is sized by ncomponents(y) = 2r+1 for ConvDiff (SURVEY.md 3.2 deviation)."""
    from _fake_device import backend
    d, n = 3, 30
    sym = cls == "Laplace"
    if sym:
        xs = np.arange(1, n + 1) / (n + 1)
        b = O.normalize_rhs([xs * (1 - xs) + 0.01 * np.random.default_rng(7).random(n)] * d)
    else:
        b = O.normalize_rhs([np.random.default_rng(12345).random(n)] * d)
    A = tkamd.KroneckerMatrix.gallery(tkamd.SymInstance if sym else tkamd.NonSymInstance, d, n, cls)
    conv = tkamd.ConvergenceData(n - 1)
    x = tkamd.tensorkrylov(conv, A, [bs.copy() for bs in b], tol, n - 1, method, backend=backend)
    conv_o, x_o, _ = O.tensorkrylov([O.gallery_csc(n, cls)] * d, b, tol, n - 1, method, cls, sym,
                                    A_dense=None if sym else O.convdiff_dense(n))
    assert x is not None and x_o is not None
    assert np.abs(x.lam - x_o[0]).max() <= 1e-12 * np.abs(x_o[0]).max()
    for s in range(d):
        assert np.abs(x.fmat[s] - x_o[1][s]).max() <= 1e-12 * np.abs(x_o[1][s]).max()
    if not sym:
        assert x.ncomponents() == 3                      # 2r+1 with r = 1
    k = conv.niterations if conv.relative_residual_norm[-1] < tol else \
        [i + 1 for i, r in enumerate(conv.relative_residual_norm) if i > 0 and r < tol][0]
    vecb = b[-1]
    for s in range(d - 2, -1, -1):
        vecb = np.kron(vecb, b[s])
    res = np.linalg.norm(tkamd.kronecker_sum_matvec(A, tkamd.kroneckervectorize(x)) - vecb)
    assert abs(res - conv.relative_residual_norm[k - 1]) <= 1e-6 * conv.relative_residual_norm[k - 1]


def test_orthogonality_losses_from_one_gram():
    """orthogonality_data from one Gram matrix (deferred Gram, tk_decomp_gram): every prefix
    loss norm(G[:k,:k] - I) (src/orthogonal_bases.jl:250-257) equals the per-k form."""
    from tkamd.compressed import orthogonality_loss_from_gram, orthogonality_losses_from_gram
    rng = np.random.default_rng(0)
    V = np.linalg.qr(rng.standard_normal((500, 40)))[0] + 1e-13 * rng.standard_normal((500, 40))
    G = V.T @ V
    a = orthogonality_losses_from_gram(G)
    b = np.array([orthogonality_loss_from_gram(G, k) for k in range(1, 41)])
    assert np.allclose(a, b, rtol=1e-12, atol=0)
    assert np.allclose(a, [np.linalg.norm(V[:, :k].T @ V[:, :k] - np.eye(k)) for k in range(1, 41)], rtol=1e-6)


def test_deferred_orthogonality_after_breakdown(monkeypatch):
    """a CompressedNormBreakdown at iteration k ends the Python loop with
    orthogonality_data[2..k-1] filled, as the reference fills it on every iteration before the
    breakdown (src/tensor_krylov_method.jl:103, then :85-96) -- also with a deferred Gram."""
    import tkamd.solver as S
    from _fake_device import backend
    monkeypatch.setenv("TK_FAKE_GRAM_DEFERRED", "1")
    d, n, K, kb = 3, 80, 12, 7
    A = tkamd.KroneckerMatrix.gallery(tkamd.SymInstance, d, n, tkamd.Laplace)
    rng = np.random.default_rng(3)
    b = [x / np.linalg.norm(x) for x in (rng.random(n) for _ in range(d))]
    full = tkamd.ConvergenceData(K)
    tkamd.tensorkrylov(full, A, [x.copy() for x in b], 1e-10, K, "TensorArnoldi", backend=backend, native=False)
    real = S.residualnorm

    def breaks(Hm, lam, Ys, k, *a):
        if k == kb:
            raise tkamd.CompressedNormBreakdown(-1.0)
        return real(Hm, lam, Ys, k, *a)

    monkeypatch.setattr(S, "residualnorm", breaks)
    conv = tkamd.ConvergenceData(K)
    tkamd.tensorkrylov(conv, A, [x.copy() for x in b], 1e-10, K, "TensorArnoldi", backend=backend, native=False)
    assert conv.niterations == kb - 1
    o = np.asarray(conv.orthogonality_data)
    assert len(o) == kb - 1
    assert np.all(o[1:] > 0)
    assert np.array_equal(o[1:], np.asarray(full.orthogonality_data)[1:kb - 1])


@pytest.mark.parametrize("cls,sym", [("ConvDiff", False), ("Laplace", True)])
def test_evaluation_split_over_helpers_is_bitwise_serial(monkeypatch, cls, sym):
    """The tail iterations' evaluation split into tasks on the solver's helper threads
    (exp-sum terms, column blocks of Y = Q M, the residual's factors; tkh::ParFor) gives
    bitwise the single-thread results at every k."""
    import _fake_device as FD
    d, n, K = 5, 300, 30
    rng = np.random.default_rng(5)
    b = [x / np.linalg.norm(x) for x in (rng.random(n) for _ in range(d))]
    inst = tkamd.SymInstance if sym else tkamd.NonSymInstance
    A = tkamd.KroneckerMatrix.gallery(inst, d, n, cls)
    td = tkamd.TensorArnoldi(A, K, backend=FD.backend)
    td.orthonormalize_first(b)
    f = FD.FakeDecomposition(td, b)
    recs = [f.init()] + [f.step(j) for j in range(K)]
    T = tkamd.compressed.IterationTables(A, K, 1e-9, d)
    sv = tkamd.compressed.NativeSolver(td.method, d, K, sym, 1.0, T)
    try:
        sv.apply(-1, recs[0])
        for j in range(K):
            sv.apply(j, recs[j + 1])
        ks = [k for k in range(2, K + 1) if T.rank[k - 1] >= 1]
        assert len(ks) > 10
        out = {}
        for th in ("1", "3", "4"):
            monkeypatch.setenv("TKHIP_EVAL_THREADS", th)
            res = []
            for k in ks:
                r = sv.evaluate(k)
                lam, Y = sv.solution(k)
                res.append((np.array(r), np.array(lam), np.concatenate([np.ravel(y) for y in Y])))
            out[th] = res
        for th in ("3", "4"):
            for a_, b_ in zip(out["1"], out[th]):
                for x, y in zip(a_, b_):
                    assert np.array_equal(x, y, equal_nan=True)
    finally:
        sv.close()


def test_host_gemm_avx512_bitwise_avx2():
    import sys
    """The host GEMM's AVX-512 kernel (zmm blocks, masked row edges) and its AVX2 kernel form
    every product entry as the same k-ordered FMA chain: a nonsymmetric and a symmetric
    iteration evaluation give the same bits with either (TKHIP_HOST_AVX512=0 / 1)."""
    import json
    code = r'''
import sys, json
sys.path[:0] = [%r, %r, %r]
import numpy as np, tkamd
import _fake_device as FD
out = []
for cls, sym in (("ConvDiff", False), ("Laplace", True)):
    d, n, K = 4, 300, 26
    rng = np.random.default_rng(7)
    b = [x / np.linalg.norm(x) for x in (rng.random(n) for _ in range(d))]
    inst = tkamd.SymInstance if sym else tkamd.NonSymInstance
    A = tkamd.KroneckerMatrix.gallery(inst, d, n, cls)
    td = tkamd.TensorArnoldi(A, K, backend=FD.backend)
    td.orthonormalize_first(b)
    f = FD.FakeDecomposition(td, b)
    recs = [f.init()] + [f.step(j) for j in range(K)]
    T = tkamd.compressed.IterationTables(A, K, 1e-9, d)
    sv = tkamd.compressed.NativeSolver(td.method, d, K, sym, 1.0, T)
    sv.apply(-1, recs[0])
    for j in range(K):
        sv.apply(j, recs[j + 1])
    for k in range(2, K + 1):
        if T.rank[k - 1] < 1:
            continue
        r = sv.evaluate(k)
        lam, Y = sv.solution(k)
        out.append([float(x).hex() for x in r] + [float(x).hex() for x in np.concatenate([np.ravel(y) for y in Y])])
    sv.close()
print(json.dumps(out))
''' % (os.path.join(ROOT, "tensorkrylov.jl_amd"), ROOT, os.path.join(ROOT, "tests"))
    res = {}
    for v in ("0", "1"):
        env = dict(os.environ, TKHIP_HOST_AVX512=v)
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-2000:]
        res[v] = json.loads(p.stdout.strip().splitlines()[-1])
    assert len(res["0"]) > 10
    assert res["0"] == res["1"]


def test_orthogonality_losses_native_edges_and_lower_triangle():
    """tk_orthogonality_losses (the sum the native loop applies to the Gram it reads) reads the
    lower triangle only, in the order tk_solver_evaluate sums a tracked factor's Gram rows:
    a garbage upper triangle changes nothing; K = 1 and an exact identity give exact values;
    K = 0 is accepted."""
    import ctypes
    from tkamd import _lib as L
    from tkamd.compressed import orthogonality_losses_from_gram
    rng = np.random.default_rng(3)
    K = 23
    V = np.linalg.qr(rng.standard_normal((200, K)))[0] + 1e-9 * rng.standard_normal((200, K))
    G = V.T @ V
    Gu = np.tril(G) + np.triu(rng.standard_normal((K, K)), 1)     # upper triangle: noise
    assert np.array_equal(orthogonality_losses_from_gram(G), orthogonality_losses_from_gram(Gu))
    # the sequential sum, restated (the library contracts products into FMAs: rounding-level
    # differences only)
    acc, ref = 0.0, []
    for c in range(K):
        dd = G[c, c] - 1.0
        off = 0.0
        for i in range(c):
            off += G[c, i] * G[c, i]
        acc += dd * dd + 2.0 * off
        ref.append(math.sqrt(acc))
    assert np.allclose(orthogonality_losses_from_gram(G), np.array(ref), rtol=1e-13, atol=0)
    assert np.array_equal(orthogonality_losses_from_gram(np.eye(7)), np.zeros(7))
    assert orthogonality_losses_from_gram(np.array([[1.5]]))[0] == 0.5
    out = np.zeros(1)
    assert L.lib().tk_orthogonality_losses(0, L.dptr(out), L.dptr(out)) == 0


def test_split_wanted_only_when_node_locality_is_known(monkeypatch):
    """the evaluation split (a node-local /dev/shm mailbox) is used only when every
    rank is positively known to be on this node: LOCAL_WORLD_SIZE == WORLD_SIZE == the
    partition's rank count.  Unset variables (another launcher) or a multi-node job: unsplit."""
    from tkamd.solver import _split_wanted
    part = tkamd.Partition(4, 2, 0)
    for k in ("LOCAL_WORLD_SIZE", "WORLD_SIZE", "TKHIP_EVAL_SPLIT"):
        monkeypatch.delenv(k, raising=False)
    assert not _split_wanted(part)                      # no launcher information
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert not _split_wanted(part)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")         # two nodes, one rank each
    assert not _split_wanted(part)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert _split_wanted(part)
    monkeypatch.setenv("TKHIP_EVAL_SPLIT", "0")
    assert not _split_wanted(part)
    monkeypatch.delenv("TKHIP_EVAL_SPLIT")
    assert not _split_wanted(tkamd.Partition(4, 1, 0))  # one rank
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert not _split_wanted(part)                      # the partition is not the launcher's world
