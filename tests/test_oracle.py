"""Pin the oracle (CPU restatement) to the reference's own recorded results and tests.

  * experiments/data/reproduction_data/{laplace_new,nonsym_new} (decoded to
    tests/golden/reproduction.json by tests/golden/make_golden.py)
  * test/eigenvalues.jl:5-73   (Lanczos / Sturm-sequence KAT)
  * test/eigenvalues.jl:75-100 (analytic eigenvalues == extremes of the minors)
  * test/utils.jl:188-227      (squared_tensor_entries KAT -> [1936, 1768, 1768])
  * test/decompositions.jl:4-56 (orthonormality and SPD properties)
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import tk_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "reproduction.json")))


@pytest.mark.parametrize("fname,cls,sym,method,d,K,tol", [
    ("laplace_new", "Laplace", True, "TensorLanczosReorth", 5, 51, 1e-10),
    ("laplace_new", "Laplace", True, "TensorLanczosReorth", 10, 51, 1e-10),
    ("nonsym_new", "ConvDiff", False, "TensorArnoldi", 5, 26, 1e-10),
])
def test_oracle_reproduces_recorded_trajectory(fname, cls, sym, method, d, K, tol):
    g = G[fname]
    b = np.array(g["rhs"][str(d)])
    n = 200
    A = O.laplace_dense(n) if cls == "Laplace" else O.convdiff_dense(n)
    csc = O.dense_to_csc(A)
    conv, _, _ = O.tensorkrylov([csc] * d, [b.copy() for _ in range(d)], 1e-9, K, method, cls, sym,
                                A_dense=A)
    ref = np.array(g["convergence"][str(d)]["relative_residual_norm"][:K])
    mine = np.array(conv.relative_residual_norm)
    assert conv.niterations == K
    rel = np.abs(mine[1:] - ref[1:]) / ref[1:]
    assert rel.max() <= tol, rel.max()
    # orthogonality_data: rounding noise; order of magnitude
    oref = np.array(g["convergence"][str(d)]["orthogonality_data"][:K])
    om = np.array(conv.orthogonality_data)
    assert np.all(om[1:] < 1e-12) and np.all(oref[1:] < 1e-12)


def test_recorded_rhs_is_normalized():
    for fname in ("laplace_new", "nonsym_new"):
        for d, b in G[fname]["rhs"].items():
            assert abs(np.linalg.norm(b) - 1.0) < 1e-15


def test_lanczos_sturm_kat():
    """test/eigenvalues.jl:5-73: Lanczos on Tridiagonal(-1,2,-1), n=50, v=ones/sqrt(50)."""
    n, k = 50, 5
    A = np.diag(2.0 * np.ones(n)) + np.diag(-np.ones(n - 1), 1) + np.diag(-np.ones(n - 1), -1)
    v = (1.0 / math.sqrt(n)) * np.ones(n)
    f = O.Factor(O.dense_to_csc(A), v, k + 1)
    f.lanczos_ttr(1)
    polys = [[1.0], [f.H[0, 0], -1.0]]
    for j in range(2, k + 1):
        f.lanczos_ttr(j)
        O.next_coefficients(polys, j, f.H[j - 1, j - 1], f.H[j - 1, j - 2])
    test_values = [1.0, -1.96, -0.04166666666666724, 1.9565217391304344, 0.04545454545454549,
                   -1.9523809523809523]
    for p, tv in zip(polys, test_values):
        assert math.isclose(O.evalpoly(2.0, p), tv, rel_tol=math.sqrt(np.finfo(float).eps))
    assert O.sign_changes(2.0, polys) == 3
    assert O.sign_changes(1.0, polys) == 2
    assert O.sign_changes(0.25, polys) == 1
    T = f.H[:k, :k]
    exact = np.linalg.eigvalsh(T)
    for e in exact:
        assert abs(O.evalpoly(e, polys[-1])) < 1e-13


def test_analytic_eigenvalues_match_minors():
    """test/eigenvalues.jl:75-100."""
    d, n = 3, 60
    A = O.laplace_dense(n)
    for i in range(1, n):
        ev = np.linalg.eigvalsh(A[:i, :i])
        lo, hi = O.analytic_eigenvalues(d, n, i)
        assert math.isclose(lo, ev.min() * d, rel_tol=1e-9)
        assert math.isclose(hi, ev.max() * d, rel_tol=1e-9)


def test_squared_tensor_entries_kat():
    """test/utils.jl:188-227."""
    Y = [np.array([[2.0, 1.0], [1.0, 2.0]]), np.array([[3.0, 4.0], [3.0, 4.0]]),
         np.array([[2.0, 2.0], [2.0, 2.0]])]
    lam = np.ones(2)
    Ly = [np.tril(y.T @ y) for y in Y]
    Lam = np.tril(np.outer(lam, lam))
    out = []
    for s in range(3):
        Gam = np.tril(np.outer(Y[s][1, :], Y[s][1, :])) * Lam
        out.append(O.squared_tensor_entries([Ly[q] for q in range(3) if q != s], Gam))
    manual = [np.linalg.norm(v) ** 2 for v in ([22.0] * 4, [20.0, 20, 22, 22], [20.0, 20, 22, 22])]
    assert np.allclose(out, manual) and np.allclose(out, [1936, 1768, 1768])


def test_arnoldi_lanczos_orthonormal_large():
    """test/decompositions.jl:4-19 (n=1000, k=500) on the C restatement."""
    from oracle import tk_ref
    n, k = 1000, 500
    h = 1.0 / (n + 1)
    A = (1.0 / (h * h)) * (np.diag(2.0 * np.ones(n)) - np.diag(np.ones(n - 1), 1) - np.diag(np.ones(n - 1), -1))
    b = np.random.default_rng(12345).random(n)
    f = tk_ref.RefFactor(O.dense_to_csc(A), b, k)
    for j in range(k):
        f.arnoldi_step(j)
    assert O.orthogonality_loss(f.V, k) < 1e-8


def test_tensor_decompositions_properties():
    """test/decompositions.jl:21-56: d=5, n=200, k=2..50: T_k SPD, bases orthonormal."""
    d, n, k = 5, 200, 50
    csc = O.gallery_csc(n, "Laplace")
    rng = np.random.default_rng(12345)
    for _ in range(d):
        b = rng.random(n)
        fa = O.Factor(csc, b, k)
        fl = O.Factor(csc, b, k)
        for j in range(1, k + 1):
            fa.arnoldi_mgs(j)
            fl.lanczos_ttr(j)
        assert np.all(np.linalg.eigvalsh(fl.H[:k, :k]) > 0)
        assert O.orthogonality_loss(fa.V, k) < 1e-8
        assert O.orthogonality_loss(fl.V, k) < 1e-8


def test_c_and_numpy_restatements_agree():
    from oracle import tk_ref
    for cls in ("Laplace", "ConvDiff"):
        csc = O.gallery_csc(300, cls)
        b = np.random.default_rng(2).random(300)
        fc = tk_ref.RefFactor(csc, b, 40)
        fo = O.Factor(csc, b, 40)
        for j in range(40):
            fc.arnoldi_step(j)
            fo.arnoldi_mgs(j + 1)
        scale = np.abs(fo.H).max()
        assert np.abs(fc.H[:41, :40] - fo.H[:41, :40]).max() <= 1e-13 * scale
        assert np.abs(fc.V - fo.V).max() <= 1e-12
        x = np.random.default_rng(3).standard_normal(300)
        assert np.array_equal(fc.matvec(x), O.csc_matvec(csc, x))


def test_all_cores_baseline_sweep_matches_port():
    """bench.py's all-cores CPU baseline (rows over OpenMP threads) computes the same MGS2
    sweep as the 1-core port: only the dot reduction order differs (rounding level)."""
    from oracle import tk_ref
    import tkamd
    n, K = 6000, 30
    for cls in ("Laplace", "RandSparseSPD"):
        csc = tkamd.assemble_matrix(n, cls)
        b = np.random.default_rng(5).random(n)
        b /= np.linalg.norm(b)
        f = tk_ref.RefFactor(csc, b, K)
        for j in range(K):
            f.arnoldi_step(j)
        csr = tk_ref.csc_to_csr(csc)
        V1, H1 = tk_ref.arnoldi_sweep_omp(csr, b, K, threads=1)
        assert np.array_equal(V1, f.V) and np.array_equal(H1[:K + 1, :K], f.H[:K + 1, :K])
        V, H = tk_ref.arnoldi_sweep_omp(csr, b, K, threads=4)
        scale = np.abs(f.H).max()
        assert np.abs(H[:K + 1, :K] - f.H[:K + 1, :K]).max() <= 1e-12 * scale
        assert np.abs(V - f.V).max() <= 1e-12


def test_oracle_driver_with_c_factors_matches_numpy_factors():
    """tk_oracle.tensorkrylov(..., factor=tk_ref.CFactor) -- the form the full-size C2
    north-star test uses -- gives the NumPy-factor driver's trajectory (the two factor
    restatements agree to rounding, src/orthogonal_bases.jl:15-37)."""
    from oracle import tk_ref
    d, n, K = 4, 200, 30
    csc = O.gallery_csc(n, "Laplace")
    rng = np.random.default_rng(11)
    b = O.normalize_rhs([rng.random(n) for _ in range(d)])
    c_np, _, _ = O.tensorkrylov([csc] * d, b, 1e-9, K, "TensorArnoldi", "Laplace", True)
    c_c, _, fs = O.tensorkrylov([csc] * d, b, 1e-9, K, "TensorArnoldi", "Laplace", True,
                                factor=tk_ref.CFactor)
    assert isinstance(fs[0], tk_ref.CFactor)
    assert c_np.niterations == c_c.niterations
    r_np = np.array(c_np.relative_residual_norm[1:])
    r_c = np.array(c_c.relative_residual_norm[1:])
    assert np.abs(r_c - r_np).max() <= 1e-11 * r_np.max()
    assert np.abs(np.array(c_c.orthogonality_data[1:]) - np.array(c_np.orthogonality_data[1:])).max() <= 1e-13
