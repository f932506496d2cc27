"""orthogonality_loss's Gram matrix as one MFMA SYRK (tk_decomp_gram, k_gram) and the deferred
orthogonality_data of factor 1 built from it (src/orthogonal_bases.jl:231-257,
src/tensor_krylov_method.jl:103).

G = V[:, :k]' V[:, :k] on v_mfma_f64_16x16x4f64 must equal the host product of the basis the
device holds (entries are O(1) on the diagonal and O(eps) off it: absolute 1e-14 at n = 5000,
1e-13 at n = 2^20, where each entry sums 2^20 products); k covers every column-group layout
(even/odd groups, 16-column runs, a tail of 1..4 columns on the VALU) and odd k exercises the
masked last column of a pair.  The driver's orthogonality_data with
a deferred Gram (TensorLanczos' default) must be rounding noise of the same size as with a
Gram row per step, and the rest of the trajectory bitwise the same (TensorArnoldi) or equal to
rounding (TensorLanczos, whose gram-free step is another kernel, k_lan_1w).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tk():
    import tkamd
    return tkamd


@pytest.mark.parametrize("method", [0, 1])
def test_gram_matches_host_product(ctx, method):
    tk = _tk()
    n, K, d = 5000, 63, 2
    csc = tk.assemble_matrix(n, "Laplace")
    rng = np.random.default_rng(21)
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, method, d, 0, [A] * d, bs, K)
    dev.init(False)
    dev.sweep(0, K)
    # every column-group layout of k_gram: even/odd groups only (k <= 32), a VALU tail of
    # 1..4 columns (33..36, 49..52), a padded 16-column group (37..48, 53..64)
    for k in (1, 2, 7, 31, 32, 33, 34, 35, 36, 37, 40, 47, 48, 49, 50, 51, 52, 53, 63, 64):
        G = dev.gram(1, k)
        V = dev.basis(1, 0, k)
        ref = V.T @ V
        assert G.shape == (k, k)
        assert np.array_equal(G, G.T)
        assert np.abs(G - ref).max() <= 1e-14, (k, np.abs(G - ref).max())
    # bitwise reproducible
    assert np.array_equal(dev.gram(0, 50), dev.gram(0, 50))
    dev.close()
    A.close()


def test_gram_full_size(ctx):
    """n = 2^20 (the C2 factor size), k = 51."""
    tk = _tk()
    n, K = 1 << 20, 50
    csc = tk.assemble_matrix(n, "Laplace")
    b = np.random.default_rng(1000).random(n)
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, 0, 1, 0, [A], [b / np.linalg.norm(b)], K)
    dev.init(False)
    dev.sweep(0, K)
    G = dev.gram(0, K + 1)
    V = dev.basis(0, 0, K + 1)
    ref = V.T @ V
    assert np.abs(G - ref).max() <= 1e-13, np.abs(G - ref).max()
    assert np.abs(G - np.eye(K + 1)).max() <= 1e-12          # the basis is orthonormal
    dev.close()
    A.close()


@pytest.mark.parametrize("method", ["TensorArnoldi", "TensorLanczos"])
def test_deferred_orthogonality_data(ctx, method, monkeypatch):
    tk = _tk()
    d, n, K = 3, 4000, 40
    A = tk.KroneckerMatrix.gallery(tk.SymInstance, d, n, tk.Laplace)
    b = tk.normalize_rhs(tk.random_rhs(d, n, np.random.default_rng(12345)))
    out = {}
    for mode in ("rows", "deferred"):
        monkeypatch.setenv("TKHIP_GRAM", mode)
        conv = tk.ConvergenceData(K)
        tk.tensorkrylov(conv, A, [x.copy() for x in b], 1e-9, K, method, ctx=ctx, keep_decomposition=True)
        assert conv.decomposition.dev.gram_deferred == (mode == "deferred")
        conv.decomposition.close()
        out[mode] = conv
    r, q = out["rows"], out["deferred"]
    if method == "TensorArnoldi":
        assert np.array_equal(r.relative_residual_norm, q.relative_residual_norm)
        assert np.array_equal(r.projected_residual_norm, q.projected_residual_norm)
    else:
        # without a Gram row the Lanczos step runs as k_lan_1w (wide windows): its dots are
        # summed in another order than k_lan_1s', so alpha and beta differ in the last bits
        for a_, b_ in ((r.relative_residual_norm, q.relative_residual_norm),
                       (r.projected_residual_norm, q.projected_residual_norm)):
            a_, b_ = np.asarray(a_[1:]), np.asarray(b_[1:])
            assert np.abs(a_ - b_).max() <= 1e-9 * np.abs(a_).max(), np.abs(a_ - b_).max()
    o1, o2 = np.asarray(r.orthogonality_data[1:]), np.asarray(q.orthogonality_data[1:])
    assert np.all(np.isfinite(o2))
    if method == "TensorArnoldi":
        assert np.all(o1 < 1e-12) and np.all(o2 < 1e-12)
    # the same Gram entries summed in another order: each differs by ~1e-15, the norm over
    # k^2 entries by at most ~k 1e-14
    assert np.abs(o1 - o2).max() <= 1e-12, np.abs(o1 - o2).max()


@pytest.mark.parametrize("method,K", [("TensorArnoldi", 32), ("TensorLanczos", 32), ("TensorArnoldi", 31)])
def test_gram_ahead_identical(ctx, method, K):
    """tk_decomp_gram_ahead: the native loop launches factor 1's Gram right behind its last
    step (over the columns already written), and the driver's tk_decomp_gram then reads that
    result.  A run to nmax (no convergence) gives orthogonality_data bitwise equal to the Gram
    taken at the end (TKHIP_GRAM_AHEAD=0, read once per process: a subprocess).  K = 31 ends on
    an even step whose column is still buffered: the Gram launched ahead covers 30 columns and
    the driver's 31-column Gram is launched as before."""
    import json
    import os
    import subprocess
    import sys
    code = r'''
import json, sys
sys.path[:0] = %r
import numpy as np
import tkamd as tk
ctx = tk.Context(0)
d, n, K = 3, 4000, %d
A = tk.KroneckerMatrix.gallery(tk.SymInstance, d, n, tk.Laplace)
b = tk.normalize_rhs(tk.random_rhs(d, n, np.random.default_rng(4)))
conv = tk.ConvergenceData(K)
tk.tensorkrylov(conv, A, b, 1e-13, K, "%s", ctx=ctx)
print(json.dumps({"niter": conv.niterations, "orth": list(map(float, conv.orthogonality_data))}))
''' % (sys.path, K, method)
    out = {}
    for v in ("1", "0"):
        env = dict(os.environ, TKHIP_GRAM_AHEAD=v)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        out[v] = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["1"]["niter"] == out["0"]["niter"] == K
    assert out["1"]["orth"] == out["0"]["orth"]
    assert all(0 < x < 1e-10 for x in out["1"]["orth"][1:]) or method == "TensorLanczos"


def test_gram_ahead_converged_within_rounding(ctx):
    """when the run converges before nmax, the Gram launched behind the last
    issued step covers more columns than the converged k, and orthogonality_data comes from
    the leading block of that larger SYRK -- whose k_gram configuration groups the columns
    differently (a column in the VALU tail at one k sits in an MFMA group at the other), so
    the sums round differently: equal to TKHIP_GRAM_AHEAD=0 within 1e-13, not bitwise (the
    non-converging runs above are bitwise).  Laplace d = 3, n = 30, a shared U(0,1) RHS at tol
    0.3: converges at k = 12 of nmax = 29."""
    import json
    import os
    import subprocess
    import sys
    code = r'''
import json, sys
sys.path[:0] = %r
import numpy as np
import tkamd as tk
ctx = tk.Context(0)
n, d, tol = 30, 3, 0.3
b0 = np.random.default_rng(777).random(n)
b0 = b0 / np.linalg.norm(b0)
A = tk.KroneckerMatrix.gallery(tk.SymInstance, d, n, tk.Laplace)
conv = tk.ConvergenceData(n - 1)
x = tk.tensorkrylov(conv, A, [b0.copy() for _ in range(d)], tol, n - 1, "TensorArnoldi", ctx=ctx)
rel = np.asarray(conv.relative_residual_norm)
kend = int(np.nonzero(rel[1:] < tol)[0][0]) + 2 if x is not None else n - 1
print(json.dumps({"kend": kend, "conv": x is not None, "orth": list(map(float, conv.orthogonality_data))}))
''' % (sys.path,)
    out = {}
    for v in ("1", "0"):
        env = dict(os.environ, TKHIP_GRAM_AHEAD=v)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        out[v] = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["1"]["conv"] and out["0"]["conv"]
    k = out["1"]["kend"]
    assert out["0"]["kend"] == k and 4 <= k < 20        # well before nmax = 29
    o1, o0 = np.array(out["1"]["orth"][1:k]), np.array(out["0"]["orth"][1:k])
    assert np.all(np.isfinite(o1)) and np.abs(o1 - o0).max() <= 1e-13
