"""The solution tensorkrylov! returns, against the oracle and against the system itself
(VERDICT r2 "what's missing" 1).

On convergence the reference forms x = KruskalTensor(lambda, X_s = V_s[:, 1:k] Y_s)
(src/tensor_krylov_method.jl:108-118, basis_tensor_mul! src/utils.jl:478-488).  Here
tkamd.tensorkrylov runs the device steps and basis_tensor_mul! on the GPU (k_fin_vy: the
pending column's flush + V*Y in one pass) and must return the oracle's (lambda, X_s) to
1e-12; kroneckervectorize(x) (src/tensor_struct.jl:361-384) must then actually solve the
Kronecker-sum system to the relative residual the driver reported (Lemma 3.4 is exact for
x = V y; the tolerance covers the cancellation in the compressed residual).

The cases converge at tolerances the exp-sum approximation reaches at these sizes (the
reference's own recordings never reach 1e-9): Laplace d = 3, n = 30 with a
smooth right-hand side at tol 1e-2 (all three methods), and ConvDiff d = 3, n = 30 at tol 0.3
(TensorArnoldi), where Y has t = 2r+1 = 3 columns while approxdata.rank = r = 1: the
reference would size X with r columns (src/tensor_krylov_method.jl:110) and throw a
DimensionMismatch in mul! (src/utils.jl:484); the build sizes X by ncomponents(y), the
deviation pinned below.
"""
import numpy as np
import pytest

from oracle import tk_oracle as O

pytestmark = pytest.mark.gpu


def _tk():
    import tkamd
    return tkamd


def _smooth_rhs(n, d):
    xs = np.arange(1, n + 1) / (n + 1)
    b = xs * (1 - xs) + 0.01 * np.random.default_rng(7).random(n)
    return O.normalize_rhs([b] * d)


CASES = [
    ("Laplace", "TensorArnoldi", 1e-2),
    ("Laplace", "TensorLanczos", 1e-2),
    ("Laplace", "TensorLanczosReorth", 1e-2),
    ("ConvDiff", "TensorArnoldi", 0.3),
]


@pytest.mark.parametrize("cls,method,tol", CASES)
def test_returned_solution_matches_oracle_and_solves_the_system(ctx, cls, method, tol):
    tk = _tk()
    d, n = 3, 30
    nmax = n - 1
    sym = cls == "Laplace"
    if sym:
        b = _smooth_rhs(n, d)
    else:
        b = O.normalize_rhs([np.random.default_rng(12345).random(n)] * d)
    A = tk.KroneckerMatrix.gallery(tk.SymInstance if sym else tk.NonSymInstance, d, n,
                                   tk.Laplace if sym else tk.ConvDiff)
    conv = tk.ConvergenceData(nmax)
    x = tk.tensorkrylov(conv, A, [bs.copy() for bs in b], tol, nmax, method, ctx=ctx)
    Ad = None if sym else O.convdiff_dense(n)
    conv_o, x_o, _ = O.tensorkrylov([O.gallery_csc(n, cls)] * d, b, tol, nmax, method, cls, sym, A_dense=Ad)
    assert x_o is not None, "oracle did not converge: the case no longer exercises the solution path"
    assert x is not None, "device driver did not converge where the oracle did"
    k = [i + 1 for i, r in enumerate(conv_o.relative_residual_norm) if i > 0 and r < tol][0]
    assert conv.relative_residual_norm[k - 1] < tol
    assert all(r >= tol for r in conv.relative_residual_norm[1:k - 1])
    lam_o, X_o = x_o
    t = len(lam_o)
    # The Lanczos methods converge here at k = 28 of n = 30, next to the full Krylov space: plain
    # TTR has lost orthogonality there and amplifies rounding differences (reduction order, the
    # one-sweep beta formula), LanczosReorth takes MGS redos at loss ~ sqrt(eps) (test_gpu_parity
    # follows its decisions at 1e-7): their X agree with the oracle's to ~1e-12 relative, Arnoldi's
    # to 1e-13
    xtol = 1e-10 if method in ("TensorLanczos", "TensorLanczosReorth") else 1e-12
    # lambda and the factor matrices (basis_tensor_mul! on the device) vs the oracle
    assert x.ncomponents() == t and x.ndims() == d
    assert np.abs(x.lam - lam_o).max() <= 1e-12 * np.abs(lam_o).max()
    for s in range(d):
        Xs = np.asarray(x.fmat[s])
        assert Xs.shape == (n, t)
        assert np.abs(Xs - X_o[s]).max() <= xtol * np.abs(X_o[s]).max(), (s, np.abs(Xs - X_o[s]).max())
    if not sym:
        # the deviation from src/tensor_krylov_method.jl:110: X has ncomponents(y) = 2r+1
        # columns, not approxdata.rank = r
        apx = tk.ApproximationData(tol, False)
        spec = tk.SpectralData(A, nmax)
        for _ in range(k - 1):
            spec.update(d)
        apx.update(spec)
        r = apx.rank
        assert t == 2 * r + 1 and r >= 1
    # vec(x) solves the Kronecker-sum system to the reported relative residual
    vecx = tk.kroneckervectorize(x)
    vecb = b[-1]
    for s in range(d - 2, -1, -1):
        vecb = np.kron(vecb, b[s])
    res = np.linalg.norm(tk.kronecker_sum_matvec(A, vecx) - vecb) / np.linalg.norm(vecb)
    rel = conv.relative_residual_norm[k - 1]
    assert abs(res - rel) <= 1e-6 * rel, (res, rel)


def test_keep_decomposition_continues_after_native_loop(ctx):
    """after the native loop (tk_solver_run issues steps ahead of what it reads),
    a kept decomposition continues with orthonormalize(k) -- already-enqueued steps are
    collected, not re-issued -- and its H matches the oracle's."""
    tk = _tk()
    d, n, nmax = 2, 200, 12
    b = _smooth_rhs(n, d)
    A = tk.KroneckerMatrix.gallery(tk.SymInstance, d, n, tk.Laplace)
    conv = tk.ConvergenceData(nmax)
    tk.tensorkrylov(conv, A, [bs.copy() for bs in b], 1e-9, nmax, "TensorArnoldi", ctx=ctx,
                    keep_decomposition=True)
    td = conv.decomposition
    try:
        assert td.dev.next_step >= nmax - 1
        td.orthonormalize(nmax)          # step nmax-1: already issued by the native loop
        _, _, fs = O.tensorkrylov([O.gallery_csc(n, "Laplace")] * d, b, 1e-9, nmax, "TensorArnoldi",
                                  "Laplace", True)
        for s in range(d):
            ref = fs[s].H[:nmax + 1, :nmax]
            assert np.abs(td.H[s, :nmax + 1, :nmax] - ref).max() <= 1e-12 * np.abs(ref).max()
    finally:
        td.close()
