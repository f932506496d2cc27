"""The north-star criterion at the headline workload, through the exact timed path.

BASELINE.json north_star: "residual within 1e-10 of CPU reference" on d = 8, n_s = 2^20
tridiagonal Laplacian (configs[2], C2), TensorArnoldi, K = nmax = 50.

  * test_c2_bench_path_parity: the calls bench.py's timed step makes, in its order and with
    its defaults (bench.py sweep(): tk_decomp_init without a record, tk_decomp_sweep(0, 50)
    over untracked factors in two factor groups with the step bookkeeping riding in the next
    launch, tk_decomp_basis_mul at the solver's t = 17 -- the fused flush + V*Y, k_fin_vy --
    and factor 1's deferred Gram SYRK), repeated as the bench repeats them (a warm-up sweep,
    then the measured one on the same handle).  Every factor's H, b-tilde and V, every X_s
    and G are compared with the C restatement of MGS2 (oracle/tk_ref.c,
    src/orthogonal_bases.jl:15-37; src/utils.jl:478-488; src/orthogonal_bases.jl:231-257)
    on the bench's seeded inputs.
  * test_c2_tensorkrylov_relres_vs_oracle: tkamd.tensorkrylov (the native pipelined driver
    over the device steps) against the oracle's tensorkrylov! restatement
    (src/tensor_krylov_method.jl:36-125) whose factors the C restatement steps: relative
    residuals within 1e-10 relative at every k (the north-star bound), the same iteration
    count, orthogonality_data within 1e-12 absolute.

  * test_c2_tensorkrylov_converged_solution_vs_oracle: the convergence branch at C2 scale
    (tol 0.4: both stop at k = 7) -- the returned (lambda, X_s) against the oracle's.

The oracle's tol = 1e-9 run is shared by the first two tests (module fixture: 8 full MGS2 sweeps at n = 2^20,
about 10 s over 8 host threads).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D, N, K = 8, 1 << 20, 50


def _bench_rhs(n, d):
    """bench.py's b_s: U(0,1) with seed 1000+s, normalized."""
    out = []
    for s in range(d):
        b = np.random.default_rng(1000 + s).random(n)
        out.append(b / np.linalg.norm(b))
    return out


@pytest.fixture(scope="module")
def c2_oracle():
    """The oracle's tensorkrylov! on C2 with the C restatement stepping the factors."""
    import tkamd as tk
    from oracle import tk_oracle as O
    from oracle import tk_ref
    csc = tk.assemble_matrix(N, "Laplace")
    bs = _bench_rhs(N, D)
    conv_o, x_o, fs = O.tensorkrylov([csc] * D, bs, 1e-9, K, "TensorArnoldi", "Laplace", True,
                                     factor=tk_ref.CFactor, threads=8)
    assert x_o is None and conv_o.niterations == K        # C2 does not converge within 50 steps
    yield csc, bs, conv_o, fs
    del fs


def _bench_t_rank(tk, csc):
    """bench.py: the exp-sum rank the solver uses at k = K (Laplace: kappa independent of n)."""
    spec = tk.SpectralData(tk.KroneckerMatrix("SymInstance", [csc] * D, "Laplace"), K)
    for _ in range(K - 1):
        spec.update(D)
    apx = tk.ApproximationData(1e-9, True)
    apx.update(spec)
    return len(apx.omega)


def test_c2_bench_path_parity(ctx, c2_oracle):
    import tkamd as tk
    csc, bs, _, fs = c2_oracle
    lay = tk._lib.RecordLayout(K)
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, D, 0, [A] * D, bs, K, n=N)
    # the bench's configuration, not a test-only one
    assert dev.arnoldi_sweeps == 1 and dev.gram_deferred and dev.factor_groups == 2
    t = _bench_t_rank(tk, csc)
    assert t == 17
    rng = np.random.default_rng(7)
    Ys = [rng.standard_normal((K, t)) for _ in range(D)]
    X = G = None
    for rep in range(2):                  # bench.py: warm-up sweep(s), then the timed ones
        last = rep == 1
        dev.init(False)
        dev.sweep(0, K)
        X = dev.basis_mul(K, Ys, want=last)
        G = dev.gram(0, K, want=last)
    recs = dev.records(0, K + 2)          # slot 0: init; slot j+1: step j; K+1: the flush
    for f in range(D):
        ref = fs[f]
        Hr, Vr = ref.H[:K + 1, :K], ref.V[:, :K + 1]
        Hd = np.zeros((K + 1, K))
        bt = np.full(K + 1, np.nan)
        for j in range(K):
            Hd[:j + 2, j] = recs[j + 1][f, lay.H:lay.H + j + 2]
        for r in recs:
            c = int(r[f, lay.col])
            if 0 <= c <= K:
                bt[c] = r[f, lay.bt]
        assert not np.isnan(bt).any()      # every column's b-tilde came back in a record
        scale = np.abs(Hr).max()
        eH = np.abs(Hd - Hr).max() / scale
        eB = np.abs(bt - Vr.T @ bs[f]).max()
        V = dev.basis(f, 0, K + 1)
        eV = np.abs(V - Vr).max()
        XR = V[:, :K] @ Ys[f]
        eX = np.abs(X[f] - XR).max() / np.abs(XR).max()
        eXo = np.abs(X[f] - Vr[:, :K] @ Ys[f]).max() / np.abs(XR).max()
        print("C2 bench path factor %d: H %.2e bt %.2e V %.2e X(dev V) %.2e X(oracle V) %.2e"
              % (f, eH, eB, eV, eX, eXo))
        assert eH <= 1e-12                 # H: 1e-12 relative to max|H|
        assert eB <= 1e-13                 # b-tilde: 1e-13 absolute
        assert eV <= 1e-12                 # V: 1e-12 absolute (unit columns)
        assert eX <= 1e-13                 # X_s = V_s Y_s on the device basis: 1e-13 relative
        assert eXo <= 1e-11                # ... and on the oracle's basis (V within 1e-12)
        if f == 0:
            GR = Vr[:, :K].T @ Vr[:, :K]
            eG = np.abs(G - GR).max()
            print("C2 bench path factor 0 Gram: %.2e (||G - I|| %.2e)" % (eG, np.linalg.norm(G - np.eye(K))))
            assert eG <= 1e-12             # G: 1e-12 absolute (entries O(1) on the diagonal)
        del V, XR
    dev.close()
    A.close()


def test_c2_tensorkrylov_relres_vs_oracle(ctx, c2_oracle):
    import tkamd as tk
    csc, bs, conv_o, _ = c2_oracle
    kron = tk.KroneckerMatrix("SymInstance", [csc] * D, "Laplace")
    conv = tk.ConvergenceData(K)
    x = tk.tensorkrylov(conv, kron, [b.copy() for b in bs], 1e-9, K, "TensorArnoldi", ctx=ctx)
    assert x is None
    assert conv.niterations == conv_o.niterations == K
    ref = np.array(conv_o.relative_residual_norm)
    got = np.asarray(conv.relative_residual_norm)
    rel = np.abs(got[1:] - ref[1:]) / ref[1:]
    eo = np.abs(np.asarray(conv.orthogonality_data[1:]) - np.array(conv_o.orthogonality_data[1:])).max()
    print("C2 tensorkrylov: relres rel err max %.2e (final %.6f vs %.6f), orthogonality %.2e"
          % (rel.max(), got[-1], ref[-1], eo))
    assert rel.max() <= 1e-10              # the north-star bound: residual within 1e-10
    assert eo <= 1e-12


def test_c2_tensorkrylov_converged_solution_vs_oracle(ctx):
    """The convergence branch (src/tensor_krylov_method.jl:108-118) at C2 scale, which the
    tol = 1e-9 runs above never reach: at tol 0.4 the oracle stops at k = 7 (relres 0.3811 after
    0.4441 and 0.4513 -- margins of ~5 %, far beyond the 1e-10 agreement) and returns
    x = (lambda, X_s = V_s[:, 1:k] Y_s) with 2^20 rows per factor (t = 2 exp-sum terms).  The
    device driver must stop at the same k with the same residual trajectory (1e-10 relative) and
    return lambda to 1e-12 and every X_s to 1e-11 relative (basis_tensor_mul! on the device)."""
    import tkamd as tk
    from oracle import tk_oracle as O
    from oracle import tk_ref
    tol = 0.4
    csc = tk.assemble_matrix(N, "Laplace")
    bs = _bench_rhs(N, D)
    conv_o, x_o, fs = O.tensorkrylov([csc] * D, bs, tol, K, "TensorArnoldi", "Laplace", True,
                                     factor=tk_ref.CFactor, threads=8)
    del fs
    assert x_o is not None
    ref = np.array(conv_o.relative_residual_norm)
    k0 = [i + 1 for i, r in enumerate(ref) if i > 0 and r < tol][0]
    assert k0 == 7
    kron = tk.KroneckerMatrix("SymInstance", [csc] * D, "Laplace")
    conv = tk.ConvergenceData(K)
    x = tk.tensorkrylov(conv, kron, [b.copy() for b in bs], tol, K, "TensorArnoldi", ctx=ctx)
    assert x is not None, "the device driver did not converge where the oracle did"
    got = np.asarray(conv.relative_residual_norm)
    assert got[k0 - 1] < tol and all(r >= tol for r in got[1:k0 - 1])
    rel = np.abs(got[1:k0] - ref[1:k0]) / ref[1:k0]
    lam_o, X_o = x_o
    assert x.ncomponents() == len(lam_o) and x.ndims() == D
    el = np.abs(np.asarray(x.lam) - lam_o).max() / np.abs(lam_o).max()
    eX = max(np.abs(np.asarray(x.fmat[s]) - X_o[s]).max() / np.abs(X_o[s]).max() for s in range(D))
    print("C2 converged at k = %d: relres rel err max %.2e, lambda %.2e, X %.2e" % (k0, rel.max(), el, eX))
    assert rel.max() <= 1e-10
    assert el <= 1e-12
    assert eX <= 1e-11
