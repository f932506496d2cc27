"""GPU parity at the BASELINE.json workload sizes: every kernel variant the bench runs on C1-C4 is checked
here at exactly the bench's n, d and K, through the C ABI, against the C restatement of
the reference (oracle/tk_ref.c: CSC-scatter SpMV + MGS2 / TTR in the reference's order,
src/orthogonal_bases.jl:15-67), on the same seeded inputs.

  * C2: d = 8, n = 2^20 Laplace, K = 50, all 8 factors (the headline bench workload).
  * C1: d = 4, n = 2^18 Laplace, K = 50, all 4 factors (one-sweep Arnoldi; its window
    count and reduce-partial count differ from C2's).
  * C3: d = 5, n = 2^19 random sparse SPD (~15 nnz/row, SELL-256 storage, two-sweep
    CGS2), K = 50, two factors; plus a TTR Lanczos run at the same size (trajectory while
    orthonormal, step-by-step shadowing for all 50 steps).
  * C4: d = 10, n = 2^17 convection-diffusion (src/tensor_struct.jl:60-68), K = 50,
    all 10 factors (one-sweep Arnoldi), plus V*Y at the solver's t = 3 against V @ Y.

Tolerances (each at its assert): H 1e-12 relative to max|H|, V 1e-12 absolute (unit
columns), b-tilde 1e-13 absolute (an n-term dot carries ~sqrt(n) eps on both sides),
Arnoldi relation A V_K = V_{K+1} Hbar_K within 1e-11 max|H|, orthonormality of the
device Gram rows within 1e-12 (Frobenius), V*Y 1e-13 relative.
"""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


def _tk():
    import tkamd
    return tkamd


def _bench_rhs(n, d):
    """bench.py's inputs: b_s ~ U(0,1) with seed 1000+s, normalized."""
    out = []
    for s in range(d):
        b = np.random.default_rng(1000 + s).random(n)
        out.append(b / np.linalg.norm(b))
    return out


def _spm(csc):
    n = len(csc[0]) - 1
    return sp.csc_matrix((csc[2], csc[1], csc[0]), shape=(n, n))


def _check_arnoldi(ctx, cls, n, d, K, check, expect_sweeps, expect_format=None, vy_t=None):
    """Run d factors of the bench workload on the device (all in one decomposition, as the
    bench does), then compare the factors listed in `check` with the C oracle."""
    from oracle import tk_ref
    tk = _tk()
    csc = tk.assemble_matrix(n, cls)
    bs = _bench_rhs(n, d)
    A = tk.DeviceMatrix(ctx, csc)
    if expect_format is not None:
        assert A.format == expect_format
    dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, d, 0, [A] * d, bs, K, track_all_gram=True)
    assert dev.arnoldi_sweeps == expect_sweeps
    lay = tk._lib.RecordLayout(K)
    recs = [dev.init()] + [dev.step(j) for j in range(K)] + [dev.flush()]
    worst = {}
    for f in check:
        b = bs[f]
        ref = tk_ref.RefFactor(csc, b, K)
        for j in range(K):
            ref.arnoldi_step(j)
        Hd = np.zeros((K + 1, K))
        for j in range(K):
            Hd[:j + 2, j] = recs[j + 1][f, :j + 2]
        scale = np.abs(ref.H[:K + 1, :K]).max()
        eH = np.abs(Hd - ref.H[:K + 1, :K]).max() / scale
        V = dev.basis(f, 0, K + 1)
        eV = np.abs(V - ref.V[:, :K + 1]).max()
        G = np.zeros((K + 1, K + 1))
        bt = np.zeros(K + 1)
        for r in recs:
            c = int(r[f, lay.col])
            if c >= 0:
                G[c, :c + 1] = r[f, lay.gram:lay.gram + c + 1]
                bt[c] = r[f, lay.bt]
        eB = np.abs(bt - ref.V[:, :K + 1].T @ b).max()
        Gs = np.tril(G) + np.tril(G, -1).T
        eG = np.linalg.norm(Gs - np.eye(K + 1))
        AV = _spm(csc) @ V[:, :K]
        eR = np.abs(AV - V @ Hd).max() / scale
        worst[f] = (eH, eV, eB, eG, eR)
        print("%s n=%d factor %d: H %.2e V %.2e bt %.2e gram %.2e arnoldi-rel %.2e"
              % (cls, n, f, eH, eV, eB, eG, eR))
        assert eH <= 1e-12                    # H: 1e-12 relative
        assert eV <= 1e-12                    # V: 1e-12 absolute
        assert eB <= 1e-13                    # btilde: 1e-13 absolute
        assert eG <= 1e-12                    # orthonormality (device Gram rows)
        assert eR <= 1e-11                    # Arnoldi relation, relative to max|H|
        del ref, AV
        if vy_t is not None:
            rng = np.random.default_rng(100 + f)
            Y = rng.standard_normal((K, vy_t))
            Ys = [Y if g == f else np.zeros((K, vy_t)) for g in range(d)]
            X = dev.basis_mul(K, Ys)[f]
            XR = V[:, :K] @ Y
            assert np.abs(X - XR).max() <= 1e-13 * max(1.0, np.abs(XR).max())   # V*Y: 1e-13 rel
        del V
    dev.close()
    A.close()
    return worst


def test_c2_laplace_2p20_all_8_factors(ctx):
    """C2 (BASELINE.json configs[2], the bench's headline workload): d = 8, n_s = 2^20 Laplace,
    K = 50, all eight factors stepped in one decomposition exactly as bench.py does and every
    one of them checked against the C oracle (C2 was checked with 2 factors)."""
    _check_arnoldi(ctx, "Laplace", 1 << 20, 8, 50, check=range(8), expect_sweeps=1)


def test_c1_laplace_2p18_all_factors(ctx):
    """C1 (BASELINE.json configs[1]): d = 4, n_s = 2^18 Laplace, K = 50, every factor."""
    _check_arnoldi(ctx, "Laplace", 1 << 18, 4, 50, check=range(4), expect_sweeps=1)


def test_c1_laplace_2p18_cgs2(ctx, monkeypatch):
    """C1 through the two-sweep CGS2 kernels (what non-banded storage and steps beyond the
    register row run), two factors."""
    monkeypatch.setenv("TKHIP_ARNOLDI", "cgs2")
    _check_arnoldi(ctx, "Laplace", 1 << 18, 4, 50, check=(0, 3), expect_sweeps=2)


def test_c3_rand_sparse_spd_2p19_arnoldi(ctx):
    """C3 (configs[3]): d = 5, n_s = 2^19 random sparse SPD at ~15 nnz/row in SELL-256,
    K = 50 (two-sweep CGS2); factors 0 and 4 checked, all five stepped."""
    tk = _tk()
    csc = tk.assemble_matrix(1 << 19, "RandSparseSPD")
    assert 14.5 <= len(csc[2]) / (1 << 19) <= 15.0
    _check_arnoldi(ctx, "RandSparseSPD", 1 << 19, 5, 50, check=(0, 4), expect_sweeps=2,
                   expect_format=-2)


def test_c3_rand_sparse_spd_2p19_lanczos(ctx):
    """C3's SPD matrix through TTR Lanczos (src/orthogonal_bases.jl:39-67), K = 50.

    Plain TTR loses orthogonality once a Ritz value converges (here within ~15 steps: the
    random matrix's extreme eigenvalues are isolated); from then on the recurrence amplifies
    any rounding difference, so two correct implementations that sum dots in different
    orders drift apart (measured: 3e-4 relative by step 50).  Parity is therefore checked
      * step by step for all 50 steps ("shadowing"): the C oracle's step j, started from the
        device's v_{j-1}, v_j, beta_{j-1}, reproduces the device's alpha_j, beta_j, v_{j+1};
      * as a whole trajectory while the oracle's basis is still orthonormal
        (||V'V - I|| <= 1e-10);
      * by the three-term relation on the device basis."""
    from oracle import tk_ref
    tk = _tk()
    n, K, d = 1 << 19, 50, 2
    csc = tk.assemble_matrix(n, "RandSparseSPD")
    bs = _bench_rhs(n, d)
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, tk._lib.TK_LANCZOS, d, 0, [A] * d, bs, K)
    recs = [dev.init()] + [dev.step(j) for j in range(K)] + [dev.flush()]
    for f in range(d):
        al = np.array([recs[j + 1][f, j] for j in range(K)])
        be = np.array([recs[j + 1][f, j + 1] for j in range(K)])
        V = dev.basis(f, 0, K + 1)
        # trajectory while the oracle basis is orthonormal
        ref = tk_ref.RefFactor(csc, bs[f], K)
        j_orth = K
        for j in range(K):
            ref.lanczos_step(j)
            G = ref.V[:, :j + 2].T @ ref.V[:, :j + 2]
            if np.linalg.norm(G - np.eye(j + 2)) > 1e-10:
                j_orth = j
                break
        scale = max(np.abs(np.diag(ref.H)[:j_orth]).max(), 1.0)
        ea = np.abs(al[:j_orth] - np.diag(ref.H)[:j_orth]).max() / scale
        eb = np.abs(be[:j_orth] - np.diag(ref.H, -1)[:j_orth]).max() / scale
        eV = np.abs(V[:, :j_orth + 1] - ref.V[:, :j_orth + 1]).max()
        del ref
        # shadowing: one oracle step from the device's state, every step
        sh = tk_ref.RefFactor(csc, bs[f], K)
        sa = sb = sv = 0.0
        for j in range(K):
            if j > 0:
                sh.V[:, j - 1] = V[:, j - 1]
                sh.beta = be[j - 1]
            sh.V[:, j] = V[:, j]
            a_, b_ = sh.lanczos_step(j)
            sa = max(sa, abs(a_ - al[j]) / scale)
            sb = max(sb, abs(b_ - be[j]) / scale)
            sv = max(sv, np.abs(sh.V[:, j + 1] - V[:, j + 1]).max())
        del sh
        AVl = _spm(csc) @ V
        er = 0.0
        for j in range(1, K):
            r = AVl[:, j] - be[j - 1] * V[:, j - 1] - al[j] * V[:, j] - be[j] * V[:, j + 1]
            er = max(er, np.abs(r).max() / scale)
        print("C3 Lanczos factor %d: orthonormal through step %d: alpha %.2e beta %.2e V %.2e; "
              "shadowing (50 steps): alpha %.2e beta %.2e v %.2e; ttr %.2e"
              % (f, j_orth, ea, eb, eV, sa, sb, sv, er))
        assert j_orth >= 8                    # a meaningful stretch of trajectory
        assert ea <= 1e-12 and eb <= 1e-12    # alpha, beta: 1e-12 relative (trajectory)
        assert eV <= 1e-12                    # V: 1e-12 absolute (trajectory)
        assert sa <= 1e-13 and sb <= 1e-13    # one step from the same state: rounding only
        assert sv <= 1e-13
        assert er <= 1e-11                    # three-term relation
        del V, AVl
    dev.close()
    A.close()


def test_c4_convdiff_2p17_all_factors_and_vy(ctx):
    """C4 (configs[4]): d = 10, n_s = 2^17 ConvDiff (nonsymmetric, 4 diagonals), K = 50, one-
    sweep Arnoldi, every factor; V*Y at the solver's exp-sum rank t = 3 for each factor."""
    _check_arnoldi(ctx, "ConvDiff", 1 << 17, 10, 50, check=range(10), expect_sweeps=1, vy_t=3)


def test_c2_laplace_2p20_lanczos_all_8_factors(ctx):
    """C2 with TensorLanczos (the one-sweep TTR step the bench line 'c2_TensorLanczos' times,
    k_lan_1w + k_red_lan with the deferred Gram): d = 8, n_s = 2^20 Laplace, K = 50, swept
    exactly as bench.py does, every factor checked against the C oracle's TTR
    (src/orthogonal_bases.jl:39-67): alpha, beta and V while the oracle basis is orthonormal
    (1e-12), one oracle step from the device's state at every step (shadowing, rounding only),
    and the three-term relation on the device basis."""
    from oracle import tk_ref
    tk = _tk()
    n, K, d = 1 << 20, 50, 8
    csc = tk.assemble_matrix(n, "Laplace")
    bs = _bench_rhs(n, d)
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, tk._lib.TK_LANCZOS, d, 0, [A] * d, bs, K)
    assert dev.arnoldi_sweeps == 1 and dev.gram_deferred
    dev.init(False)
    dev.sweep(0, K)
    dev.flush(False)
    recs = dev.records(0, K + 1)
    S = _spm(csc)
    for f in range(d):
        al = np.array([recs[j + 1][f, j] for j in range(K)])
        be = np.array([recs[j + 1][f, j + 1] for j in range(K)])
        V = dev.basis(f, 0, K + 1)
        ref = tk_ref.RefFactor(csc, bs[f], K)
        j_orth = K
        for j in range(K):
            ref.lanczos_step(j)
            if j % 5 == 4 or j == K - 1:
                G = ref.V[:, :j + 2].T @ ref.V[:, :j + 2]
                if np.linalg.norm(G - np.eye(j + 2)) > 1e-10:
                    j_orth = j - 4
                    break
        scale = max(np.abs(np.diag(ref.H)[:K]).max(), 1.0)
        ea = np.abs(al[:j_orth] - np.diag(ref.H)[:j_orth]).max() / scale
        eb = np.abs(be[:j_orth] - np.diag(ref.H, -1)[:j_orth]).max() / scale
        eV = np.abs(V[:, :j_orth + 1] - ref.V[:, :j_orth + 1]).max()
        del ref
        sh = tk_ref.RefFactor(csc, bs[f], K)
        sa = sb = sv = 0.0
        for j in range(K):
            if j > 0:
                sh.V[:, j - 1] = V[:, j - 1]
                sh.beta = be[j - 1]
            sh.V[:, j] = V[:, j]
            a_, b_ = sh.lanczos_step(j)
            sa = max(sa, abs(a_ - al[j]) / scale)
            sb = max(sb, abs(b_ - be[j]) / scale)
            sv = max(sv, np.abs(sh.V[:, j + 1] - V[:, j + 1]).max())
        del sh
        AVl = S @ V
        er = 0.0
        for j in range(1, K):
            r = AVl[:, j] - be[j - 1] * V[:, j - 1] - al[j] * V[:, j] - be[j] * V[:, j + 1]
            er = max(er, np.abs(r).max() / scale)
        print("C2 Lanczos factor %d: orthonormal through step %d: alpha %.2e beta %.2e V %.2e; "
              "shadowing: alpha %.2e beta %.2e v %.2e; ttr %.2e" % (f, j_orth, ea, eb, eV, sa, sb, sv, er))
        assert j_orth >= 15                   # a meaningful stretch of trajectory (TTR loses
                                              # orthogonality after 20-50 steps here)
        assert ea <= 1e-12 and eb <= 1e-12    # alpha, beta: 1e-12 relative (trajectory)
        assert eV <= 1e-12                    # V: 1e-12 absolute (trajectory)
        assert sa <= 1e-13 and sb <= 1e-13    # one step from the same state: rounding only
        assert sv <= 1e-13
        assert er <= 1e-11                    # three-term relation
        del V, AVl
    dev.close()
    A.close()
