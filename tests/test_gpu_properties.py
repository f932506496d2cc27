"""GPU parity at full size and on the edge cases, through the C ABI.

  * n = 2^20 (BASELINE config C2's factor size; C1/C3/C4 sizes are in test_gpu_configs.py),
    K = 50: the device's H, V and records
    against the C restatement (oracle/tk_ref.c, MGS2) on the same inputs, plus the
    size-independent properties (orthonormality from the device Gram rows, the Arnoldi
    relation A V_K = V_{K+1} Hbar_K).
  * factor partitioning: a factor's records and basis are bitwise independent of which
    decomposition / rank owns it (the multi-GPU path relies on this).
  * breakdown (beta = 0): Lanczos writes a zero column (src/orthogonal_bases.jl:59); Arnoldi
    divides by zero like the reference (`v .* inv(0.0)`, :36) -> NaN column.
  * single-matrix drivers arnoldi_algorithm / lanczos_algorithm / isorthonormal
    (src/orthogonal_bases.jl:182-284; test/decompositions.jl:4-19 sizes).
  * recorded ConvDiff trajectory (nonsym_new, d=5) and a distinct-b nonsymmetric solve.
Tolerances as in test_gpu_parity.py; each is stated at its assert.
"""
import json
import os

import numpy as np
import pytest

from oracle import tk_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _tk():
    import tkamd
    return tkamd


def _unit(v):
    return v / np.linalg.norm(v)


# ------------------------------------------------------------------ full size
def test_full_size_arnoldi_vs_c_oracle(ctx):
    """C2 factor size n = 2^20, K = 50, two factors with distinct b_s."""
    from oracle import tk_ref
    tk = _tk()
    n, K = 1 << 20, 50
    csc = tk.assemble_matrix(n, "Laplace")
    rng = np.random.default_rng(1001)
    bs = [_unit(rng.random(n)) for _ in range(2)]
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, 2, 0, [A, A], bs, K, track_all_gram=True)
    lay = tk._lib.RecordLayout(K)
    recs = [dev.init()] + [dev.step(j) for j in range(K)] + [dev.flush()]
    for f, b in enumerate(bs):
        ref = tk_ref.RefFactor(csc, b, K)
        for j in range(K):
            ref.arnoldi_step(j)
        Hd = np.zeros((K + 1, K))
        for j in range(K):
            Hd[:j + 2, j] = recs[j + 1][f, :j + 2]
        scale = np.abs(ref.H[:K + 1, :K]).max()
        assert np.abs(Hd - ref.H[:K + 1, :K]).max() <= 1e-12 * scale          # H: 1e-12 relative
        V = dev.basis(f, 0, K + 1)
        assert np.abs(V - ref.V[:, :K + 1]).max() <= 1e-12                      # V: 1e-12 absolute
        G = np.zeros((K + 1, K + 1))
        bt = np.zeros(K + 1)
        for r in recs:
            c = int(r[f, lay.col])
            if c >= 0:
                G[c, :c + 1] = r[f, lay.gram:lay.gram + c + 1]
                bt[c] = r[f, lay.bt]
        bt_ref = ref.V[:, :K + 1].T @ b
        # btilde: a 2^20-term dot carries ~sqrt(n)*eps rounding on both sides -> 1e-13 abs
        assert np.abs(bt - bt_ref).max() <= 1e-13
        # orthonormality from the device Gram rows (size-independent property)
        Gs = np.tril(G) + np.tril(G, -1).T
        assert np.linalg.norm(Gs - np.eye(K + 1)) <= 1e-12
        # Arnoldi relation  A V_K = V_{K+1} Hbar_K  (columns 0..K-1)
        AV = np.stack([O.csc_matvec_fast(csc, V[:, j]) for j in range(K)], axis=1)
        R = AV - V @ Hd
        assert np.abs(R).max() <= 1e-11 * scale
        del ref, V, AV, R
    dev.close()
    A.close()


def test_full_size_lanczos_properties(ctx):
    """TTR at n = 2^20: alpha/beta against the C restatement for the first 30 steps and
    the three-term relation A v_j = beta_{j-1} v_{j-1} + alpha_j v_j + beta_j v_{j+1}."""
    from oracle import tk_ref
    tk = _tk()
    n, K = 1 << 20, 30
    csc = tk.assemble_matrix(n, "Laplace")
    b = _unit(np.random.default_rng(1002).random(n))
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, tk._lib.TK_LANCZOS, 1, 0, [A], [b], K)
    recs = [dev.init()] + [dev.step(j) for j in range(K)] + [dev.flush()]
    ref = tk_ref.RefFactor(csc, b, K)
    al, be = np.zeros(K), np.zeros(K)
    for j in range(K):
        ref.lanczos_step(j)
        al[j], be[j] = recs[j + 1][0, j], recs[j + 1][0, j + 1]
    scale = max(np.abs(np.diag(ref.H)).max(), 1.0)
    assert np.abs(al - np.diag(ref.H)[:K]).max() <= 1e-12 * scale
    assert np.abs(be - np.diag(ref.H, -1)[:K]).max() <= 1e-12 * scale
    V = dev.basis(0, 0, K + 1)
    for j in range(1, K):
        r = O.csc_matvec_fast(csc, V[:, j]) - be[j - 1] * V[:, j - 1] - al[j] * V[:, j] - be[j] * V[:, j + 1]
        assert np.abs(r).max() <= 1e-11 * scale
    dev.close()
    A.close()


# ------------------------------------------------------------------ partition independence
@pytest.mark.parametrize("method", [0, 1, 2])
def test_factor_results_independent_of_partition(ctx, method):
    """Each factor stepped inside a d=4 decomposition equals the same factor stepped
    alone (d_total=4, first=s, nf=1) bit for bit: records and basis.  Reductions use a
    partial count that depends on n only, so the result cannot depend on the rank layout."""
    tk = _tk()
    n, K, d = 5000, 30, 4
    csc = tk.assemble_matrix(n, "ConvDiff" if method == 0 else "Laplace")
    rng = np.random.default_rng(44)
    bs = [_unit(rng.random(n)) for _ in range(d)]
    A = tk.DeviceMatrix(ctx, csc)

    def run(first, nf):
        dev = tk.DeviceDecomposition(ctx, method, d, first, [A] * nf, bs[first:first + nf], K,
                                     track_all_gram=True)
        recs = [dev.init()] + [dev.step(j) for j in range(K)] + [dev.flush()]
        V = [dev.basis(f, 0, K + 1) for f in range(nf)]
        dev.close()
        return recs, V

    recs_all, V_all = run(0, d)
    for s in range(d):
        recs_s, V_s = run(s, 1)
        for ra, rs in zip(recs_all, recs_s):
            assert np.array_equal(ra[s], rs[s])
        assert np.array_equal(V_all[s], V_s[0])
    A.close()


# ------------------------------------------------------------------ breakdown
def _breakdown_case(n=300):
    diag = np.linspace(1.0, 3.0, n)
    csc = O.dense_to_csc(np.diag(diag))
    b = np.zeros(n)
    b[0] = 1.0                        # an eigenvector: the Krylov space is 1-dimensional
    return csc, b, diag


def test_lanczos_breakdown_zero_column(ctx):
    tk = _tk()
    csc, b, diag = _breakdown_case()
    K = 6
    recs, V = _run(ctx, tk._lib.TK_LANCZOS, csc, [b], K)
    fo = O.Factor(csc, b, K)
    for j in range(1, K + 1):
        fo.lanczos_ttr(j)
    assert recs[1][0, 0] == diag[0] and recs[1][0, 1] == 0.0                  # alpha_1, beta_1 = 0
    for j in range(1, K):
        assert recs[j + 1][0, j] == 0.0 and recs[j + 1][0, j + 1] == 0.0
    assert np.array_equal(V[0], fo.V[:, :K + 1])                              # zero columns, exactly


def test_arnoldi_breakdown_matches_reference_division(ctx):
    tk = _tk()
    csc, b, diag = _breakdown_case()
    K = 3
    recs, V = _run(ctx, tk._lib.TK_ARNOLDI, csc, [b], K)
    fo = O.Factor(csc, b, K)
    with np.errstate(all="ignore"):
        fo.arnoldi_mgs(1)
    assert recs[1][0, 0] == diag[0] and recs[1][0, 1] == 0.0                  # H[1,1], H[2,1] = 0
    assert np.isnan(fo.V[:, 1]).all()                                         # 0 * inv(0) in Julia
    assert np.isnan(V[0][:, 1]).all()


def _run(ctx, method, csc, bs, K):
    tk = _tk()
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, method, len(bs), 0, [A] * len(bs), bs, K)
    recs = [dev.init()] + [dev.step(j) for j in range(K)] + [dev.flush()]
    V = [dev.basis(f, 0, K + 1) for f in range(len(bs))]
    dev.close()
    A.close()
    return recs, V


# ------------------------------------------------------------------ single-matrix drivers (a12)
def test_single_matrix_drivers(ctx):
    """test/decompositions.jl:4-19: n = 1000, k = 500, scaled tridiagonal Laplacian."""
    from oracle import tk_ref
    tk = _tk()
    n, k = 1000, 500
    A = O.laplace_dense(n)
    b = np.random.default_rng(12345).random(n)
    ar = tk.arnoldi_algorithm(A, b, k, ctx=ctx)
    assert ar.V.shape == (n, k + 1) and ar.H.shape == (k + 1, k)
    assert tk.isorthonormal(ar, k)
    ref = tk_ref.RefFactor(O.dense_to_csc(A), b, k)
    for j in range(k):
        ref.arnoldi_step(j)
    scale = np.abs(ref.H).max()
    assert np.abs(ar.H - ref.H[:k + 1, :k]).max() <= 1e-10 * scale             # 500 steps: 1e-10 rel
    la = tk.lanczos_algorithm(A, b, 60, ctx=ctx)
    fo = O.Factor(O.dense_to_csc(A), b, 60)
    for j in range(1, 60):
        fo.lanczos_ttr(j)
    assert np.abs(la.H[:59, :59] - fo.H[:59, :59]).max() <= 1e-12 * np.abs(fo.H).max()
    lr = tk.lanczos_algorithm(A, b, 60, reorth=True, ctx=ctx)
    assert tk.isorthonormal(lr, 59)


# ------------------------------------------------------------------ driver: nonsymmetric
@pytest.mark.parametrize("d,K", [(5, 26), (10, 51)])
def test_tensorkrylov_convdiff_golden(ctx, d, K):
    """Recorded reference trajectories experiments/data/reproduction_data/nonsym_new
    (d=5: k<=26, d=10: k<=51), TensorArnoldi, through the product driver: relative
    residuals within 1e-10 of the recording."""
    tk = _tk()
    g = json.load(open(os.path.join(HERE, "golden", "reproduction.json")))["nonsym_new"]
    n = 200
    b = np.array(g["rhs"][str(d)])
    A = tk.KroneckerMatrix.gallery(tk.NonSymInstance, d, n, tk.ConvDiff)
    conv = tk.ConvergenceData(K)
    tk.tensorkrylov(conv, A, [b.copy() for _ in range(d)], 1e-9, K, "TensorArnoldi", ctx=ctx)
    ref = np.array(g["convergence"][str(d)]["relative_residual_norm"][:K])
    rel = np.abs(conv.relative_residual_norm[1:] - ref[1:]) / ref[1:]
    assert rel.max() <= 1e-10


def test_tensorkrylov_nonsym_distinct_rhs_vs_oracle(ctx):
    tk = _tk()
    d, n, K = 4, 300, 30
    rng = np.random.default_rng(77)
    b = [_unit(rng.random(n)) for _ in range(d)]
    A = tk.KroneckerMatrix.gallery(tk.NonSymInstance, d, n, tk.ConvDiff)
    conv = tk.ConvergenceData(K)
    tk.tensorkrylov(conv, A, [x.copy() for x in b], 1e-9, K, "TensorArnoldi", ctx=ctx)
    dense = O.convdiff_dense(n)
    conv_o, _, _ = O.tensorkrylov([O.dense_to_csc(dense)] * d, b, 1e-9, K, "TensorArnoldi", "ConvDiff",
                                  False, A_dense=dense)
    assert conv.niterations == conv_o.niterations
    ref = np.array(conv_o.relative_residual_norm)
    assert np.abs(conv.relative_residual_norm[1:] - ref[1:]).max() <= 1e-10 * ref[1:].max()


# ------------------------------------------------------------------ exchange path (N > 1 code)
@pytest.mark.parametrize("method", [0, 1, 2])
def test_rccl_exchange_path_matches_local_records(ctx, method, monkeypatch):
    """The multi-rank path -- records summed by ncclAllReduce on the exchange stream, slot
    events, the receive buffer -- forced on a 1-rank communicator, gives bitwise the same
    records and basis as the local path (what every rank of an N-GPU run relies on)."""
    tk = _tk()
    n, K, d = 3000, 25, 3
    csc = tk.assemble_matrix(n, "Laplace")
    rng = np.random.default_rng(5)
    bs = [_unit(rng.random(n)) for _ in range(d)]

    def run(c, sig=None):
        A = tk.DeviceMatrix(c, csc)
        dev = tk.DeviceDecomposition(c, method, d, 0, [A] * d, bs, K, track_all_gram=True)
        if sig is not None:
            assert dev.exchange_signalled == sig
        recs = [dev.init()] + [dev.step(j) for j in range(K)] + [dev.flush()]
        dev.init(False)                       # asynchronous sweep through the same path
        dev.sweep(0, K)
        dev.flush(False)
        recs2 = dev.records(0, K + 2)
        V = [dev.basis(f, 0, K + 1) for f in range(d)]
        dev.close()
        A.close()
        return recs, recs2, V

    local = run(ctx)
    c2 = tk.Context(0)
    c2.init_comm(tk.unique_id(), 1, 0)
    monkeypatch.setenv("TKHIP_EXCHANGE_ALWAYS", "1")
    # Arnoldi / Lanczos steps trigger the exchange through the signal word (the
    # hipStreamWaitValue64 path), LanczosReorth through events; the signalled slots of a
    # sweep go out in groups (TKHIP_XCH_GROUP; 3 leaves a partial group at the sweep's end)
    for grp in ("1", "3", "4"):
        monkeypatch.setenv("TKHIP_XCH_GROUP", grp)
        xch = run(c2, sig=method != 2)
        for a, b in zip(local[0], xch[0]):
            assert np.array_equal(a, b)
        for s in range(K + 2):
            assert np.array_equal(local[1][s], xch[1][s])
        for a, b in zip(local[2], xch[2]):
            assert np.array_equal(a, b)
    c2.close()


@pytest.mark.parametrize("grp", ["1", "4", "5"])
def test_native_loop_through_grouped_exchange(ctx, grp, monkeypatch):
    """The whole tensorkrylov! loop (native host loop reading records while steps run ahead)
    over the multi-rank record path with grouped all-reduces: bitwise the local run."""
    tk = _tk()
    d, n, K = 4, 3000, 30
    rng = np.random.default_rng(33)
    b = [_unit(rng.random(n)) for _ in range(d)]
    A = tk.KroneckerMatrix.gallery(tk.SymInstance, d, n, tk.Laplace)
    ref = tk.ConvergenceData(K)
    tk.tensorkrylov(ref, A, [v.copy() for v in b], 1e-9, K, "TensorArnoldi", ctx=ctx)
    c2 = tk.Context(0)
    c2.init_comm(tk.unique_id(), 1, 0)
    monkeypatch.setenv("TKHIP_EXCHANGE_ALWAYS", "1")
    monkeypatch.setenv("TKHIP_XCH_GROUP", grp)
    conv = tk.ConvergenceData(K)
    tk.tensorkrylov(conv, A, [v.copy() for v in b], 1e-9, K, "TensorArnoldi", ctx=c2)
    c2.close()
    assert conv.niterations == ref.niterations
    assert np.array_equal(conv.relative_residual_norm, ref.relative_residual_norm)
    assert np.array_equal(conv.orthogonality_data, ref.orthogonality_data)


@pytest.mark.parametrize("method", ["TensorArnoldi", "TensorLanczos", "TensorLanczosReorth"])
def test_pipelined_driver_identical_to_sequential(ctx, method):
    """The driver enqueues step k+1 before the host evaluates iteration k; every iterate,
    residual and the returned solution must be those of the sequential loop (bitwise)."""
    tk = _tk()
    d, n, K = 4, 3000, 30
    rng = np.random.default_rng(21)
    b = [_unit(rng.random(n)) for _ in range(d)]
    A = tk.KroneckerMatrix.gallery(tk.SymInstance, d, n, tk.Laplace)
    out = []
    for pipe in (False, True):
        conv = tk.ConvergenceData(K)
        x = tk.tensorkrylov(conv, A, [v.copy() for v in b], 1e-6, K, method, ctx=ctx, pipelined=pipe)
        out.append((conv, x))
    (c0, x0), (c1, x1) = out
    assert c0.niterations == c1.niterations
    assert np.array_equal(c0.relative_residual_norm, c1.relative_residual_norm)
    assert np.array_equal(c0.orthogonality_data, c1.orthogonality_data)
    assert (x0 is None) == (x1 is None)
    if x0 is not None:
        assert np.array_equal(x0.lam, x1.lam)
        for a_, b_ in zip(x0.fmat, x1.fmat):
            assert np.array_equal(a_, b_)
