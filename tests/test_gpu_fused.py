"""Fused one-sweep Arnoldi launches (TKHIP_D1_FUSE=1): step j's reduce runs in the leading blocks
of step j+1's k_arn_d1 launch instead of a k_reduce256 launch of its own; the window blocks
issue their basis-row loads, wait for the factor's step word and read the coefficients the
reducers produced in the same launch through sc1 loads.

The reduction and every product are the same as with the separate launch, so records, basis,
flushed column, V*Y and Gram must be BITWISE equal -- checked here for swept and step-by-step
sequences (each step's records read at once: the pending reduce then runs as its own launch),
a second sequence on the same handle, factor groups, the forced records exchange of a 1-rank
communicator, and the end-to-end driver (the C2 oracle parity of the default path carries over
through the bitwise equality)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tk():
    import tkamd
    return tkamd


def _run(ctx, monkeypatch, fuse, cls, n, d, K, stepwise=False, t=3):
    tk = _tk()
    monkeypatch.setenv("TKHIP_D1_FUSE", "1" if fuse else "0")
    csc = tk.assemble_matrix(n, cls)
    rng = np.random.default_rng(31)
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, d, 0, [A] * d, bs, K)
    assert dev.arnoldi_sweeps == 1
    out = {}
    for rep in range(2):                              # a second sequence on the same handle
        if stepwise:
            recs = [dev.init()] + [dev.step(j) for j in range(K)]
            out["recs%d" % rep] = np.array(recs)
        else:
            dev.init(False)
            dev.sweep(0, K)
            out["recs%d" % rep] = dev.records(0, K + 1)
    Ys = [np.random.default_rng(5 + f).standard_normal((K, t)) for f in range(d)]
    out["X"] = dev.basis_mul(K, Ys)
    out["V"] = [dev.basis(f, 0, K + 1) for f in range(d)]
    if dev.gram_deferred:
        out["G"] = dev.gram(0, K)
    dev.close()
    A.close()
    return out


def _same(a, b):
    for k in a:
        x, y = a[k], b[k]
        if isinstance(x, list):
            assert all(np.array_equal(p, q) for p, q in zip(x, y)), k
        else:
            assert np.array_equal(x, y), k


@pytest.mark.parametrize("cls,n,d,K", [("ConvDiff", 1 << 17, 2, 50), ("Laplace", 3000, 5, 40),
                                       ("Laplace", 1 << 20, 1, 24), ("Laplace", 700, 3, 63)])
def test_fused_launch_bitwise_equal_separate_reduce(ctx, monkeypatch, cls, n, d, K):
    ref = _run(ctx, monkeypatch, False, cls, n, d, K)
    fz = _run(ctx, monkeypatch, True, cls, n, d, K)
    _same(ref, fz)


def test_fused_launch_stepwise_records(ctx, monkeypatch):
    """Every step's record read at once: the pending reduce runs as its own launch (red_flush)
    before the bookkeeping, and the next launch reduces nothing."""
    ref = _run(ctx, monkeypatch, False, "ConvDiff", 5000, 3, 30, stepwise=True)
    fz = _run(ctx, monkeypatch, True, "ConvDiff", 5000, 3, 30, stepwise=True)
    _same(ref, fz)


def test_fused_launch_one_factor_group_and_exchange(ctx, monkeypatch):
    """One stream (TKHIP_FACTOR_GROUPS=1) and the records exchange on a 1-rank communicator
    (the N > 1 path): still bitwise the separate-reduce results."""
    tk = _tk()
    monkeypatch.setenv("TKHIP_FACTOR_GROUPS", "1")
    ref = _run(ctx, monkeypatch, False, "Laplace", 1 << 16, 4, 40)
    fz = _run(ctx, monkeypatch, True, "Laplace", 1 << 16, 4, 40)
    _same(ref, fz)
    monkeypatch.delenv("TKHIP_FACTOR_GROUPS")
    c2 = tk.Context(0)
    c2.init_comm(tk.unique_id(), 1, 0)
    monkeypatch.setenv("TKHIP_EXCHANGE_ALWAYS", "1")
    try:
        ref = _run(c2, monkeypatch, False, "ConvDiff", 1 << 15, 3, 30)
        fz = _run(c2, monkeypatch, True, "ConvDiff", 1 << 15, 3, 30)
        _same(ref, fz)
    finally:
        c2.close()


def test_fused_launch_end_to_end(ctx, monkeypatch):
    """tkamd.tensorkrylov (the native pipelined loop: steps issued ahead, records read as they
    arrive, the Gram launched behind the last step) gives the same trajectory bit for bit."""
    tk = _tk()
    d, n, K = 4, 1 << 14, 40
    A = tk.KroneckerMatrix.gallery(tk.NonSymInstance, d, n, tk.ConvDiff)
    b = tk.normalize_rhs(tk.random_rhs(d, n, np.random.default_rng(9)))
    out = {}
    for fuse in ("0", "1"):
        monkeypatch.setenv("TKHIP_D1_FUSE", fuse)
        conv = tk.ConvergenceData(K)
        tk.tensorkrylov(conv, A, [x.copy() for x in b], 1e-12, K, "TensorArnoldi", ctx=ctx)
        out[fuse] = conv
    for name in ("relative_residual_norm", "projected_residual_norm", "orthogonality_data"):
        assert np.array_equal(getattr(out["0"], name), getattr(out["1"], name)), name


@pytest.mark.parametrize("odd", [True, False])
def test_fused_record_read_mid_sweep_then_continue(ctx, monkeypatch, odd):
    """fused handles alternate a step's partials between P1 and P1b by step parity;
    the only reduce outside a fused launch is red_flush, which picks the buffer by j.  A grouped
    fused handle whose records are read in the middle of an asynchronous run -- at an odd step
    (P1b) and at an even one (P1) -- and that then keeps stepping (the next fused launch reduces
    nothing: its pending reduce already ran) equals the separate-reduce handle bit for bit."""
    tk = _tk()
    n, d, K = 1 << 15, 4, 30
    jr = 13 if odd else 14
    out = {}
    for fuse in (False, True):
        monkeypatch.setenv("TKHIP_D1_FUSE", "1" if fuse else "0")
        csc = tk.assemble_matrix(n, "ConvDiff")
        rng = np.random.default_rng(77)
        bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
        A = tk.DeviceMatrix(ctx, csc)
        dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, d, 0, [A] * d, bs, K)
        assert dev.factor_groups == 2
        dev.init(False)
        for j in range(K):
            if j == jr:
                mid = dev.step(j)             # a record out: red_flush + the bookkeeping now
            else:
                dev.step_async(j)
        recs = dev.records(0, K + 1)
        V = [dev.basis(f, 0, K + 1) for f in range(d)]
        out[fuse] = (mid, recs, V)
        dev.close()
        A.close()
    assert np.array_equal(out[False][0], out[True][0])
    assert np.array_equal(out[False][1], out[True][1])
    for f in range(d):
        assert np.array_equal(out[False][2][f], out[True][2][f])
