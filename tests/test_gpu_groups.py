"""One-sweep Arnoldi factor groups (tk_decomp_factor_groups): the local factors step as two
groups, each in its own launches on its own stream, so one group's launch drain and reduce
overlap the other's sweep.  Every kernel is per factor, so the records, the basis, the
flushed column and V*Y must be bitwise those of one stream (TKHIP_FACTOR_GROUPS=1), whether
the steps are taken one at a time with their records (the driver's pattern) or as a sweep,
and for an odd factor count (groups of 2 and 3).  Reference: the per-factor steps of
orthonormalize! (src/orthogonal_bases.jl:162-180) are independent of each other.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d", [2, 5])
def test_factor_groups_bitwise_equal_one_stream(ctx, d, monkeypatch):
    import tkamd as tk
    n, K, t = 3000, 40, 5
    rng = np.random.default_rng(77)
    mats = [tk.assemble_matrix(n, "Laplace"), tk.assemble_matrix(n, "ConvDiff")]
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    Ys = [rng.standard_normal((K, t)) for _ in range(d)]
    out = {}
    for G in ("1", "2", "3"):
        monkeypatch.setenv("TKHIP_FACTOR_GROUPS", G)
        A = [tk.DeviceMatrix(ctx, m) for m in mats]
        dev = tk.DeviceDecomposition(ctx, 0, d, 0, [A[s % 2] for s in range(d)], bs, K)
        assert dev.arnoldi_sweeps == 1
        assert dev.factor_groups == min(int(G), d)
        r0 = dev.init()
        recs = [dev.step(j) for j in range(12)]          # one at a time, records read
        dev.sweep(12, K - 1)                             # the rest as a sweep
        recs.append(dev.step(K - 1))
        recs.append(dev.flush())
        allrec = dev.records(0, K + 1)
        V = [dev.basis(f, 0, K + 1) for f in range(d)]
        X = dev.basis_mul(K, Ys)
        out[G] = (r0, recs, allrec, V, X)
        dev.close()
        for a in A:
            a.close()
    for G in ("2", "3"):
        (a0, ar, aa, aV, aX), (b0, br, ba, bV, bX) = out["1"], out[G]
        assert np.array_equal(a0, b0)
        for x, y in zip(ar, br):
            assert np.array_equal(x, y)
        assert np.array_equal(aa, ba)
        for x, y in zip(aV, bV):
            assert np.array_equal(x, y)
        for x, y in zip(aX, bX):
            assert np.array_equal(x, y)
    # and the basis is an orthonormal Arnoldi basis
    assert np.abs(aV[0].T @ aV[0] - np.eye(K + 1)).max() < 1e-12


@pytest.mark.parametrize("grp", ["1", "4"])
def test_factor_groups_under_records_exchange(ctx, grp, monkeypatch):
    """A rank holding several factors under a records exchange (C4 at 8 GPUs, C2 at 2 and 4):
    the two group streams signal the exchange through one word and every slot guard is waited
    for on both.  On a 1-rank communicator (the exchange path, TKHIP_EXCHANGE_ALWAYS) the
    grouped handle's records, exchanged records, basis and V*Y equal the one-stream local run
    bit for bit, for exchange groups of 1 and 4 slots."""
    import tkamd as tk
    d, n, K, t = 4, 3000, 30, 4
    rng = np.random.default_rng(5)
    mats = [tk.assemble_matrix(n, "Laplace"), tk.assemble_matrix(n, "ConvDiff")]
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    Ys = [rng.standard_normal((K, t)) for _ in range(d)]

    def run(c, G):
        monkeypatch.setenv("TKHIP_FACTOR_GROUPS", G)
        A = [tk.DeviceMatrix(c, m) for m in mats]
        dev = tk.DeviceDecomposition(c, 0, d, 0, [A[s % 2] for s in range(d)], bs, K)
        assert dev.factor_groups == int(G)
        r0 = dev.init()
        recs = [dev.step(j) for j in range(6)]
        for j in range(6, 14):
            dev.step_async(j)
        recs.append(dev.records(7, 14))
        dev.sweep(14, K)
        recs.append(dev.records(0, K + 1))
        V = [dev.basis(f, 0, K) for f in range(d)]
        X = dev.basis_mul(K, Ys)
        recs.append(dev.records(K + 1, K + 2))
        dev.close()
        for a in A:
            a.close()
        return r0, recs, V, X

    local = run(ctx, "1")
    c2 = tk.Context(0)
    c2.init_comm(tk.unique_id(), 1, 0)
    monkeypatch.setenv("TKHIP_EXCHANGE_ALWAYS", "1")
    monkeypatch.setenv("TKHIP_XCH_GROUP", grp)
    try:
        xch = run(c2, "2")
        xch3 = run(c2, "3")
    finally:
        c2.close()
    for a, b in zip(xch[1], xch3[1]):
        assert np.array_equal(a, b)
    for a, b in zip(xch[3], xch3[3]):
        assert np.array_equal(a, b)
    assert np.array_equal(local[0], xch[0])
    for a, b in zip(local[1], xch[1]):
        assert np.array_equal(a, b)
    for a, b in zip(local[2], xch[2]):
        assert np.array_equal(a, b)
    for a, b in zip(local[3], xch[3]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("fuse", ["0", "1"])
def test_factor_groups_exchange_waits_for_every_group(ctx, fuse, monkeypatch):
    """The groups' streams run apart: with group 0's stream held back before every launch
    (TKHIP_TEST_GROUP_DELAY_US) group 1 runs steps ahead, and a shared signal count could then
    be reached with group 0's row of a slot still unwritten (the exchanged record read as
    zeros -- seen once with the fused launches).  Each factor signals its own word and the
    exchange waits for all of them: the exchanged records equal the one-stream local run bit for
    bit, with and without the fused launches."""
    import tkamd as tk
    d, n, K = 3, 1 << 15, 30
    monkeypatch.setenv("TKHIP_D1_FUSE", fuse)
    rng = np.random.default_rng(12)
    mat = tk.assemble_matrix(n, "ConvDiff")
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]

    def run(c, G):
        monkeypatch.setenv("TKHIP_FACTOR_GROUPS", G)
        A = tk.DeviceMatrix(c, mat)
        dev = tk.DeviceDecomposition(c, 0, d, 0, [A] * d, bs, K)
        assert dev.factor_groups == int(G)
        dev.init(False)
        dev.sweep(0, K)
        r = dev.records(0, K + 1)
        dev.close()
        A.close()
        return r

    local = run(ctx, "1")
    c2 = tk.Context(0)
    c2.init_comm(tk.unique_id(), 1, 0)
    monkeypatch.setenv("TKHIP_EXCHANGE_ALWAYS", "1")
    monkeypatch.setenv("TKHIP_TEST_GROUP_DELAY_US", "300")
    try:
        for _ in range(2):
            assert np.array_equal(local, run(c2, "2"))
    finally:
        monkeypatch.delenv("TKHIP_TEST_GROUP_DELAY_US")
        c2.close()


@pytest.mark.parametrize("alt", ["0", "1"])
def test_back_to_back_sequences_under_records_exchange(ctx, alt, monkeypatch):
    """Sequences issued back to back on one exchange handle, the host running ahead (group 0
    held back, no records read between the second and third sequence): the send rows alternate
    between two buffers by sequence (TKHIP_REC_ALT, default on), the slot guards tracking each
    buffer's last all-reduce.  Every sequence's exchanged records equal the local run bit for
    bit -- the zero-initialised second buffer read before its rows were written would show as
    zero rows."""
    import tkamd as tk
    d, n, K = 3, 1 << 14, 24
    monkeypatch.setenv("TKHIP_REC_ALT", alt)
    rng = np.random.default_rng(21)
    mat = tk.assemble_matrix(n, "ConvDiff")
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]

    def run(c, G):
        monkeypatch.setenv("TKHIP_FACTOR_GROUPS", G)
        A = tk.DeviceMatrix(c, mat)
        dev = tk.DeviceDecomposition(c, 0, d, 0, [A] * d, bs, K)
        out = []
        for seq in range(4):
            dev.init(False)
            dev.sweep(0, K)
            if seq != 1:
                out.append(dev.records(0, K + 1))
        dev.close()
        A.close()
        return out

    local = run(ctx, "1")
    assert all(np.array_equal(local[0], r) for r in local[1:])
    c2 = tk.Context(0)
    c2.init_comm(tk.unique_id(), 1, 0)
    monkeypatch.setenv("TKHIP_EXCHANGE_ALWAYS", "1")
    monkeypatch.setenv("TKHIP_TEST_GROUP_DELAY_US", "100")
    try:
        for G in ("1", "2"):
            for r in run(c2, G):
                assert np.array_equal(local[0], r)
    finally:
        monkeypatch.delenv("TKHIP_TEST_GROUP_DELAY_US")
        c2.close()


@pytest.mark.parametrize("d", [2, 5])
def test_lanczos_factor_groups_bitwise_equal_one_stream(ctx, d, monkeypatch):
    """One-sweep TensorLanczos without Gram rows (k_lan_1w + k_red_lan, the deferred Gram)
    steps its factors as two groups on two streams: records (taken one step at a time and as a
    sweep), the basis, the flushed column and V*Y bitwise those of one stream."""
    import tkamd as tk
    monkeypatch.delenv("TKHIP_GRAM", raising=False)
    monkeypatch.setenv("TKHIP_LANCZOS_GROUPS", "1")   # (opt-in: slower at C2)
    n, K, t = 3000, 40, 5
    rng = np.random.default_rng(78)
    mat = tk.assemble_matrix(n, "Laplace")
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    Ys = [rng.standard_normal((K, t)) for _ in range(d)]
    out = {}
    for G in ("1", "2", "3"):
        monkeypatch.setenv("TKHIP_FACTOR_GROUPS", G)
        A = tk.DeviceMatrix(ctx, mat)
        dev = tk.DeviceDecomposition(ctx, tk._lib.TK_LANCZOS, d, 0, [A] * d, bs, K)
        assert dev.arnoldi_sweeps == 1 and dev.gram_deferred
        assert dev.factor_groups == min(int(G), d)
        r0 = dev.init()
        recs = [dev.step(j) for j in range(9)]
        for j in range(9, 17):
            dev.step_async(j)
        recs.append(dev.records(10, 17))
        dev.sweep(17, K)
        recs.append(dev.records(0, K + 1))
        V = [dev.basis(f, 0, K) for f in range(d)]
        X = dev.basis_mul(K, Ys)
        recs.append(dev.records(K + 1, K + 2))
        out[G] = (r0, recs, V, X)
        dev.close()
        A.close()
    for G in ("2", "3"):
        (a0, ar, aV, aX), (b0, br, bV, bX) = out["1"], out[G]
        assert np.array_equal(a0, b0)
        for x, y in zip(ar, br):
            assert np.array_equal(x, y)
        for x, y in zip(aV, bV):
            assert np.array_equal(x, y)
        for x, y in zip(aX, bX):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("d,K", [(2, 40), (3, 41)])
def test_lanczos_single_column_layout_bitwise_equal_pairs(ctx, d, K, monkeypatch):
    """The Gram-free one-sweep TensorLanczos keeps V_s in single-column tiles (its step reads
    v_{j-1} and writes v_j: 40 bytes per row instead of 48).  Every reader of the basis takes
    the layout: records (step by step, as a sweep), the columns read back before and after the
    flush, the fused flush + V*Y and the MFMA V*Y with a VALU tail are bitwise those of the
    paired-column layout (TKHIP_LANCZOS_SL=0), odd and even K; factor 1's Gram (MFMA SYRK,
    two rows per lane and load in single columns: its row sums in another order) to 1e-13."""
    import tkamd as tk
    monkeypatch.delenv("TKHIP_GRAM", raising=False)
    monkeypatch.delenv("TKHIP_LANCZOS_GROUPS", raising=False)
    n = 3000
    rng = np.random.default_rng(79)
    mat = tk.assemble_matrix(n, "Laplace")
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    Y1 = [rng.standard_normal((K, 5)) for _ in range(d)]
    Y2 = [rng.standard_normal((K + 1, 17)) for _ in range(d)]
    out = {}
    for sl in ("0", "1"):
        monkeypatch.setenv("TKHIP_LANCZOS_SL", sl)
        A = tk.DeviceMatrix(ctx, mat)
        dev = tk.DeviceDecomposition(ctx, tk._lib.TK_LANCZOS, d, 0, [A] * d, bs, K)
        assert dev.arnoldi_sweeps == 1 and dev.gram_deferred
        assert dev.single_columns == (sl == "1")
        r0 = dev.init()
        recs = [dev.step(j) for j in range(9)]
        for j in range(9, 17):
            dev.step_async(j)
        recs.append(dev.records(10, 17))
        dev.sweep(17, K)
        recs.append(dev.records(0, K + 1))
        G = dev.gram(0, K - 1)                         # written columns only
        V0 = [dev.basis(f, 0, K - 1) for f in range(d)]
        X1 = dev.basis_mul(K, Y1)                      # pending column: the fused flush + V*Y
        recs.append(dev.records(K + 1, K + 2))
        X2 = dev.basis_mul(K + 1, Y2)                  # flushed: k_basis_mul (MFMA + VALU tail)
        V1 = [dev.basis(f, 0, K + 1) for f in range(d)]
        G1 = dev.gram(0, K + 1)
        out[sl] = (r0, recs, G, V0, X1, X2, V1, G1)
        dev.close()
        A.close()
    a, b = out["0"], out["1"]
    assert np.array_equal(a[0], b[0])
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x, y)
    for i in (3, 4, 5, 6):
        for x, y in zip(a[i], b[i]):
            assert np.array_equal(x, y)
    for i in (2, 7):
        assert a[i].shape == b[i].shape
        assert np.abs(a[i] - b[i]).max() <= 1e-13
        assert np.abs(np.diag(b[i]) - 1.0).max() < 1e-8


@pytest.mark.parametrize("n", [3000, 1 << 18, 1 << 20])
def test_window_major_partials_bitwise_equal_value_major(ctx, n, monkeypatch):
    """Round 6: factor groups over long grids store the one-sweep Arnoldi step's window partials
    window-major (each value group one whole 128-byte line) and reduce them in two levels
    (red_d1_block); one stream and fused launches keep value-major partials (red256_block).  Both
    reduces sum in the same order, so the layout never changes a bit: the records and bases of a
    grouped handle with window-major partials (forced at every size in a subprocess,
    TKHIP_D1_PGRP_MIN=0; one split at n = 3000, several at 2^18 and 2^20) equal those of a
    one-stream handle of the same factors, bit for bit."""
    import hashlib
    import json
    import subprocess
    import sys
    tk = __import__("tkamd")
    d, K = 3, 30
    code = r'''
import hashlib, json, sys
sys.path[:0] = %r
import numpy as np
import tkamd as tk
n, d, K = %d, %d, %d
ctx = tk.Context(0)
mats = [tk.DeviceMatrix(ctx, tk.assemble_matrix(n, c)) for c in ("Laplace", "ConvDiff")]
bs = [v / np.linalg.norm(v) for v in (np.random.default_rng(1000 + s).random(n) for s in range(d))]
dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, d, 0, [mats[s %% 2] for s in range(d)], bs, K)
assert dev.factor_groups == 2 and dev.arnoldi_sweeps == 1
dev.init(False)
dev.sweep(0, K)
rec = dev.records(0, K + 1)
V = [hashlib.sha256(dev.basis(s, 0, K).tobytes()).hexdigest() for s in range(d)]
print(json.dumps({"rec": hashlib.sha256(rec.tobytes()).hexdigest(), "V": V}))
''' % (sys.path, n, d, K)
    env = dict(os.environ, TKHIP_D1_PGRP_MIN="0")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    got = json.loads(p.stdout.strip().splitlines()[-1])
    monkeypatch.setenv("TKHIP_FACTOR_GROUPS", "1")
    mats = [tk.DeviceMatrix(ctx, tk.assemble_matrix(n, c)) for c in ("Laplace", "ConvDiff")]
    bs = [v / np.linalg.norm(v) for v in (np.random.default_rng(1000 + s).random(n) for s in range(d))]
    dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, d, 0, [mats[s % 2] for s in range(d)], bs, K)
    assert dev.factor_groups == 1
    dev.init(False)
    dev.sweep(0, K)
    rec = dev.records(0, K + 1)
    V = [hashlib.sha256(dev.basis(s, 0, K).tobytes()).hexdigest() for s in range(d)]
    dev.close()
    for m in mats:
        m.close()
    assert got["rec"] == hashlib.sha256(rec.tobytes()).hexdigest()
    assert got["V"] == V
