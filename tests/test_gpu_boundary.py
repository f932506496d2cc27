"""The C-ABI boundary from a non-Python caller, and its failure behaviour.

  * tests/c/julia_glue_replay.c (built by __graft_entry__.build()) replays the Julia drop-in's
    ccall sequence with the glue's literal 1-based record offsets
    (julia/TensorKrylovHIP.jl:84-105, 227-255): the H, b-tilde and Gram rows it assembles
    must equal the Python mirror's (tkamd.decompositions) bit for bit -- same library, same
    kernels, so any difference is an offset or sequencing error in one of the two callers.
  * a duplicate (row, column) entry in a non-canonical CSC is added like Julia's scatter
    mul! (both products in turn), never stored over (the DIA format is refused for it).
  * a failing step marks the handle failed instead of leaving the records exchange waiting
    for a signal that never comes: later steps are refused and destroy returns.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import tk_oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = os.path.join(ROOT, "tests", "c", "_build", "julia_glue_replay")


def _tk():
    import tkamd
    return tkamd


@pytest.mark.parametrize("method", ["TensorArnoldi", "TensorLanczos", "TensorLanczosReorth"])
def test_c_caller_replays_julia_glue(ctx, method, tmp_path):
    tk = _tk()
    code = {"TensorArnoldi": 0, "TensorLanczos": 1, "TensorLanczosReorth": 2}[method]
    d, n, K = 3, 5000, 30
    rng = np.random.default_rng(404)
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    rhs = tmp_path / "rhs.bin"
    np.concatenate(bs).tofile(rhs)
    out = tmp_path / "out.bin"
    assert os.path.exists(REPLAY), "build() did not produce %s" % REPLAY
    r = subprocess.run([REPLAY, str(code), str(d), str(n), str(K), str(rhs), str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(out, dtype=np.float64)
    per = (K + 2) ** 2 + (K + 1) + (K + 1) ** 2
    assert raw.size == d * per

    csc = tk.assemble_matrix(n, "Laplace")
    A = tk.KroneckerMatrix(tk.SymInstance, [csc] * d, tk.Laplace)
    td = {"TensorArnoldi": tk.TensorArnoldi, "TensorLanczos": tk.TensorLanczos,
          "TensorLanczosReorth": tk.TensorLanczosReorth}[method](A, K, ctx=ctx, track_all_gram=2)
    td.orthonormalize_first([b.copy() for b in bs])
    for k in range(2, K + 1):
        td.orthonormalize(k)
    for s in range(d):
        blk = raw[s * per:(s + 1) * per]
        Hj = blk[:(K + 2) ** 2].reshape(K + 2, K + 2, order="F")
        btj = blk[(K + 2) ** 2:(K + 2) ** 2 + K + 1]
        Gj = blk[(K + 2) ** 2 + K + 1:].reshape(K + 1, K + 1, order="F")
        # the glue's H is (kmax+2)^2; its last column is never written
        assert np.array_equal(Hj[:, :K + 1], td.H[s]), (method, s)
        assert not Hj[:, K + 1].any()
        # b-tilde of columns 0..K-1 (column K is written by the flush neither caller ran)
        assert np.array_equal(btj[:K], td.btilde[s, :K]), (method, s)
        if s in td.gram:
            assert np.array_equal(Gj[:K, :K], td.gram[s][:K, :K]), (method, s)
        else:
            assert not Gj.any()
    assert 0 in td.gram                       # factor 1's Gram rows (orthogonality_data)
    td.close()


def test_duplicate_csc_entries_are_summed_like_the_scatter(ctx):
    """A[0,0] given as two entries 1.5 + 0.5 of a tridiagonal matrix: Julia's mul! adds
    nz1*x + nz2*x in turn; the device must not pick DIA (one slot per position)."""
    tk = _tk()
    n = 300
    colptr, rowval, nz = tk.assemble_matrix(n, "Laplace")
    nz = nz / nz.max()
    # split the (0, 0) entry (column 0's second stored entry is row 1)
    rowval = np.concatenate([[0, 0], rowval[1:]])
    nz = np.concatenate([[nz[0] * 0.75, nz[0] * 0.25], nz[1:]])
    colptr = colptr.copy()
    colptr[1:] += 1
    csc = (colptr, rowval, nz)
    A = tk.DeviceMatrix(ctx, csc)
    assert A.format <= 0                       # not DIA
    x = np.random.default_rng(3).standard_normal(n)
    assert np.array_equal(A.matvec(x), O.csc_matvec(csc, x))
    A.close()


def _in_test_build(code, env_extra, timeout=180):
    """Run `code` in a fresh process on the test build (tests/_build/libtkhip_test.so via
    TKHIP_LIB): the switches that inject failures exist only there, never in libtkhip.so."""
    import sys
    lib = os.path.join(ROOT, "tests", "_build", "libtkhip_test.so")
    assert os.path.exists(lib), "build() did not produce %s" % lib
    env = dict(os.environ, TKHIP_LIB=lib, **env_extra)
    pre = "import sys\nsys.path[:0] = %r\n" % [ROOT, os.path.join(ROOT, "tensorkrylov.jl_amd")]
    p = subprocess.run([sys.executable, "-c", pre + code], env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return p.stdout


def test_product_library_has_no_test_switches():
    """the switches that skip work, drop guards or inject failures are compiled
    into the test build only."""
    lib = os.path.join(ROOT, "tensorkrylov.jl_amd", "tkamd", "libtkhip.so")
    blob = open(lib, "rb").read()
    for name in (b"TKHIP_TEST_SKIP", b"TKHIP_TEST_XCH_SKIP", b"TKHIP_TEST_NO_GUARD", b"TKHIP_TEST_SHARED_XSIG",
                 b"TKHIP_TEST_XCH_STALL", b"TKHIP_TEST_FAIL_STEP", b"TKHIP_TEST_FUSE_SPIN", b"tk_comm_init_test"):
        assert name not in blob, name


def test_failed_step_refuses_later_steps_and_destroys():
    """Step 3 reports an injected error on a handle that routes its records through the RCCL
    exchange (1-rank communicator): step 4 and flush are refused with TK_ERR_STATE and
    destroy returns (no exchange left waiting for the failed step's signal)."""
    out = _in_test_build(r'''
import numpy as np, pytest
import tkamd as tk
n, K, d = 3000, 10, 2
csc = tk.assemble_matrix(n, "Laplace")
rng = np.random.default_rng(9)
bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
c2 = tk.Context(0)
c2.init_comm(tk.unique_id(), 1, 0)
A = tk.DeviceMatrix(c2, csc)
dev = tk.DeviceDecomposition(c2, tk._lib.TK_ARNOLDI, d, 0, [A] * d, bs, K)
dev.init()
for j in range(3):
    dev.step(j)
with pytest.raises(tk.TKError, match="injected"):
    dev.step(3)
with pytest.raises(tk.TKError, match="earlier step"):
    dev.step(4)
with pytest.raises(tk.TKError, match="earlier step"):
    dev.flush()
dev.close()
A.close()
c2.close()
print("OK")
''', {"TKHIP_EXCHANGE_ALWAYS": "1", "TKHIP_TEST_FAIL_STEP": "3"})
    assert out.strip().endswith("OK")


def test_fused_wait_that_gives_up_is_reported():
    """a fused one-sweep launch whose bounded wait for its in-launch reducers gives
    up (forced here: TKHIP_TEST_FUSE_SPIN=1, one poll) sets the context's error word; the
    records read after the sync then fail with TK_ERR_INTERNAL instead of returning wrong
    values with TK_OK, and so do tk_ctx_sync and tk_decomp_destroy."""
    out = _in_test_build(r'''
import numpy as np, pytest
import tkamd as tk
ctx = tk.Context(0)
n, K, d = 1 << 17, 24, 4
csc = tk.assemble_matrix(n, "ConvDiff")
A = tk.DeviceMatrix(ctx, csc)
bs = [v / np.linalg.norm(v) for v in (np.random.default_rng(1000 + s).random(n) for s in range(d))]
dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, d, 0, [A] * d, bs, K)
assert dev.factor_groups == 2
dev.init(False)
with pytest.raises(tk.TKError, match="gave up"):
    dev.sweep(0, K)                 # (red_flush at the sweep's end may already see it) ...
    dev.records(0, K + 1)           # ... else the records read after the sync do
with pytest.raises(tk.TKError, match="gave up"):
    ctx.sync()
st = ctx._lib.tk_decomp_destroy(dev.h)      # (released either way; the status says why)
dev.h = None
assert st == 8, st                          # TK_ERR_INTERNAL
print("OK")
''', {"TKHIP_TEST_FUSE_SPIN": "1", "TKHIP_D1_FUSE": "1", "TKHIP_RED_MM": "0"})
    assert out.strip().endswith("OK")


@pytest.mark.parametrize("comm", [False, True])
def test_rank_without_factors(ctx, comm, monkeypatch):
    """A rank of a job with more ranks than factors (d < N) owns no factor: create, init, the
    sweep, the flush and the records exchange run with every launch skipped, and its records
    are all zero (the all-reduce adds nothing) -- forced through the RCCL path on a 1-rank
    communicator too."""
    tk = _tk()
    n, K, d = 3000, 12, 3
    c = ctx
    if comm:
        c = tk.Context(0)
        c.init_comm(tk.unique_id(), 1, 0)
        monkeypatch.setenv("TKHIP_EXCHANGE_ALWAYS", "1")
    for method in (0, 1, 2):
        dev = tk.DeviceDecomposition(c, method, d, d, [], [], K, n=n)
        rec0 = dev.init()
        dev.sweep(0, K)
        assert dev.basis_mul(K, [], want=True) == []
        recs = dev.records(0, K + 2)
        dev.close()
        assert not np.any(rec0)
        assert not np.any(recs)
    if comm:
        c.close()


@pytest.mark.parametrize("method", [0, 1, 2])
def test_replica_sends_zero_rows_and_splits_terms(ctx, method, monkeypatch):
    """Exp-sum-term split (tk_decomp_set_replica; more ranks than factors): a replica runs the
    owner's steps -- its basis is the owner's bit for bit -- but sends zero rows into the
    records all-reduce (on a 1-rank communicator every received record is zero), and V*Y on
    a slice Y[:, c0:c1] of the terms is the owner's X[:, c0:c1].  set_replica is refused on a
    handle without a records exchange and after init."""
    tk = _tk()
    n, K, d, t = 3000, 12, 2, 7
    csc = tk.assemble_matrix(n, "Laplace")
    rng = np.random.default_rng(5)
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    Y = [rng.standard_normal((K, t)) for _ in range(d)]
    A0 = tk.DeviceMatrix(ctx, csc)
    own = tk.DeviceDecomposition(ctx, method, d, 0, [A0] * d, bs, K)
    with pytest.raises(tk.TKError, match="replica needs"):
        own.set_replica()
    own.init(False)
    own.sweep(0, K)
    Xo = own.basis_mul(K, Y)
    Vo = [own.basis(f, 0, K + 1) for f in range(d)]
    own.close()
    A0.close()

    c = tk.Context(0)
    c.init_comm(tk.unique_id(), 1, 0)
    monkeypatch.setenv("TKHIP_EXCHANGE_ALWAYS", "1")
    A1 = tk.DeviceMatrix(c, csc)
    rep = tk.DeviceDecomposition(c, method, d, 0, [A1] * d, bs, K)
    rep.set_replica()
    rec0 = rep.init()
    with pytest.raises(tk.TKError, match="after tk_decomp_init"):
        rep.set_replica()
    rep.sweep(0, K)
    c0, c1 = 2, 6
    Xr = rep.basis_mul(K, [y[:, c0:c1] for y in Y])
    recs = rep.records(0, K + 1)
    Vr = [rep.basis(f, 0, K + 1) for f in range(d)]
    empty = rep.basis_mul(K, [y[:, :0] for y in Y])        # an empty slice of the terms
    rep.close()
    A1.close()
    c.close()
    assert not np.any(rec0) and not np.any(recs)
    for f in range(d):
        assert np.array_equal(Vr[f], Vo[f])
        ref = Xo[f][:, c0:c1]
        assert Xr[f].shape == ref.shape and empty[f].shape == (n, 0)
        assert np.abs(Xr[f] - ref).max() <= 1e-14 * np.abs(ref).max()


def test_exchange_wait_has_a_deadline():
    """A records exchange that never completes (TKHIP_TEST_XCH_STALL, test build: the
    all-reduce of the group holding slot 7 (slots 5..8) waits on a word nobody writes -- a peer
    that never joins) ends in TK_ERR_RCCL after TKHIP_WAIT_S, naming the slot / step and RCCL's
    state, instead of spinning forever; afterwards the communicator refuses further collectives
    at once and destroy returns (its buffers are left to process exit).  1-rank communicator."""
    out = _in_test_build(r'''
import time
import numpy as np, pytest
import tkamd as tk
n, K, d = 3000, 12, 2
csc = tk.assemble_matrix(n, "Laplace")
rng = np.random.default_rng(11)
bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
c = tk.Context(0)
c.init_comm(tk.unique_id(), 1, 0)
A = tk.DeviceMatrix(c, csc)
dev = tk.DeviceDecomposition(c, tk._lib.TK_ARNOLDI, d, 0, [A] * d, bs, K)
dev.init(False)
dev.sweep(0, K)                             # enqueues without waiting
r1 = dev.records(1, 5)                      # slots 1..4 went out before the stalled group
assert r1.shape == (4, d, dev.m) and (r1[:, :, dev.layout.beta] > 0).all()
t0 = time.time()
with pytest.raises(tk.TKError, match=r"error 5: records exchange: not complete after 2 s \(record slot 7 = step 6"):
    dev.records(7, 8)
assert time.time() - t0 < 30
with pytest.raises(tk.TKError, match="communicator is unusable"):
    dev.flush()
t0 = time.time()
dev.close()
A.close()
c.close()
assert time.time() - t0 < 30
print("OK")
''', {"TKHIP_EXCHANGE_ALWAYS": "1", "TKHIP_TEST_XCH_STALL": "7", "TKHIP_WAIT_S": "2"})
    assert out.strip().endswith("OK")


def test_reduce_handoff_self_check(ctx):
    """the one-sweep reduce's relaxed hand-off is confirmed at the process's
    first decomposition by a self-check against the memory-model form (tk_reduce_handoff: 0
    = relaxed, checked; 1 = the check found a difference and the process runs the memory-model
    form).  Either way the records are bitwise those of the memory-model form: compared here
    with a process that forces it (TKHIP_RED_MM=1), on a C2-sized factor pair."""
    import json
    import subprocess
    import sys
    tk = _tk()
    code = r'''
import json, sys
sys.path[:0] = %r
import numpy as np
import tkamd as tk
ctx = tk.Context(0)
n, K = 1 << 20, 24
csc = tk.assemble_matrix(n, "Laplace")
A = tk.DeviceMatrix(ctx, csc)
bs = [np.random.default_rng(1000 + s).random(n) for s in range(2)]
dev = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, 2, 0, [A, A], [b / np.linalg.norm(b) for b in bs], K)
dev.init(False)
dev.sweep(0, K)
r = dev.records(0, K + 1)
print(json.dumps({"handoff": int(tk._lib.lib().tk_reduce_handoff()), "sweeps": dev.arnoldi_sweeps,
                  "rec": r.ravel().tolist()}))
''' % (sys.path,)
    out = {}
    for v in (None, "1"):
        env = dict(os.environ)
        env.pop("TKHIP_RED_MM", None)
        if v:
            env["TKHIP_RED_MM"] = v
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
        assert p.returncode == 0, p.stderr[-2000:]
        out[v] = json.loads(p.stdout.strip().splitlines()[-1])
    assert out[None]["sweeps"] == 1
    assert out[None]["handoff"] in (0, 1)          # settled by the self-check
    assert out["1"]["handoff"] == 1                 # forced
    assert out[None]["rec"] == out["1"]["rec"]      # bitwise the memory-model form's records
    assert tk._lib.lib().tk_reduce_handoff() in (0, 1, 2)
