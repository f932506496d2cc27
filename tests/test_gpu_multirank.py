"""The native multi-rank exchange with real peer processes.

Reference shard point: src/orthogonal_bases.jl:162-180 (the factor fan-out) and the driver
loop src/tensor_krylov_method.jl:63-103.  RCCL refuses several ranks on one device, so 2 or 3
fresh worker processes share this GPU and join through the test build's shared-memory
stand-in for ncclAllReduce (tests/_build/libtkhip_test.so, tk_comm_init_test; the same call
sites as RCCL: the records exchange on the exchange stream and the host all-reduces).
Everything else runs at its defaults -- the contiguous factor partition, factor groups,
per-factor signal words, alternating send buffers, coalesced slot guards, replicas when N > d,
and the evaluation split's mailbox -- except the fused one-sweep launch (see _launch: it
assumes one process per GPU; tests/test_gpu_fused.py covers it under a forced exchange).  Done = every rank's records, bases, trajectories and solutions equal the
single process' bit for bit (X to 1e-14 where the MFMA V*Y groups terms by t)."""
import hashlib
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
TEST_LIB = os.path.join(HERE, "_build", "libtkhip_test.so")
sys.path.insert(0, os.path.join(HERE, "dist"))
from gpu_worker import case_inputs, y_of  # noqa: E402

C1 = dict(kind="records", d=4, n=1 << 18, cls="Laplace", method="TensorArnoldi", K=50, t=17)
C4 = dict(kind="records", d=10, n=1 << 17, cls="ConvDiff", method="TensorArnoldi", K=50, t=3)
LAN = dict(kind="records", d=4, n=1 << 17, cls="Laplace", method="TensorLanczos", K=40, t=9)
REO = dict(kind="records", d=4, n=1 << 16, cls="Laplace", method="TensorLanczosReorth", K=30, t=5)
S_C4 = dict(kind="solve", d=10, n=1 << 17, cls="ConvDiff", method="TensorArnoldi", K=50, tol=1e-9)
S_SH = dict(kind="solve", d=3, n=30, cls="Laplace", method="TensorArnoldi", K=29, tol=0.3, shared=True)
S_SH_LAN = dict(S_SH, method="TensorLanczos")
REP = dict(kind="records", d=2, n=1 << 16, cls="Laplace", method="TensorArnoldi", K=30, t=7)
S_REP = dict(kind="solve", d=2, n=30, cls="Laplace", method="TensorArnoldi", K=29, tol=0.3, shared=True)


def _launch(tmp_path, world, cases, env_extra=None):
    assert os.path.exists(TEST_LIB), "build() did not produce %s" % TEST_LIB
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"key": uuid.uuid4().hex[:16], "cases": cases}))
    prefix = str(tmp_path / "res")
    procs = []
    for r in range(world):
        # (no fused one-sweep launches, and the reduce hand-off forced instead of self-checked,
        # whose job runs fused: a fused launch's windows wait for reducers of the same launch
        # and rely on their dispatch order and residency -- which holds for one process per
        # GPU, the product's model, but not for ranks sharing one GPU, whose spinning windows
        # can hold the CUs another rank's reducers need; their bounded waits then give up)
        env = dict(os.environ, TKHIP_LIB=TEST_LIB, WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   RANK=str(r), LOCAL_RANK="0", TKHIP_WAIT_S="60", TKHIP_D1_FUSE="0", TKHIP_RED_MM="0",
                   **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist", "gpu_worker.py"), str(spec), prefix],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, e))
    for r, (rc, e) in enumerate(outs):
        assert rc == 0, "rank %d: %s" % (r, e[-3000:])
    res = [dict(np.load(prefix + ".%d.npz" % r)) for r in range(world)]
    for r in res:
        assert int(r["rccl_nranks"][0]) == world
    return res


def _single_records(tk, ctx, c):
    kron, csc, b = case_inputs(c)
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, {"TensorArnoldi": 0, "TensorLanczos": 1, "TensorLanczosReorth": 2}[c["method"]],
                                 c["d"], 0, [A] * c["d"], b, c["K"])
    dev.init(False)
    dev.sweep(0, c["K"])
    X = dev.basis_mul(c["K"], y_of(c))
    recs = dev.records(0, c["K"] + 2)
    V = [hashlib.sha256(dev.basis(s, 0, c["K"] + 1).tobytes()).digest() for s in range(c["d"])]
    dev.close()
    A.close()
    return recs, V, X


def _check_records(tk, ctx, res, i, c):
    recs, V, X = _single_records(tk, ctx, c)
    seen = np.zeros((c["d"], c["t"]), int)
    for r in res:
        tag = "c%d_" % i
        assert np.array_equal(r[tag + "recs"], recs), "rank records differ (case %d)" % i
        c0, c1 = r[tag + "terms"]
        for s in r[tag + "local"][:-1]:
            assert bytes(r[tag + "V%d" % s]) == V[s], "basis of factor %d differs" % s
            ref = X[s][::64, c0:c1]
            got = r[tag + "X%d" % s]
            assert got.shape == ref.shape
            if ref.size:
                assert np.abs(got - ref).max() <= 1e-14 * np.abs(X[s]).max()
            seen[s, c0:c1] += 1
    assert (seen == 1).all()            # every factor's every term exactly once (owners + replicas)


def _check_solve(tk, ctx, res, i, c, world):
    kron, csc, b = case_inputs(c)
    conv = tk.ConvergenceData(c["K"])
    x = tk.tensorkrylov(conv, kron, b, c["tol"], c["K"], c["method"], ctx=ctx)
    tag = "c%d_" % i
    for rank, r in enumerate(res):
        assert int(r[tag + "niter"][0]) == conv.niterations
        assert np.array_equal(r[tag + "relres"], conv.relative_residual_norm)
        assert np.array_equal(r[tag + "proj"], conv.projected_residual_norm)
        assert np.array_equal(r[tag + "orth"], conv.orthogonality_data, equal_nan=True)
        assert list(r[tag + "split"]) == [world, rank]      # the mailbox split ran
        assert (tag + "lam" in r) == (x is not None)
        if x is not None:
            c0, c1 = r[tag + "terms"]
            assert np.array_equal(r[tag + "lam"], x.lam[c0:c1])
            for s in r[tag + "local"][:-1]:
                ref = x.fmat[s][:, c0:c1]
                if ref.size:
                    assert np.abs(r[tag + "X%d" % s] - ref).max() <= 1e-14 * np.abs(x.fmat[s]).max()
    return x


@pytest.mark.parametrize("world", [2, 3])
def test_peer_ranks_records_equal_single_process(ctx, tmp_path, world):
    """C1 and C4 sized factor blocks (Arnoldi: one sweep, factor groups), TensorLanczos and
    TensorLanczosReorth: every rank's all-reduced records, its bases and its X equal the single
    process'."""
    tk = __import__("tkamd")
    cases = [C1, C4, LAN, REO]
    res = _launch(tmp_path, world, cases)
    for i, c in enumerate(cases):
        _check_records(tk, ctx, res, i, c)
    g = res[0]["c0_groups"]
    assert g[0] == 2 and g[1] == 1 and g[2] == 1   # factor groups, signal words, one sweep


@pytest.mark.parametrize("world", [2, 3])
def test_peer_ranks_solver_equal_single_process(ctx, tmp_path, world):
    """tkamd.tensorkrylov over the ranks (the native loop, its issue agreement and the
    evaluation split's mailbox): C4 without convergence, and a small shared-RHS Laplace that
    converges (Arnoldi and Lanczos): trajectories bitwise the single process', (lambda, X)
    equal on every rank."""
    tk = __import__("tkamd")
    cases = [S_C4, S_SH, S_SH_LAN]
    res = _launch(tmp_path, world, cases)
    _check_solve(tk, ctx, res, 0, S_C4, world)
    assert _check_solve(tk, ctx, res, 1, S_SH, world) is not None
    assert _check_solve(tk, ctx, res, 2, S_SH_LAN, world) is not None


def test_replica_rank_with_peers(ctx, tmp_path):
    """N = 3 > d = 2: rank 2 holds a replica of factor 0 -- it sends zero rows into the real
    three-way all-reduce and computes its own slice of the exp-sum terms of X_0."""
    tk = __import__("tkamd")
    res = _launch(tmp_path, 3, [REP, S_REP])
    assert list(res[2]["c0_local"]) == [0, -1]          # the replica
    _check_records(tk, ctx, res, 0, REP)
    _check_solve(tk, ctx, res, 1, S_REP, 3)


def test_peer_ranks_under_group_skew(ctx, tmp_path):
    """TKHIP_TEST_GROUP_DELAY_US holds factor group 0's stream back before every launch on
    every rank, so the other group runs ahead: the per-factor signal words must still make each
    exchange wait for every factor's row (the round-5 race), with real peers."""
    tk = __import__("tkamd")
    res = _launch(tmp_path, 2, [C4], env_extra={"TKHIP_TEST_GROUP_DELAY_US": "20"})
    _check_records(tk, ctx, res, 0, C4)
