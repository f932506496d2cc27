"""Multi-rank path on CPU (gloo, world_size 2 and 3): the factor partition plus the
per-step all-reduce of records must reproduce the single-process ConvergenceData
bit for bit (the partition does not change any per-factor arithmetic, and the
all-reduce only adds zeros to each factor's record).  Workers run in fresh processes
launched by torch.distributed.run (127.0.0.1 rendezvous)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import tkamd
from _fake_device import backend

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _single(method, d, K, n=200, tol=1e-9, want_x=False, shared=False):
    rng = np.random.default_rng(777)
    if shared:
        bs = rng.random(n)
        b = [bs / np.linalg.norm(bs) for _ in range(d)]
    else:
        b = [x / np.linalg.norm(x) for x in (rng.random(n) for _ in range(d))]
    A = tkamd.KroneckerMatrix.gallery(tkamd.SymInstance, d, n, tkamd.Laplace)
    conv = tkamd.ConvergenceData(K)
    x = tkamd.tensorkrylov(conv, A, b, tol, K, method, backend=backend)
    return (conv, x) if want_x else conv


def _launch(tmp_path, world, method, d, K, *extra, env_extra=None):
    out = str(tmp_path / "res")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "dist", "worker.py"), out, method, str(d), str(K)] + [str(e) for e in extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return [json.load(open("%s.%d.json" % (out, k))) for k in range(world)]


@pytest.mark.parametrize("world,method,d,K", [(2, "TensorArnoldi", 4, 20), (3, "TensorLanczosReorth", 5, 15)])
def test_partitioned_run_equals_single_process(tmp_path, world, method, d, K):
    out = str(tmp_path / "res")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "dist", "worker.py"), out, method, str(d), str(K)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = [json.load(open("%s.%d.json" % (out, k))) for k in range(world)]
    ref = _single(method, d, K)
    owned = sorted(s for rr in res for s in rr["local"])
    assert owned == list(range(d))
    for rr in res:                       # every rank ends with the same compressed residuals
        # (each rank evaluates the iterations k = rank mod world and reads the others' from the
        # shared-memory mailbox: tk_solver_share)
        assert rr["eval_split"] == [world, rr["rank"]]
        assert rr["niter"] == ref.niterations
        assert np.array_equal(rr["relres"], ref.relative_residual_norm)
        assert np.array_equal(rr["proj"], ref.projected_residual_norm)
        assert np.array_equal(rr["orth"], ref.orthogonality_data)


def test_partition_term_split_slices():
    """More ranks than factors: rank r >= d replicates factor r % d and the ranks holding a
    factor split its t exp-sum terms into consecutive near-equal slices covering 0..t."""
    d, N, t = 3, 8, 17
    parts = [tkamd.Partition(d, N, r) for r in range(N)]
    assert [p.first for p in parts] == [r % d for r in range(N)]
    assert all(p.nf == 1 for p in parts)
    assert [p.replica for p in parts] == [r >= d for r in range(N)]
    for s in range(d):
        sl = sorted(p.terms(t) for p in parts if p.first == s)
        assert sl[0][0] == 0 and sl[-1][1] == t
        assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
        assert max(c1 - c0 for c0, c1 in sl) - min(c1 - c0 for c0, c1 in sl) <= 1
    off = tkamd.Partition(d, N, 5, term_split=False)       # the old behaviour: idle ranks
    assert (off.nf, off.replica, off.terms(t)) == (0, False, (0, t))
    assert tkamd.Partition(4, 4, 2).terms(t) == (0, t) and not tkamd.Partition(4, 4, 2).replica


@pytest.mark.parametrize("world,method,d", [(3, "TensorArnoldi", 2), (5, "TensorLanczosReorth", 2)])
def test_term_split_replicas_equal_single_process(tmp_path, world, method, d):
    """world > d: the replicas send zero rows into the all-reduce, so every rank's trajectory
    is the single-process one bit for bit; at convergence the ranks holding factor s return
    consecutive column slices of X_s = V_s Y_s that together are the single-process X_s."""
    n, K, tol = 30, 29, 0.5          # (shared rhs, random_rhs: converges mid-way)
    res = _launch(tmp_path, world, method, d, K, n, tol, "shared")
    ref, xref = _single(method, d, K, n=n, tol=tol, want_x=True, shared=True)
    assert xref is not None
    for rr in res:
        assert rr["niter"] == ref.niterations
        assert np.array_equal(rr["relres"], ref.relative_residual_norm)
        assert np.array_equal(rr["proj"], ref.projected_residual_norm)
    t = len(xref.lam)
    assert t >= 2
    for s in range(d):
        cols = np.full(t, -1)
        for rr in res:
            if rr["x_factors"] != [s]:
                continue
            c0, c1 = rr["x_terms"]
            assert np.array_equal(rr["x_lam"], xref.lam[c0:c1])
            X = np.asarray(rr["x_fmat"][0]).reshape(n, c1 - c0)
            if c1 > c0:
                assert np.abs(X - xref.fmat[s][:, c0:c1]).max() <= 1e-14 * np.abs(xref.fmat[s]).max()
            cols[c0:c1] += 1
        assert (cols == 0).all()         # every term exactly once


@pytest.mark.parametrize("method,K", [("TensorArnoldi", 21), ("TensorLanczos", 20)])
def test_deferred_gram_multirank_no_convergence(tmp_path, monkeypatch, method, K):
    """with a deferred Gram and no convergence the driver ends with factor 1's
    Gram on ONE rank.  A pending column must be flushed by every rank first -- the flush starts
    record all-reduces, and the ABI (and this stand-in) refuse a Gram on a multi-rank handle
    while a column is pending.  Odd and even nmax, tolerance never met: the orthogonality data
    equal the single process' bit for bit."""
    monkeypatch.setenv("TK_FAKE_GRAM_DEFERRED", "1")
    res = _launch(tmp_path, 2, method, 4, K, 60, 1e-10, env_extra={"TK_FAKE_GRAM_DEFERRED": "1"})
    ref = _single(method, 4, K, n=60, tol=1e-10)
    assert ref.niterations == K
    for rr in res:
        assert rr["niter"] == ref.niterations
        assert np.array_equal(rr["relres"], ref.relative_residual_norm)
        assert np.array_equal(rr["orth"], ref.orthogonality_data)
        assert np.count_nonzero(rr["orth"][1:]) == K - 1
