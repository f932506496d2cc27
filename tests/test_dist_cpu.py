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


def _single(method, d, K):
    n = 200
    rng = np.random.default_rng(777)
    b = [x / np.linalg.norm(x) for x in (rng.random(n) for _ in range(d))]
    A = tkamd.KroneckerMatrix.gallery(tkamd.SymInstance, d, n, tkamd.Laplace)
    conv = tkamd.ConvergenceData(K)
    tkamd.tensorkrylov(conv, A, b, 1e-9, K, method, backend=backend)
    return conv


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
    for rr in res:                       # every rank evaluates the same compressed residual
        assert rr["niter"] == ref.niterations
        assert np.array_equal(rr["relres"], ref.relative_residual_norm)
        assert np.array_equal(rr["proj"], ref.projected_residual_norm)
        assert np.array_equal(rr["orth"], ref.orthogonality_data)
