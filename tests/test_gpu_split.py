"""The evaluation split over ranks (tk_solver_share / tk_solver_share_emulated)
through the native pipelined driver on the GPU.

With N ranks, rank r evaluates only the iterations k = r (mod N) of tensorkrylov!'s loop
(compressed solve + residual, src/tensor_krylov_method.jl:72-103) and takes the others'
results from their owners.  One GPU cannot host two RCCL ranks, so the owners are emulated
the way bench.py --emulate-ranks does it: the other factors' records come from a full run
(tk_solver_overlay) and the other ranks' results from that run's per-iteration table
(tk_solver_share_emulated).  The real mailbox between processes is covered on CPU
(tests/test_dist_cpu.py: gloo world 2/3/5; tests/test_xsched.py: concurrent ranks).

Checked for every rank of N = 2, 3, 4: the relative-residual trajectory, the projected
residuals and the iteration count bitwise equal to the single-rank run, only the owned
iterations evaluated locally, and -- on a converging run, including convergence at an
iteration another rank owns -- the returned (lambda, X_s) bitwise equal to the full run's."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _case(tk, name):
    """golden10: the recorded RHS of experiments/data/reproduction_data (decoded in
    tests/golden), d = 10, n = 200, Laplace / ConvDiff -- no convergence within K;
    shared3: d = 3, n = 30 Laplace with a shared U(0,1) RHS, converging at k = 12 (tol 0.3)
    (tests/test_gpu_solution.py)."""
    if name == "shared3":
        n, d = 30, 3
        b0 = np.random.default_rng(777).random(n)
        b0 = b0 / np.linalg.norm(b0)
        return tk.KroneckerMatrix.gallery(tk.SymInstance, d, n, tk.Laplace), [b0.copy() for _ in range(d)]
    cls = name[len("golden10-"):]
    g = json.load(open(os.path.join(HERE, "golden", "reproduction.json")))
    key = "nonsym_new" if cls == "ConvDiff" else "laplace_new"
    b = np.array(g[key]["rhs"]["10"])
    inst = tk.NonSymInstance if cls == "ConvDiff" else tk.SymInstance
    kron = tk.KroneckerMatrix.gallery(inst, 10, len(b), getattr(tk, cls))
    return kron, [b.copy() for _ in range(10)]


@pytest.mark.parametrize("name,tol,K,ranks", [("golden10-ConvDiff", 1e-9, 50, (2, 3, 4)),
                                             ("golden10-Laplace", 1e-9, 40, (2, 3, 4)),
                                             ("shared3", 0.3, 29, (2, 3))])
def test_emulated_evaluation_split_bitwise(ctx, name, tol, K, ranks):
    tk = __import__("tkamd")
    kron, b = _case(tk, name)
    d, n = len(b), len(b[0])
    conv1 = tk.ConvergenceData(K)
    x1 = tk.tensorkrylov(conv1, kron, [v.copy() for v in b], tol, K, "TensorArnoldi", ctx=ctx)
    res1 = conv1.native_results
    k_end = int(np.nonzero(~np.isnan(res1[:, 0]))[0].max()) + 1   # the last iteration consumed
    assert np.all(res1[1:k_end, 5] >= 0)            # (all evaluated on the single rank)
    assert (x1 is not None) == (name == "shared3")  # the converging case converges ...
    assert (k_end < K) == (name == "shared3")       # ... before nmax
    # the other factors' records of a full run (bench.py --emulate-ranks)
    A = tk.DeviceMatrix(ctx, kron[0])
    full = tk.DeviceDecomposition(ctx, tk._lib.TK_ARNOLDI, d, 0, [A] * d, b, K)
    full.init(False)
    full.sweep(0, K)
    overlay = np.zeros((K + 2, d, full.m))
    overlay[:K + 1] = full.records(0, K + 1)
    full.close()
    A.close()
    for N in ranks:
        # (converging: the ranks r != k_end % N end on an iteration another rank evaluated)
        for r in range(N):
            part = tk.Partition(d, N, r, term_split=False)
            conv = tk.ConvergenceData(K)
            x = tk.tensorkrylov(conv, kron, [v.copy() for v in b], tol, K, "TensorArnoldi", ctx=ctx,
                                partition=part, overlay=overlay, eval_overlay=res1)
            assert tuple(conv.eval_split) == (N, r)
            assert conv.niterations == conv1.niterations
            assert np.array_equal(conv.relative_residual_norm, conv1.relative_residual_norm)
            assert np.array_equal(conv.projected_residual_norm, conv1.projected_residual_norm)
            res = conv.native_results
            for k in range(2, k_end + 1):
                assert (res[k - 1, 5] >= 0) == (k % N == r), (N, r, k)   # evaluated here iff owned
            if x1 is not None:
                assert x is not None and np.array_equal(x.lam, x1.lam)
                for i, s in enumerate(part.local()):
                    assert np.array_equal(x.fmat[i], x1.fmat[s]), (N, r, s)
