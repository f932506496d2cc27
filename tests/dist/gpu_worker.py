"""One rank of a multi-process job on ONE GPU -- TEST INFRASTRUCTURE ONLY
(tests/test_gpu_multirank.py).

RCCL refuses several ranks on one device, so the ranks join through the test build's
shared-memory stand-in for RCCL (tests/_build/libtkhip_test.so, TKHIP_LIB; tk_comm_init_test).
Everything else is the product path at its defaults: the factor partition, factor groups,
per-factor signal words, alternating send buffers, coalesced slot guards, fused launches where
the default picks them, replicas, and the evaluation split's shared-memory mailbox.

argv: spec.json out_prefix.  The spec lists cases; every rank runs all of them in order (the
same call sequence on every rank) and saves its results to out_prefix.<rank>.npz."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tensorkrylov.jl_amd")]

import numpy as np  # noqa: E402

import tkamd as tk  # noqa: E402

METHOD = {"TensorArnoldi": 0, "TensorLanczos": 1, "TensorLanczosReorth": 2}


def case_inputs(c):
    """(kron, csc, b) of a case: the gallery matrix and either distinct U(0,1) right-hand
    sides (seed 1000 + s, as bench.py) or one shared one (random_rhs)."""
    d, n, cls = c["d"], c["n"], c["cls"]
    inst = tk.NonSymInstance if cls == "ConvDiff" else tk.SymInstance
    csc = tk.assemble_matrix(n, cls)
    kron = tk.KroneckerMatrix(inst, [csc] * d, cls)
    if c.get("shared"):
        b0 = np.random.default_rng(777).random(n)
        b = [b0 / np.linalg.norm(b0) for _ in range(d)]
    else:
        b = [v / np.linalg.norm(v) for v in (np.random.default_rng(1000 + s).random(n) for s in range(d))]
    return kron, csc, b


def y_of(c):
    rng = np.random.default_rng(7)
    return [rng.standard_normal((c["K"], c["t"])) for _ in range(c["d"])]


def run_records(ctx, part, c, out, tag):
    """The device path alone: init, the K steps as one sweep, the flush, V*Y over this rank's
    term slice; every factor's records (the all-reduced slots), the local basis and X."""
    kron, csc, b = case_inputs(c)
    A = tk.DeviceMatrix(ctx, csc)
    dev = tk.DeviceDecomposition(ctx, METHOD[c["method"]], c["d"], part.first, [A] * part.nf,
                                 [b[s] for s in part.local()], c["K"], n=c["n"])
    if part.replica:
        dev.set_replica()
    K = c["K"]
    dev.init(False)
    dev.sweep(0, K)
    Y = y_of(c)
    c0, c1 = part.terms(c["t"])
    X = dev.basis_mul(K, [Y[s][:, c0:c1] for s in part.local()])     # (the flush first)
    out[tag + "recs"] = dev.records(0, K + 2)
    out[tag + "groups"] = np.array([dev.factor_groups, int(dev.exchange_signalled), dev.arnoldi_sweeps])
    for i, s in enumerate(part.local()):
        # the basis by its SHA-256 (bitwise), X by every 64th row (a tolerance: the MFMA V*Y
        # groups the terms by t, and a replica's slice has another t)
        out[tag + "V%d" % s] = np.frombuffer(hashlib.sha256(dev.basis(i, 0, K + 1).tobytes()).digest(), np.uint8)
        out[tag + "X%d" % s] = X[i][::64]
    out[tag + "terms"] = np.array([c0, c1])
    dev.close()
    A.close()


def run_solve(ctx, part, c, out, tag):
    """tkamd.tensorkrylov (the native pipelined loop with the evaluation split)."""
    kron, csc, b = case_inputs(c)
    conv = tk.ConvergenceData(c["K"])
    x = tk.tensorkrylov(conv, kron, b, c["tol"], c["K"], c["method"], ctx=ctx, partition=part)
    out[tag + "relres"] = conv.relative_residual_norm
    out[tag + "proj"] = conv.projected_residual_norm
    out[tag + "orth"] = conv.orthogonality_data
    out[tag + "niter"] = np.array([conv.niterations])
    sp = getattr(conv, "eval_split", None)
    out[tag + "split"] = np.array(sp if sp else [0, 0])
    if x is not None:
        out[tag + "lam"] = x.lam
        out[tag + "terms"] = np.array(x.terms)
        for i, s in enumerate(x.factors):
            out[tag + "X%d" % s] = x.fmat[i]


def main():
    spec = json.load(open(sys.argv[1]))
    prefix = sys.argv[2]
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    ctx = tk.Context(0)
    ctx.init_comm_test(spec["key"], world, rank)
    out = {"rccl_nranks": np.array([ctx.comm_count()])}
    for i, c in enumerate(spec["cases"]):
        part = tk.Partition(c["d"], world, rank)
        (run_solve if c["kind"] == "solve" else run_records)(ctx, part, c, out, "c%d_" % i)
        out["c%d_local" % i] = np.array(list(part.local()) + [-1 if part.replica else -2])
    np.savez(prefix + ".%d.npz" % rank, **out)
    ctx.sync()
    ctx.allreduce_host(np.zeros(1))      # (a last collective: every rank has saved)
    ctx.close()


if __name__ == "__main__":
    main()
