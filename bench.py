#!/usr/bin/env python3
"""Benchmark: Krylov iterations/sec of the tensor-Krylov inner iteration on MI355X.

Workload (BASELINE.json configs[2], SURVEY.md 8d "C2"): d = 8 factors, n_s = 2^20
tridiagonal Laplacian (assemble_matrix(n, Laplace), src/tensor_struct.jl:48-57), fp64,
distinct b_s ~ U(0,1) (seed 1000+s) normalized, K = nmax = 50, TensorArnoldi (SpMV +
two-pass MGS per factor, src/orthogonal_bases.jl:15-37).

One bench "step" = one full device sweep of the iteration: V[:,1] = b/|b|, then the
K = 50 orthonormalize!(td, k) iterations over all d factors (k = 1..50; each one the
SpMV + MGS2 step of every factor plus update_rhs!'s <V_k, b_s> and factor 1's Gram
row), with the per-iteration RCCL all-reduce of the factors' records when N > 1, and
the final basis_tensor_mul! X_s = V_s Y_s (t = the exp-sum rank at k = 50), which also
finalizes the last basis column (fused into one pass over V for Arnoldi; the MFMA
V*Y kernel is timed beside it as basis_mul_mfma).
Inputs are resident in HBM before timing.  value = K * steps / time (whole job).
Factors are partitioned over ranks (one process per GPU): the total work is fixed, so
the scaling is STRONG (see DESIGN.md "Multi-GPU").

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C1|C2|C3|C4]
       N > 1: one rank per GPU.  Either launch it under torch.distributed.run yourself, or run
       `python bench.py --gpus N ...` and it starts `python -m torch.distributed.run
       --nproc-per-node N ... bench.py <same args>` as a child process (before anything here
       touches the GPU), passes rank 0's JSON line through and exits with the child's status.

Multi-rank control plane: the RCCL unique id is handed from rank 0 to the others
through a file keyed by the launcher's pid, and the barrier / max-over-ranks use RCCL
itself (tk_comm_allreduce_host).  torch is deliberately not imported: its wheel
bundles its own HIP runtime, and loading it next to libtkhip would put two HIP
runtimes in one process (DESIGN.md "Process model").
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tensorkrylov.jl_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
FP64_MFMA_PEAK_TF = 78.6

CONFIGS = {
    # name: (d, n, matrix class, method, K, instance)
    "C1": (4, 1 << 18, "Laplace", "TensorArnoldi", 50, "SymInstance"),
    "C2": (8, 1 << 20, "Laplace", "TensorArnoldi", 50, "SymInstance"),
    "C3": (5, 1 << 19, "RandSparseSPD", "TensorArnoldi", 50, "SymInstance"),
    "C4": (10, 1 << 17, "ConvDiff", "TensorArnoldi", 50, "NonSymInstance"),
}


def matrix_bytes(n, nnz, method="TensorArnoldi", sweeps=2, mat_bytes=None):
    """Bytes of A_s one SpMV reads (SURVEY.md 8d, int32 CSR: 12 nnz + 4 (n+1)); the one-sweep
    kernels read only what their banded storage holds (`mat_bytes`: 0 for a Toeplitz band,
    whose diagonals are 4 scalars)."""
    if sweeps == 1 and method in ("TensorArnoldi", "TensorLanczos") and mat_bytes is not None:
        return mat_bytes
    return 12 * nnz + 4 * (n + 1)


def alg_bytes_step(n, nnz, k, method="TensorArnoldi", sweeps=2, mat_bytes=None, with_matrix=True):
    """algorithmic bytes of one factor-step with k basis columns (int32 CSR).
    Arnoldi as two-sweep CGS2 (sweeps=2): B_spmv + 2 MGS passes + write V_{k+1} + the RHS
    dot.  One-sweep Arnoldi (sweeps=1, delayed reorthogonalization):
    V_1..V_{k-1} read once + the raw vector u read and written + V_k written (both SpMVs
    take their vector from LDS; <V_k, b> = norm(b) <V_k, V_1> needs no read of b) + the
    matrix bytes its storage must read (matrix_bytes).  Lanczos: B_spmv + read V_{k-1} +
    write V_{k+1} + the RHS dot; LanczosReorth adds the Gram row of the new column, 8n(k+1)
    (its redo steps are extra work, not counted).  with_matrix=False leaves out A_s's bytes
    (8d: factors sharing A_s in one batched SpMV count them once per batch)."""
    mb = matrix_bytes(n, nnz, method, sweeps, mat_bytes) if with_matrix else 0
    vec = 8 * n + 8 * n                      # SpMV x read, y written
    if method == "TensorArnoldi" and sweeps == 1:
        return 8 * n * (k - 1) + 3 * 8 * n + mb
    if method == "TensorArnoldi":
        return mb + vec + 2 * 8 * n * k + 8 * n + 8 * n
    if method == "TensorLanczos" and sweeps == 1:
        # one-sweep TTR (k_lan_1w / k_lan_1s): u_{k-1} and v_{k-1} read, v_k and u_k written,
        # <v_k, b>; the SpMV takes v_k from LDS (+ the tracked factor's Gram row,
        # gram_bytes_step).  Not counted: the paired-column layout's half (v_{k-1} read from
        # its pair after an even step, rewritten with v_k after an odd one), 8n per step
        return 5 * 8 * n + mb
    b = mb + vec + 8 * n + 8 * n + 8 * n
    if method == "TensorLanczosReorth":
        b += 8 * n * (k + 1)
    return b


def launcher_argv(n, argv, port):
    """The child command of a self-launched N-rank run: torch.distributed.run on this node,
    one rank per GPU, rendezvous on 127.0.0.1, each rank running this file with the same
    arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv):
    """`--gpus N` without a launcher: start the N ranks as a child (torch.distributed.run),
    wait for it and return its exit status.  Nothing in this process has loaded the HIP
    runtime or libtkhip (tkamd is imported only inside main's rank path), so the ranks own
    the GPUs alone; the ranks' stdout -- rank 0's JSON line -- is this process's stdout."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    p = subprocess.Popen(launcher_argv(n, argv, _free_port()), env=env)
    try:
        return p.wait()
    except KeyboardInterrupt:
        p.terminate()
        return p.wait()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--method", default=None, choices=["TensorArnoldi", "TensorLanczos", "TensorLanczosReorth"],
                    help="orthonormalization type (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU work per baseline mode (1 core, all cores)")
    ap.add_argument("--force-comm", action="store_true",
                    help="1 rank: still build an RCCL communicator and route every step's records "
                         "through the all-reduce on the exchange stream (the N>1 code path)")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="diagnostic: on 1 GPU run only rank 0's factor block of an N-rank "
                         "partition (records exchanged over a 1-rank communicator) to predict "
                         "the per-GPU step time at N GPUs; the JSON line is marked as emulated")
    ap.add_argument("--emulate-rank", type=int, default=0,
                    help="with --emulate-ranks: which rank's factor block to run (default 0, "
                         "the rank holding the tracked factor 1)")
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="skip the (untimed) full-driver measurement reported as end_to_end")
    ap.add_argument("--e2e-reps", type=int, default=5,
                    help="end-to-end solves; end_to_end reports the median (one solve is a few ms)")
    ap.add_argument("--pmc-mode", action="store_true",
                    help="run exactly one untimed sweep (for rocprofv3 --pmc passes)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # (before tkamd is imported: the parent never maps the HIP runtime)
        return launch_ranks(args.gpus, sys.argv[1:])

    import tkamd
    from tkamd import _lib as L

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but the launcher started %d rank(s) (WORLD_SIZE)" % (args.gpus, world))

    d, n, cls, method, K, inst = CONFIGS[args.config]
    if args.method:
        method = args.method
    ctx = tkamd.Context(local_rank)
    part = tkamd.Partition(d, world, rank)
    if args.emulate_ranks > 1 and world == 1:
        part = tkamd.Partition(d, args.emulate_ranks, args.emulate_rank, term_split=False)
        args.force_comm = os.environ.get("TK_EMULATE_NOCOMM") != "1"
    uid_path = None
    if world > 1:
        uid_path = exchange_uid(tkamd, rank)
        ctx.init_comm(uid_path[1], world, rank)
    elif args.force_comm:
        ctx.init_comm(tkamd.unique_id(), 1, 0)
        os.environ["TKHIP_EXCHANGE_ALWAYS"] = "1"

    csc = tkamd.assemble_matrix(n, cls)
    nnz = int(csc[0][-1])
    A = tkamd.DeviceMatrix(ctx, csc)
    bs = []
    for s in part.local():
        b = np.random.default_rng(1000 + s).random(n)
        bs.append(b / np.linalg.norm(b))
    mcode = {"TensorArnoldi": L.TK_ARNOLDI, "TensorLanczos": L.TK_LANCZOS,
             "TensorLanczosReorth": L.TK_LANCZOS_REORTH}[method]
    dev = tkamd.DeviceDecomposition(ctx, mcode,
                                    d, part.first, [A] * part.nf, bs, K, n=n)
    if part.replica:        # more ranks than factors: this rank's factor is another rank's replica
        dev.set_replica()
    # exp-sum rank at k = K (Laplace: kappa independent of n and d)
    sym = inst == "SymInstance"
    if sym and cls == "Laplace":
        spec = tkamd.SpectralData(tkamd.KroneckerMatrix(inst, [csc] * d, cls), K)
        for _ in range(K - 1):
            spec.update(d)
        apx = tkamd.ApproximationData(1e-9, True)
        apx.update(spec)
        t_rank = len(apx.omega)
    else:
        t_rank = 17 if sym else 3
    rng = np.random.default_rng(7)
    # this rank's slice of the t exp-sum terms (all of them unless replicas split the terms)
    tc0, tc1 = part.terms(t_rank)
    Ys = [rng.standard_normal((K, t_rank))[:, tc0:tc1] for _ in range(part.nf)]
    t_loc = tc1 - tc0
    sweeps = dev.arnoldi_sweeps if method in ("TensorArnoldi", "TensorLanczos") else 0
    if world > 1:
        preflight(ctx, world, rank, {"d": d, "n_s": n, "K": K, "method": mcode, "world": world,
                                     "t": t_rank, "config": sorted(CONFIGS).index(args.config),
                                     "steps": args.steps, "warmup": args.warmup})

    host_issue = [0.0, 0]
    # orthogonality_data of factor 1 (src/tensor_krylov_method.jl:103): a Gram row per step,
    # or (deferred) one MFMA SYRK of its basis per solve, timed inside the step here
    gram_owner = dev.gram_deferred and part.first == 0 and part.nf > 0 and not part.replica

    def sweep():
        dev.init(False)
        h0 = time.perf_counter()
        dev.sweep(0, K)                 # enqueues K steps; returns before they run
        host_issue[0] += time.perf_counter() - h0
        host_issue[1] += 1
        dev.basis_mul(K, Ys, want=False)   # finalizes the pending column V[:, K] first (fused for Arnoldi)
        if gram_owner:
            # orthogonality_data for k = 2..K from one Gram of V[:, :K] (after the V*Y: run
            # beside it, the two kernels took longer together than one after the other)
            dev.gram(0, K, want=False)

    def barrier():
        ctx.sync()
        if world > 1:
            ctx.allreduce_host(np.zeros(1))     # RCCL all-reduce == barrier

    if args.pmc_mode:
        sweep()
        dev.basis_mul(K, Ys, want=False)   # the standalone MFMA V*Y (no column pending now)
        barrier()
        dev.close()
        A.close()
        ctx.close()
        return

    for _ in range(args.warmup):
        sweep()
    barrier()
    ctx.timing(1)                    # per-step HIP events on the library's stream
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sweep()
    barrier()
    elapsed = time.perf_counter() - t0
    host_us_per_step = 1e6 * host_issue[0] / max(host_issue[1], 1) / K
    sweep_ms, sweep_cnt = ctx.timing_read(L.T_SWEEP)    # K step groups per sweep
    step_ms, step_cnt = sweep_ms, sweep_cnt * K
    vy_ms, vy_cnt = ctx.timing_read(L.T_VY)
    gram_ms, gram_cnt = ctx.timing_read(L.T_GRAM)
    if world > 1:                               # max over ranks (one-hot sum)
        v = np.zeros(world)
        v[rank] = elapsed
        elapsed = float(ctx.allreduce_host(v).max())

    # per-kernel breakdown (separate, untimed pass with per-kernel events)
    ctx.timing(2)
    sweep()
    ctx.sync()
    kern = {}
    p1name = "sweep_spmv2_dcgs2" if sweeps == 1 else "pass1_spmv_cgs"
    for name, cls_id in ((p1name, L.T_PASS1), ("pass2_cgs", L.T_PASS2), ("finalize", L.T_FIN),
                         ("reduce_post", L.T_RED), ("basis_mul", L.T_VY), ("exchange", L.T_XCH)):
        ms, cnt = ctx.timing_read(cls_id)
        kern[name] = {"avg_us": round(1e3 * ms / cnt, 3) if cnt else None, "launches": cnt}
    ctx.timing(0)
    # the standalone V*Y on MFMA (v_mfma_f64_16x16x4f64; what basis_mul runs when no column
    # is pending, or without the fused flush), on the same basis: untimed above
    ctx.timing(1)
    for _ in range(3):
        dev.basis_mul(K, Ys, want=False)
    ctx.sync()
    mf_ms, mf_cnt = ctx.timing_read(L.T_VY)
    ctx.timing(0)

    # end-to-end: the whole tensorkrylov! loop (device steps + the host's compressed solve,
    # residual and spectral update per iteration, pipelined), same workload, untimed above
    e2e = None
    if not args.no_end_to_end:
        allb = []
        for s_ in range(d):
            b_ = np.random.default_rng(1000 + s_).random(n)
            allb.append(b_ / np.linalg.norm(b_))
        kron = tkamd.KroneckerMatrix(inst, [csc] * d, cls)
        overlay = ref_relres = eval_overlay = eval_table_full_us = None
        if args.emulate_ranks > 1 and world == 1:
            # the other ranks' factors: their records from a full run on this GPU (the same
            # records an N-rank job all-reduces), and the N = 1 trajectory to compare with
            full = tkamd.DeviceDecomposition(ctx, mcode, d, 0, [A] * d, allb, K)
            full.init(False)
            full.sweep(0, K)
            overlay = np.zeros((K + 2, d, full.m))
            overlay[:K + 1] = full.records(0, K + 1)
            full.close()
            conv1 = tkamd.ConvergenceData(K)
            tkamd.tensorkrylov(conv1, kron, allb, 1e-9, K, method, ctx=ctx)
            ref_relres = conv1.relative_residual_norm.copy()
            # this rank evaluates only the iterations it owns (k % N == rank, the evaluation
            # split of an N-rank job); the others' results come from the full run's table
            if os.environ.get("TKHIP_EVAL_SPLIT", "1") != "0":
                eval_overlay = getattr(conv1, "native_results", None)
            if eval_overlay is not None and os.environ.get("TKHIP_EVAL_CALIBRATE", "1") != "0":
                # the full run evaluated every iteration, P at a time, so its times carry the
                # contention of an N = 1 host; an owner under the split evaluates 1 of N.  Each
                # owner's times are measured in its own emulated solve (its factors on this GPU,
                # its iterations evaluated here, the others released from the full run's table)
                # and the timed runs release iteration k after its owner's calibrated time
                Ne = args.emulate_ranks
                cal = eval_overlay.copy()
                for r_ in range(Ne):
                    cr = tkamd.ConvergenceData(K)
                    tkamd.tensorkrylov(cr, kron, allb, 1e-9, K, method, ctx=ctx, overlay=overlay,
                                       partition=tkamd.Partition(d, Ne, r_, term_split=False),
                                       eval_overlay=eval_overlay)
                    res_ = getattr(cr, "native_results", None)
                    if res_ is None:
                        break
                    for k_ in range(2, K + 1):
                        if k_ % Ne == r_ and res_[k_ - 1, 5] >= 0:
                            cal[k_ - 1, 5] = res_[k_ - 1, 5]
                else:
                    eval_table_full_us = eval_overlay[1:, 5].copy()
                    eval_overlay = cal
        samples = []
        for _ in range(max(1, args.e2e_reps)):
            conv = tkamd.ConvergenceData(K)
            barrier()
            te = time.perf_counter()
            tkamd.tensorkrylov(conv, kron, allb, 1e-9, K, method, ctx=ctx, partition=part, overlay=overlay,
                               eval_overlay=eval_overlay)
            barrier()
            te = time.perf_counter() - te
            loop = conv.timing.get("loop_s", te)
            if world > 1:   # (max over ranks of each solve's times)
                v = np.zeros(2 * world)
                v[rank], v[world + rank] = te, loop
                v = ctx.allreduce_host(v)
                te, loop = float(v[:world].max()), float(v[world:].max())
            samples.append((loop, te, conv))
        # the median solve by loop time (its phases and trajectory are reported)
        samples.sort(key=lambda x: x[0])
        loop, te, conv = samples[len(samples) // 2]
        e2e_rate = max(conv.niterations - 1, 1) / loop
        # like for like: the device rate of the loop's own work -- the K steps of a sweep
        # without the end-of-solve V*Y and Gram (a solve that does not converge runs neither)
        loop_dev = (K * sweep_cnt) / (sweep_ms / 1e3) if sweep_cnt else None
        e2e = {"iterations_s": round(e2e_rate, 2),
               "device_steps_only_iterations_s": round(loop_dev, 2) if loop_dev else None,
               "vs_device_steps_only": round(e2e_rate / loop_dev, 4) if loop_dev else None,
               "eval_split": getattr(conv, "eval_split", None),
               **({"split_table_eval_us": {"mean": round(float(np.nanmean(eval_overlay[1:, 5])), 1),
                                           "max": round(float(np.nanmax(eval_overlay[1:, 5])), 1),
                                           "last": round(float(eval_overlay[K - 1, 5]), 1),
                                           **({"full_run_mean": round(float(np.nanmean(eval_table_full_us)), 1),
                                               "full_run_last": round(float(eval_table_full_us[-1]), 1)}
                                              if eval_table_full_us is not None else {}),
                                           "calibrated": eval_table_full_us is not None,
                                           "note": "per-iteration evaluation times that release the other "
                                                   "ranks' results in the emulation: each owner's own, "
                                                   "measured in its emulated split solve (calibrated), "
                                                   "else the full N = 1 run's"}}
                  if eval_overlay is not None else {}),
               "solves": len(samples),
               "iterations_s_all": [round(max(c_.niterations - 1, 1) / l_, 2) for l_, _, c_ in samples],
               "iterations": int(conv.niterations),
               "setup_plus_teardown_s": round(te - loop, 4),
               **({"relres_bitwise_equal_to_n1": all(bool(np.array_equal(c_.relative_residual_norm, ref_relres))
                                                      for _, _, c_ in samples)}
                  if ref_relres is not None else {}),
               "host_threads": tkamd.solver._native_threads(),
               "phases_s": {k_: round(v_, 6) for k_, v_ in conv.timing.items()},
               "final_relative_residual": float(conv.relative_residual_norm[conv.niterations - 1]),
               "note": "tkamd.tensorkrylov (src/tensor_krylov_method.jl:36-125) iterations k = 2..K: "
                       "device steps enqueued ahead + the native host loop (tk_solver_run: records "
                       "applied in order, compressed solve + residual of several iterations "
                       "concurrently on host threads); setup (A_s upload, step 1) and teardown "
                       "reported apart"}
        del allb

    iters = K * args.steps
    value = iters / elapsed
    # roofline of the Arnoldi step (SpMV + MGS2 + reductions), device time from events
    # A_s's bytes once per batch of factors that share one SpMV pass over it,
    # else once per factor (dev.matrix_reads)
    tb = toeplitz_bytes(csc)
    mreads = dev.matrix_reads
    alg_step = sum(alg_bytes_step(n, nnz, k, method, sweeps, tb, with_matrix=False) * part.nf
                   + matrix_bytes(n, nnz, method, sweeps, tb) * mreads for k in range(1, K + 1))
    if method == "TensorLanczos" and sweeps == 1 and part.first == 0 and not dev.gram_deferred:
        # the Gram row of factor 1's new column (orthogonality_loss, src/tensor_krylov_method.jl
        # :103): its basis row is streamed for it alone
        alg_step += sum(8 * n * (k - 1) for k in range(1, K + 1))
    step_avg_s = (step_ms / 1e3) / max(step_cnt, 1)
    achieved = (alg_step / K) / step_avg_s / 1e9 if step_cnt else None
    # the same steps priced in the reference algorithm's bytes (MGS2 streams V
    # twice per step): what a two-sweep implementation would have to move at this rate
    ref_step = sum(alg_bytes_step(n, nnz, k, method, 2) for k in range(1, K + 1)) * part.nf
    vy_bytes = (8 * n * K + 8 * K * t_loc + 8 * n * t_loc) * part.nf
    vy_flops = 2 * n * K * t_loc * part.nf
    vy_s = (vy_ms / 1e3) / max(vy_cnt, 1)
    mf_s = (mf_ms / 1e3) / max(mf_cnt, 1)
    fused_vy = method == "TensorArnoldi"      # the step's basis_mul finalizes the pending column with it

    out = None
    if rank == 0:
        traffic = None
        # PMC HBM bytes per step of this config and method (tools/pmc_traffic.py; the config's
        # own method: pmc_<config>_n<N>.json, another: pmc_<config>_<method>_n<N>.json)
        tag = args.config if method == CONFIGS[args.config][3] else "%s_%s" % (args.config, method)
        pmc_path = os.path.join(ROOT, "profiles", "pmc_%s_n%d.json" % (tag, world))
        if os.path.exists(pmc_path) and not args.emulate_ranks:
            try:
                traffic = json.load(open(pmc_path)).get("hbm_bytes_per_step")
            except Exception:
                traffic = None
        cpu = None
        if not args.no_cpu_baseline and world == 1 and not args.emulate_ranks:
            cpu = cpu_baseline(csc, n, d, K, args.cpu_seconds)
        out = {
            "metric": "Krylov iterations/sec (d-dim Laplacian tensor Krylov; per factor SpMV + two-projection "
                      "Gram-Schmidt, one sweep over V per step)",
            "value": round(value, 3),
            "unit": "iterations/s",
            "n_gpus": world,
            "world": world,
            # ranks RCCL joined (ncclCommCount; 0 = no communicator, the N = 1 run)
            "rccl_nranks": ctx.comm_count(),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            **({"emulated": "rank %d of %d on one GPU: per-rank time of an N-GPU run, NOT a "
                            "whole-job number" % (args.emulate_rank, args.emulate_ranks)} if args.emulate_ranks else {}),
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (assemble_matrix Laplace; b_s ~ U(0,1) seed 1000+s, normalized)",
            "config": {"workload": "%s: d=%d n_s=%d %s %s K=%d, factors over %d GPU(s); "
                                   "step = 1 sweep of K iterations + V*Y (t=%d)"
                                   % (args.config, d, n, cls, method, K, world, t_rank),
                       "d": d, "n_s": n, "nmax": K, "matrix": cls, "method": method,
                       "parallelism": "factor-partition x%d (RCCL all-reduce of records per iteration%s%s)"
                                      % (world, ", forced on 1 rank" if args.force_comm else "",
                                         "; ranks >= d replicate a factor and split its V*Y terms"
                                         if part.term_split else "")},
            "roofline": {
                "bound": "hbm",
                "kernel": ("one-sweep Arnoldi factor-step (k_arn_d1: v_j, two SpMVs from LDS, CGS projections "
                           "with the reorthogonalization delayed one step; 1 reduce, post), all local factors"
                           if method == "TensorArnoldi" and sweeps == 1 else
                           "Arnoldi factor-step (pass1 SpMV+CGS fused, pass2 CGS, 2 reduce, post), all local factors"
                           if method == "TensorArnoldi" else
                           "%s factor-step (TTR SpMV pass, update pass, reduces, post%s), all local factors"
                           % (method, ", Gram row + host loss check" if method == "TensorLanczosReorth" else "")),
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": alg_step / K,
                "matrix_reads_per_step": mreads,
                "arnoldi_sweeps_over_V": sweeps if method == "TensorArnoldi" else None,
                **({"reference_algorithm_bytes_per_launch": ref_step / K,
                    "reference_algorithm_effective_GBs": round((ref_step / K) / step_avg_s / 1e9, 1)}
                   if method == "TensorArnoldi" and sweeps == 1 and step_cnt else {}),
                "avg_launch_us": round(step_avg_s * 1e6, 2),
                # 2: the local factors step as two groups, each in its own launches on its own
                # stream; avg_launch_us is then the span of a step's two concurrent launch pairs
                # (rocprofv3 lists each group's k_arn_d1 apart, over half the factors' bytes)
                "factor_groups": dev.factor_groups if method == "TensorArnoldi" and sweeps == 1 else 1,
            },
            "host_issue_us_per_iteration": round(host_us_per_step, 2),
            # the one-sweep reduce hand-off this process runs (tk_reduce_handoff): relaxed
            # atomics confirmed by the startup self-check, or the memory-model form
            "reduce_handoff": {0: "relaxed (self-checked against the memory-model form)",
                               1: "memory-model release/acquire",
                               2: "relaxed (forced, TKHIP_RED_MM=0)",
                               3: "memory-model release/acquire (the self-check could not run)"}.get(
                                   L.lib().tk_reduce_handoff(), "not used (no one-sweep step)"),
            # (its one-off cost inside the first tk_decomp_create of the process, outside the timed region)
            "reduce_handoff_check_ms": round(L.lib().tk_reduce_check_ms(), 2),
            "end_to_end": e2e,
            "basis_mul_step": {
                "engine": ("k_fin_vy: flush of the pending column + V*Y from its register row (FP64 FMA), "
                           "one read of V" if fused_vy else "k_basis_mul (MFMA) after the flush"),
                "avg_us": round(vy_s * 1e6, 2),
                "GB_s": round((vy_bytes + 8 * n * part.nf) / vy_s / 1e9, 1) if vy_cnt else None,
                **({"why_fma": "V*Y at t=%d, k=%d is %.1f flop/B, below the fp64 ridge (78.6 TF / 8 TB/s = 9.8): "
                               "HBM-bound either way, and on gfx950 fp64 MFMA and fp64 VALU FMA have the same "
                               "peak (78.6 TF); the fused kernel reads V once for the flush and the product "
                               "(the MFMA kernel, basis_mul_mfma, needs the column flushed first: a second read "
                               "of V).  Both run at 94-96 %% of the measured ceiling of this read/write mix "
                               "(profiles/r02/rwprobe_c2_vy_ceiling.txt, 779 us at C2)"
                               % (t_loc, K, vy_flops / vy_bytes)} if fused_vy else {}),
            },
            "orthogonality_gram": ({"mode": "deferred: one v_mfma_f64_16x16x4f64 SYRK of factor 1's basis "
                                            "per solve (tk_decomp_gram)",
                                    "avg_us": round(1e3 * gram_ms / gram_cnt, 2) if gram_cnt else None,
                                    "GB_s": round(8 * n * K / (1e-3 * gram_ms / gram_cnt) / 1e9, 1) if gram_cnt else None,
                                    "TFLOP_s_useful": round(n * K * (K + 1) / (1e-3 * gram_ms / gram_cnt) / 1e12, 3)
                                    if gram_cnt else None}
                                   if dev.gram_deferred else
                                   {"mode": "a Gram row of factor 1's new column in every step (from the register row)"}),
            "basis_mul_mfma": {
                "avg_us": round(mf_s * 1e6, 2),
                "GB_s": round(vy_bytes / mf_s / 1e9, 1) if mf_cnt else None,
                "TFLOP_s": round(vy_flops / mf_s / 1e12, 3) if mf_cnt else None,
                "mfma_fp64_peak_TF": FP64_MFMA_PEAK_TF,
            },
            "kernels": kern,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    barrier()
    if rank == 0 and uid_path is not None:
        try:
            os.remove(uid_path[0])
        except OSError:
            pass
    dev.close()
    A.close()
    ctx.close()


def toeplitz_bytes(csc):
    """Matrix bytes a one-sweep factor-step must read: 0 when every diagonal of the band is
    constant (the device keeps them as scalars), else the DIA values (8 B per stored
    entry, the band's nonzeros)."""
    colptr, rowval, nzval = csc
    n = len(colptr) - 1
    cols = np.repeat(np.arange(n), np.diff(colptr))
    off = cols - rowval
    for o in np.unique(off):
        v = nzval[off == o]
        if len(v) != n - abs(int(o)) or not np.all(v == v[0]):
            return 8 * len(nzval)
    return 0


def preflight(ctx, world, rank, fields):
    """Before the first sweep: every rank must run the same workload (a rank with other
    sizes would issue all-reduces of other lengths and hang the job).  Each rank writes its
    values into its own row, one RCCL all-reduce (bounded by TKHIP_WAIT_S) gives every rank
    every row, and any difference ends the run on all ranks with the table."""
    names = list(fields)
    rows = np.zeros((world, len(names)))
    rows[rank] = [float(fields[k]) for k in names]
    rows = ctx.allreduce_host(rows.ravel()).reshape(world, len(names))
    bad = [k for i, k in enumerate(names) if not np.all(rows[:, i] == rows[0, i])]
    if bad:
        sys.exit("bench preflight: ranks disagree on %s: %s" % (
            ", ".join(bad), {k: rows[:, names.index(k)].tolist() for k in bad}))


def exchange_uid(tkamd, rank, timeout=120.0):
    """Hand the RCCL unique id from rank 0 to the other ranks of this node through a
    file keyed by the launcher's pid (all ranks of one torch.distributed.run share it)."""
    key = "%d_%s" % (os.getppid(), os.environ.get("MASTER_PORT", "0"))
    path = os.path.join("/tmp", "tkhip_uid_%s.bin" % key)
    if rank == 0:
        uid = tkamd.unique_id()
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return path, uid
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > timeout:
            raise RuntimeError("rank %d: no RCCL unique id from rank 0 after %.0f s" % (rank, timeout))
        time.sleep(0.01)
    with open(path, "rb") as f:
        uid = f.read()
    assert len(uid) == 128
    return path, uid


def cpu_baseline(csc, n, d, K, seconds):
    """The C restatement's K-step Arnoldi (MGS2) sweeps on a bounded sample of the
    workload's factors: on one host core (oracle/tk_ref.py baseline(): the reference's
    effective concurrency -- its factor loop runs one task at a time) and with the rows
    split over all the cores OpenMP is given (baseline_all_cores(): the reference with a
    threaded BLAS).  `value`/`cores` are the 1-core figure; `all_cores` the other; the
    host's CPU model and core counts are reported beside them."""
    try:
        sys.path.insert(0, ROOT)
        from oracle import tk_ref
        one = tk_ref.baseline(csc, n, d, K, seconds)
        one["all_cores"] = tk_ref.baseline_all_cores(csc, n, d, K, seconds)
        one.update(tk_ref.cpu_info())
        return one
    except Exception as e:   # noqa: BLE001
        return {"value": None, "unit": "iterations/s", "cores": None, "kind": "port",
                "sample": "unavailable: %s" % e}


if __name__ == "__main__":
    try:
        rc = main()
        if rc:
            sys.exit(rc)
    except Exception as e:   # noqa: BLE001
        # a libtkhip error (e.g. TK_ERR_RCCL: a peer never joined an all-reduce within
        # TKHIP_WAIT_S) ends THIS rank with its diagnosis; exit without running destructors,
        # which could wait on the same peer
        if type(e).__name__ != "TKError":
            raise
        sys.stderr.write("bench.py rank %s: %s\n" % (os.environ.get("RANK", "0"), e))
        sys.stderr.flush()
        os._exit(3)
