"""tensorkrylov! and solve_tensorized_system on the MI355X path.

Host restatement of src/tensor_krylov_method.jl:36-125 and src/system.jl:65-83 whose
n-length work (the per-factor Krylov steps, update_rhs!, the orthogonality Gram rows
and basis_tensor_mul!) runs in libtkhip on the GPU.  With a Partition over several
ranks every rank runs this same loop; the device all-reduces each step's per-factor
records so the k-sized compressed solve below is evaluated redundantly and
identically on every rank.
"""
import time

import numpy as np

from .compressed import (ApproximationData, CompressedNormBreakdown, IterationTables, NativeSolver,
                         SpectralData, residualnorm, solve_compressed_system)
from .decompositions import METHODS
from .structures import ConvergenceData, KruskalTensor, kronprodnorm


def _native_threads():
    import os
    v = os.environ.get("TKHIP_SOLVER_THREADS")
    if v:
        return max(1, int(v))
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    return max(1, min(8, ncpu // 2))


def tensorkrylov(conv, A, b, tol, nmax, method, ctx=None, partition=None, verbose=False,
                 backend=None, keep_decomposition=False, pipelined=True, depth=2, native=True,
                 threads=None, overlay=None, eval_overlay=None):
    """tensorkrylov!(convergence_data, A, b, tol, nmax, orthonormalization_type).
    Returns the approximate solution as a KruskalTensor of the LOCAL factors
    (x_s = V_s y_s; with a term-splitting Partition only this rank's slice x.terms of the
    t exponential-sum terms) on convergence, else None.

    pipelined: steps k+1 .. k+depth are enqueued on the device before the host evaluates
    iteration k (compressed solve, residual), so device and host work overlap and the
    device never waits for the host's read of a record.  Steps after k leave V[:, 1:k],
    H[1:k, 1:k] and b~[1:k] untouched, so every iterate, residual and the returned solution
    are those of the sequential loop; on convergence at k the extra steps' results are
    simply never read.

    native: the per-iteration host work (record bookkeeping, compressed solve, residual,
    orthogonality) runs in libtkhip's tk_solver; on a device decomposition the whole loop
    does (tk_solver_run: steps enqueued ahead, iterations evaluated on `threads` host
    threads, consumed in order -- the same iterates).  native=False keeps the Python loop
    below (the mirror of the reference's driver, used to cross-check the native one).
    overlay (diagnostic, native only): a full run's records [nmax+2][d][m]; the records of
    factors this rank does not own are taken from it (bench.py --emulate-ranks).
    eval_overlay (diagnostic, with overlay): a full run's per-iteration results
    (conv.native_results) -- this rank then evaluates only its share of the iterations
    (k % N == rank) and takes the others' from the table, each released no earlier than the
    owner would have had it (tk_solver_share_emulated).

    With several ranks (partition) on one node the native solver splits the evaluations over
    the ranks (tk_solver_share, a shared-memory mailbox; TKHIP_EVAL_SPLIT=0 turns it off):
    every rank still applies every record, so each iterate is bitwise what it would have
    computed itself."""
    if isinstance(method, str):
        method = METHODS[method]
    d = len(A)
    b_norm = kronprodnorm(b)                                        # :48
    td = method(A, nmax, ctx=ctx, partition=partition, backend=backend)   # :51
    symmetric = A.symmetric
    x = None
    t_start = time.perf_counter()
    conv.timing = {}
    try:
        td.orthonormalize_first(b)                                  # :53 (+ b~ init, :55)
        if native:
            # setup: spectral bounds + exp-sum data of every k (functions of A and tol only)
            # and the native driver holding the records of init and step 1
            t_tab = time.perf_counter()
            tables = IterationTables(A, nmax, tol, d)
            conv.timing["tables_s"] = time.perf_counter() - t_tab
            sv = NativeSolver(td.method, d, nmax, symmetric, b_norm, tables)
            if pipelined and hasattr(td.dev, "h"):
                sv.prepare(threads or _native_threads())   # (worker threads: setup, not loop)
            try:
                if overlay is not None:
                    sv.overlay(td.part.first, td.part.nf, overlay)
                    if eval_overlay is not None and td.part.nranks > 1:
                        sv.share_emulated(td.part.nranks, td.part.rank, eval_overlay)
                elif _split_wanted(td.part):
                    key = _share_key(td)
                    try:
                        sv.share(key, td.part.nranks, td.part.rank)
                    except Exception as e:      # noqa: BLE001  (TKError: no mailbox on this rank)
                        # continue unsplit: tk_solver_run's agreement at the start of the run
                        # (max over the ranks of "no mailbox") turns the split off on every rank
                        import warnings
                        warnings.warn("evaluation split unavailable on rank %d (%s): every rank "
                                      "evaluates every iteration" % (td.part.rank, e))
                        sv.share(key, 1, 0)
                conv.eval_split = sv.split
                for j, rec in td.first_records:
                    sv.apply(j, rec)
                t_loop = time.perf_counter()
                conv.timing["setup_s"] = t_loop - t_start
                return _native_loop(conv, td, sv, tables, tol, nmax, verbose, pipelined, depth, threads, t_loop)
            finally:
                sv.close()
        t_loop = time.perf_counter()
        conv.timing["setup_s"] = t_loop - t_start                   # upload A_s, b_s; step 1
        spectral = SpectralData(A, nmax)                            # :57
        approx = ApproximationData(tol, symmetric)                  # :58
        depth = max(1, int(depth))
        if pipelined:
            for kk in range(2, min(nmax, 1 + depth) + 1):
                td.issue(kk)
        for k in range(2, nmax + 1):                                # :63
            if pipelined:
                td.collect(k)                                       # :66
                if k + depth <= nmax:
                    td.issue(k + depth)                             # overlaps the host work below
            else:
                td.orthonormalize(k)                                # :66
            Hm = td.minors(k)                                       # :68
            bm = [td.btilde[s, :k].copy() for s in range(d)]        # update_rhs! :71
            spectral.update(d)                                      # :72
            approx.update(spectral)                                 # :73
            lmin = spectral.lmin[k - 1]
            lam, Ys = solve_compressed_system(Hm[0], bm, approx, lmin, symmetric)   # :76
            sub = td.subdiagonal(k)                                 # :79
            try:
                r_comp, r_norm = residualnorm(Hm, lam, Ys, k, sub, bm, b_norm)      # :83
            except CompressedNormBreakdown:                         # :85-96
                if verbose:
                    print("Early termination at k = %d due to compressed norm breakdown" % k)
                # orthogonality_data[2..k-1] was filled on the iterations before the breakdown
                # (:103, then :90-94)
                _fill_deferred_orthogonality(conv, td, k - 1)
                conv.niterations = k - 1
                conv.resize(k - 1)
                conv.timing["loop_s"] = time.perf_counter() - t_loop
                return None
            rel = r_norm / b_norm                                   # :99
            conv.relative_residual_norm[k - 1] = rel
            conv.projected_residual_norm[k - 1] = r_comp
            if not _gram_deferred(td):
                conv.orthogonality_data[k - 1] = td.orthogonality_loss(0, k)      # :103
            if rel < tol:                                           # :108-118
                # basis_tensor_mul! on the device; X sized by ncomponents(y)
                # (the reference sizes it by approxdata.rank, SURVEY.md 3.2 deviation)
                x = _solution(td, k, lam, Ys)
                _fill_deferred_orthogonality(conv, td, k)
                conv.timing["loop_s"] = time.perf_counter() - t_loop
                if verbose:
                    print("Convergence")
                return x
        _fill_deferred_orthogonality(conv, td, nmax)
        conv.timing["loop_s"] = time.perf_counter() - t_loop
        if verbose:
            print("No convergence")
        return None
    finally:
        if keep_decomposition:
            conv.decomposition = td
        else:
            td.close()


def _split_wanted(part):
    """Evaluation split over the ranks (tk_solver_share): several ranks, not turned off by
    TKHIP_EVAL_SPLIT=0, and every rank positively known to be on this node -- the mailbox is
    node-local shared memory.  Known means LOCAL_WORLD_SIZE == WORLD_SIZE == the partition's
    rank count (torch.distributed.run sets both); any other launcher, or a multi-node job,
    runs unsplit (ranks on other nodes would never find the mailbox).  Every rank
    decides the same way; if a rank still ends up without a mailbox, it continues unsplit and
    tk_solver_run's agreement turns the split off everywhere."""
    import os
    if part.nranks <= 1 or os.environ.get("TKHIP_EVAL_SPLIT", "1") == "0":
        return False
    lw, w = os.environ.get("LOCAL_WORLD_SIZE"), os.environ.get("WORLD_SIZE")
    return lw is not None and w is not None and lw == w and int(w) == part.nranks


def _share_key(td):
    """A job-unique mailbox key every rank agrees on: rank 0 draws it, one host all-reduce
    (setup, not the loop) hands it to the others."""
    import os
    part = td.part
    v = np.zeros(2)
    if part.rank == 0:
        v[0] = float(int.from_bytes(os.urandom(6), "little"))
        v[1] = float(os.getpid())
    v = (td.ctx if td.ctx is not None else td.dev).allreduce_host(v)
    return "%x_%x_%d" % (int(v[0]), int(v[1]), part.nranks)


def _gram_deferred(td):
    return bool(getattr(td.dev, "gram_deferred", False))


def _fill_deferred_orthogonality(conv, td, k_last, native=None):
    """orthogonality_data[k] = orthogonality_loss(V_1, k) (src/tensor_krylov_method.jl:103,
    src/orthogonal_bases.jl:250-257) for k = 2..k_last, from ONE Gram matrix of factor 1's
    basis (tk_decomp_gram: a SYRK on the matrix cores) when the handle does not carry a Gram
    row per step (tk_decomp_gram_deferred).  The values are those the reference computes at
    iteration k: columns 1..k are final once step k is done.  With several ranks the rank
    owning factor 1 computes them and one all-reduce (every rank calls it here) shares them.
    native: orthogonality_data as tk_solver_run left it -- its losses from the Gram launched
    behind the last step, read during the last evaluations (NaN where it had none)."""
    if not _gram_deferred(td) or k_last < 2:
        return
    from .compressed import orthogonality_losses_from_gram
    t0 = time.perf_counter()
    part = td.part
    orth = np.zeros(k_last)
    tm = conv.timing
    if part.nranks > 1:
        # a pending column is written by a flush, whose record all-reduces every rank must
        # join: all ranks flush here, before the one rank's Gram (tk_decomp_gram refuses to
        # start collectives on a multi-rank handle) -- when the Gram reads it.  After step
        # last_j, columns < last_j are in V on every path and column last_j is too unless it
        # waits in the one-sweep column buffer (even last_j); the decision depends on the step
        # sequence alone, which every rank shares, so all ranks take the same branch
        last_j = td.dev.next_step - 1
        if k_last - 1 >= last_j + (0 if last_j % 2 == 0 else 1):
            td.dev.flush(False)
        tm["orth_flush_s"] = time.perf_counter() - t0
    if part.first == 0 and part.nf > 0 and not part.replica:
        t1 = time.perf_counter()
        if native is not None and np.all(np.isfinite(native[1:k_last])):
            orth[1:] = native[1:k_last]
        else:
            G = td.dev.gram(0, k_last)
            orth[:] = orthogonality_losses_from_gram(G)
        tm["orth_gram_only_s"] = time.perf_counter() - t1
    if part.nranks > 1:
        # (the context's RCCL all-reduce; a backend without a context brings its own)
        t1 = time.perf_counter()
        orth = (td.ctx if td.ctx is not None else td.dev).allreduce_host(orth)
        tm["orth_allreduce_s"] = time.perf_counter() - t1
    conv.orthogonality_data[1:k_last] = orth[1:k_last]
    tm["orth_gram_s"] = time.perf_counter() - t0


def _solution(td, k, lam, Ys):
    """basis_tensor_mul! (src/utils.jl:478-488) on the device for this rank's factors and its
    slice [c0, c1) of the exponential-sum terms (all t unless the partition splits terms
    between replicas): x.factors / x.terms say which part of the Kruskal tensor this is."""
    loc = list(td.part.local())
    c0, c1 = td.part.terms(len(lam))
    X = td.dev.basis_mul(k, [np.asarray(Ys[s])[:, c0:c1] for s in loc])
    x = KruskalTensor(lam[c0:c1].copy(), X)
    x.factors = loc
    x.terms = (c0, c1)
    return x


def _native_loop(conv, td, sv, tables, tol, nmax, verbose, pipelined, depth, threads, t_loop):
    """tensorkrylov!'s loop (src/tensor_krylov_method.jl:57-125) through tk_solver; loop_s
    covers the iterations only (the host mirror is copied back afterwards)."""
    device = hasattr(td.dev, "h") and hasattr(td.dev, "records")
    if device and pipelined:
        import os
        nthr = threads or _native_threads()
        # steps in flight ahead of the iteration being dispatched (TKHIP_SOLVER_DEPTH overrides)
        depth = int(os.environ.get("TKHIP_SOLVER_DEPTH", depth))
        t_run = time.perf_counter()
        outcome, k_end, rel, proj, orth = sv.run(td.dev, tol, 2, max(depth, nthr + 1), nthr)
        conv.timing["native_run_s"] = time.perf_counter() - t_run
        conv.relative_residual_norm[1:k_end] = rel[1:k_end]
        conv.projected_residual_norm[1:k_end] = proj[1:k_end]
        conv.orthogonality_data[1:k_end] = orth[1:k_end]
    else:
        outcome, k_end = 0, nmax
        # (split over the ranks: the owner of k evaluates it, the others read its result)
        evaluate = sv.evaluate_shared if getattr(sv, "split", None) else sv.evaluate
        for k in range(2, nmax + 1):
            if tables.rank[k - 1] < 1:
                k_end = k - 1
                break
            td.orthonormalize(k)                                    # :66
            sv.apply(k - 1, td._last_rec)
            try:
                r_comp, _, rel_k, orth_k = evaluate(k)              # :68-103
            except CompressedNormBreakdown:
                outcome, k_end = 2, k - 1
                break
            conv.relative_residual_norm[k - 1] = rel_k
            conv.projected_residual_norm[k - 1] = r_comp
            conv.orthogonality_data[k - 1] = orth_k
            if rel_k < tol:
                outcome, k_end = 1, k
                break
    x = None
    if outcome == 1:                                                # :108-118
        if not (device and pipelined) and not sv.owns(k_end):
            sv.evaluate(k_end)      # another rank evaluated it: this rank's y, bitwise the same
        lam, Ys = sv.solution(k_end)
        x = _solution(td, k_end, lam, Ys)
    _fill_deferred_orthogonality(conv, td, k_end, conv.orthogonality_data if device and pipelined else None)
    conv.timing["loop_s"] = time.perf_counter() - t_loop
    if device and pipelined:
        conv.native_results = sv.results()   # (bench.py --emulate-ranks: the eval_overlay table)
    # the host mirror of H, b~ and factor 1's Gram rows (principal_minors readers)
    H, bt, G = sv.state()
    td.H[...] = H
    td.btilde[...] = bt
    if 0 in td.gram:
        td.gram[0][...] = G
    if outcome == 2:                                                # :85-96
        if verbose:
            print("Early termination at k = %d due to compressed norm breakdown" % (k_end + 1))
        conv.niterations = k_end
        conv.resize(k_end)
        return None
    if outcome == 1:
        if verbose:
            print("Convergence")
        return x
    if k_end < nmax and tables.error is not None:
        raise tables.error
    if verbose:
        print("No convergence")
    return None


def solve_tensorized_system(system, nmax, method, tol=1e-9, **kw):
    """src/system.jl:65-83: returns ConvergenceData (the solution is discarded, as in
    the reference)."""
    conv = ConvergenceData(nmax)
    tensorkrylov(conv, system.A, system.b, tol, nmax, method, **kw)
    return conv
