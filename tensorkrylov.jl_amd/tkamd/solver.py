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

from .compressed import (ApproximationData, CompressedNormBreakdown, SpectralData,
                         residualnorm, solve_compressed_system)
from .decompositions import METHODS
from .structures import ConvergenceData, KruskalTensor, kronprodnorm


def tensorkrylov(conv, A, b, tol, nmax, method, ctx=None, partition=None, verbose=False,
                 backend=None, keep_decomposition=False, pipelined=True, depth=2):
    """tensorkrylov!(convergence_data, A, b, tol, nmax, orthonormalization_type).
    Returns the approximate solution as a KruskalTensor of the LOCAL factors
    (x_s = V_s y_s) on convergence, else None.

    pipelined: steps k+1 .. k+depth are enqueued on the device before the host evaluates
    iteration k (compressed solve, residual), so device and host work overlap and the
    device never waits for the host's read of a record.  Steps after k leave V[:, 1:k],
    H[1:k, 1:k] and b~[1:k] untouched, so every iterate, residual and the returned solution
    are those of the sequential loop; on convergence at k the extra steps' results are
    simply never read."""
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
                conv.niterations = k - 1
                conv.resize(k - 1)
                conv.timing["loop_s"] = time.perf_counter() - t_loop
                return None
            rel = r_norm / b_norm                                   # :99
            conv.relative_residual_norm[k - 1] = rel
            conv.projected_residual_norm[k - 1] = r_comp
            conv.orthogonality_data[k - 1] = td.orthogonality_loss(0, k)          # :103
            if rel < tol:                                           # :108-118
                # basis_tensor_mul! on the device; X sized by ncomponents(y)
                # (the reference sizes it by approxdata.rank, SURVEY.md 3.2 deviation)
                loc = list(td.part.local())
                X = td.dev.basis_mul(k, [Ys[s] for s in loc])
                x = KruskalTensor(lam.copy(), X)
                x.factors = loc
                conv.timing["loop_s"] = time.perf_counter() - t_loop
                if verbose:
                    print("Convergence")
                return x
        conv.timing["loop_s"] = time.perf_counter() - t_loop
        if verbose:
            print("No convergence")
        return None
    finally:
        if keep_decomposition:
            conv.decomposition = td
        else:
            td.close()


def solve_tensorized_system(system, nmax, method, tol=1e-9, **kw):
    """src/system.jl:65-83: returns ConvergenceData (the solution is discarded, as in
    the reference)."""
    conv = ConvergenceData(nmax)
    tensorkrylov(conv, system.A, system.b, tol, nmax, method, **kw)
    return conv
