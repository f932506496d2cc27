/*
 * tk.h -- C ABI of libtkhip.so, the MI355X (gfx950) implementation of the inner Krylov
 * iteration of thbake/TensorKrylov.jl (tensorkrylov!, src/tensor_krylov_method.jl:36-125).
 *
 * The library owns every device buffer; callers pass plain host pointers and sizes.
 * No call retains a host pointer after it returns.  Every entry point returns a
 * tk_status (0 = TK_OK); on failure tk_last_error() (thread-local) says why.  Nothing
 * throws or aborts across this boundary.  A tk_ctx is externally synchronised (one
 * host thread at a time), exactly like the reference's single-threaded Julia driver.
 * Handles may be destroyed in any order (garbage-collector finalizers): a matrix keeps
 * its context alive and a decomposition keeps its context and matrices alive until it
 * is destroyed itself.
 *
 * Conventions
 *   - fp64 throughout (the reference is Float64 everywhere).
 *   - Column index j of a Krylov basis is 0-based: reference step k (1-based,
 *     orthonormalize!(decomp, k, ...)) is ABI step j = k - 1; it consumes V[:, j] and
 *     produces H[0..j+1, j] and V[:, j+1].
 *   - Sparse inputs are Julia's SparseMatrixCSC{Float64,Int64} fields; one_based = 1
 *     accepts them unmodified (Julia's 1-based colptr/rowval).
 *   - One process per GPU: a tk_ctx binds one HIP device and one stream.  When the d
 *     factors are partitioned over ranks, each rank creates its decomposition with its
 *     own contiguous block of factors and the per-step records are summed over ranks
 *     with one RCCL all-reduce (tk_comm_init).
 *
 * Reference interfaces each entry point replaces are cited per declaration
 * (paths relative to the reference repository root).
 */
#ifndef TK_H_
#define TK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int tk_status;
enum {
    TK_OK = 0,
    TK_ERR_ARG = 1,      /* invalid argument / shape                          */
    TK_ERR_HIP = 2,      /* HIP runtime error (message carries hipGetErrorString) */
    TK_ERR_ALLOC = 3,    /* device or host allocation failed                  */
    TK_ERR_STATE = 4,    /* call out of sequence (e.g. step j != next step)   */
    TK_ERR_RCCL = 5,     /* RCCL error                                         */
    TK_ERR_NODEV = 6,    /* no usable gfx950 device                            */
    TK_BREAKDOWN = 7,    /* compressed norm breakdown (src/utils.jl:7-14, :395)  */
    TK_ERR_INTERNAL = 8  /* unexpected host-side exception, caught at the boundary */
};

/* Orthonormalization types: src/decompositions.jl:120-176 (TensorArnoldi,
 * TensorLanczos, TensorLanczosReorth) dispatched by get_orthogonalization,
 * src/orthogonal_bases.jl:11-13. */
enum {
    TK_ARNOLDI = 0,          /* MGS, src/orthogonal_bases.jl:15-37   */
    TK_LANCZOS = 1,          /* TTR, src/orthogonal_bases.jl:39-67   */
    TK_LANCZOS_REORTH = 2    /* TTR + loss check + MGS redo, :98-139 */
};

typedef struct tk_ctx tk_ctx;
typedef struct tk_mat tk_mat;
typedef struct tk_decomp tk_decomp;

/* ---------------------------------------------------------------- library / context */
const char* tk_last_error(void);
int tk_version(void);                         /* 100 * major + minor */
/* Bind `device` (HIP ordinal) and create the context's stream. */
tk_status tk_ctx_create(int device, tk_ctx** out);
tk_status tk_ctx_destroy(tk_ctx* ctx);
tk_status tk_ctx_sync(tk_ctx* ctx);

/* ---------------------------------------------------------------- multi-GPU (RCCL) */
/* 128-byte RCCL unique id; rank 0 creates it and the host broadcasts it. */
tk_status tk_comm_unique_id(char id_out[128]);
/* Join an nranks-wide communicator on ctx's device.  Replaces nothing in the
 * reference (which is single process); it carries the one per-iteration exchange of
 * the compressed quantities. */
tk_status tk_comm_init(tk_ctx* ctx, const char id[128], int nranks, int rank);
/* In-place sum all-reduce of `count` doubles of host memory through the device (test
 * and control-plane use; the hot path's exchange is internal to tk_decomp_step). */
tk_status tk_comm_allreduce_host(tk_ctx* ctx, double* buf, size_t count);
/* Ranks of ctx's communicator as RCCL reports them (ncclCommCount); 0 without one.
 * bench.py reports it beside the launcher's WORLD_SIZE. */
tk_status tk_comm_count(tk_ctx* ctx, int* nranks_out);

/* ---------------------------------------------------------------- coefficient matrices */
/* A_s as SparseMatrixCSC (src/tensor_struct.jl:48-68 assemble_matrix, stored in
 * KroneckerMatrix, :168-231).  Converted to device CSR (row-major, ascending column
 * within a row, int32 indices) so that each row sum y[i] = sum_p val[p]*x[col[p]]
 * adds terms in the order of Julia's CSC scatter mul! (no FMA): results equal the
 * reference SpMV bit for bit. */
tk_status tk_matrix_from_csc(tk_ctx* ctx, int64_t n, const int64_t* colptr,
                             const int64_t* rowval, const double* nzval,
                             int one_based, tk_mat** out);
tk_status tk_matrix_from_csr(tk_ctx* ctx, int64_t n, const int64_t* rowptr,
                             const int64_t* colind, const double* val,
                             int one_based, tk_mat** out);
tk_status tk_matrix_destroy(tk_mat* A);
/* Storage chosen on the device: k > 0 = DIA with k diagonals (banded matrices with
 * few, mostly full diagonals; no index loads), -2 = SELL-256 (sliced ELL, one slice
 * per 256-row tile: coalesced index/value loads), 0 = CSR.  All keep the per-row
 * ascending-column summation order.  TKHIP_FORCE_CSR=1 forces CSR. */
int tk_matrix_format(tk_mat* A);
/* y = A x on the device (host in/out buffers; test hook for mul!, used at
 * src/orthogonal_bases.jl:20,45,103). */
tk_status tk_matvec(tk_mat* A, const double* x, double* y);

/* ---------------------------------------------------------------- tensor decomposition */
/* Create the state of this rank's factors s = first_factor .. first_factor+nf-1 of a
 * d_total-factor decomposition (TensorArnoldi(A) / TensorLanczos(A) /
 * TensorLanczosReorth(A), src/decompositions.jl:127-174; storage capped at kmax+1
 * basis columns instead of n+1).  mats[i], b[i] (length n, host) are factor
 * first_factor+i's A_s and b_s.  All factors share n (src/tensor_krylov_method.jl:46).
 * kmax = nmax; steps j = 0 .. kmax-1 are allowed.
 * track_all_gram: 1 keeps the Gram row of every factor in the step records (always on for
 * TK_LANCZOS_REORTH); 2 keeps global factor 0's (the driver's orthogonality_data,
 * src/tensor_krylov_method.jl:103) for a caller that reads it after every step, like the
 * reference's loop; 0 lets the library choose between factor 0's rows and a deferred Gram
 * (tk_decomp_gram_deferred). */
tk_status tk_decomp_create(tk_ctx* ctx, int method, int d_total, int first_factor, int nf,
                           tk_mat* const* mats, const double* const* b, int64_t n, int kmax,
                           int track_all_gram, tk_decomp** out);
tk_status tk_decomp_destroy(tk_decomp* dc);

/* Sweeps over V per TK_ARNOLDI step: 1 = CGS2 with the reorthogonalization delayed by one
 * step (every local A_s banded, DIA with bandwidths <= 4), 2 = CGS2
 * (other storage, or TKHIP_ARNOLDI=cgs2 in the environment at create).  TK_LANCZOS: 1 for
 * the one-sweep TTR (banded A_s; TKHIP_LANCZOS=ttr keeps the three-pass kernels: 0);
 * TK_LANCZOS_REORTH: 0. */
int tk_decomp_arnoldi_sweeps(tk_decomp* dc);

/* 1 when the records exchange of this handle is triggered by a signal word the step's last
 * kernel increments (hipStreamWaitValue64 on the exchange stream), 0 when it uses an event
 * per step or there is no exchange (single rank; TK_LANCZOS_REORTH; TKHIP_XCH_EVENTS=1). */
int tk_decomp_exchange_signalled(tk_decomp* dc);

/* The next step j that tk_decomp_step accepts (steps 0 .. j-1 are enqueued; a driver that
 * ran ahead, like tk_solver_run, may have enqueued more steps than its caller has read). */
int tk_decomp_next_step(tk_decomp* dc);

/* How many times one step of all local factors reads the bytes of A_s: 1 when the factors
 * share one gather-format A_s and its entries are read once for all of them (CGS2 with the
 * interleaved SpMV), else the local factor count (benchmark byte
 * models, SURVEY.md 8(d): "count the CSR bytes once per batch"). */
int tk_decomp_matrix_reads(tk_decomp* dc);

/* Element-wise max of vals[0..count) over the ranks sharing dc's records exchange (no-op on
 * one rank; count <= 64).  Collective: every rank calls it at the same point of its call
 * sequence.  tk_solver_run agrees its issue depth and worker count with it, so that every
 * rank issues the same sequence of steps, record reads and therefore all-reduces. */
tk_status tk_decomp_agree(tk_decomp* dc, int* vals, int count);

/* The one-sweep steps' reduce hand-off: 0 = relaxed agent-scope atomics
 * (measured correct on gfx950, and confirmed by a self-check against the memory-model form at
 * the process's first tk_decomp_create), 1 = the HIP memory model's release/acquire form (kept
 * when the self-check finds any difference; TKHIP_RED_MM=1 forces it), 2 = relaxed, forced by
 * TKHIP_RED_MM=0 without the check, 3 = the memory-model form because the self-check could not
 * run (its context, matrix, decomposition or steps failed), -1 = not settled yet (no
 * decomposition created). */
int tk_reduce_handoff(void);
/* Wall time (ms) of that self-check -- a one-off cost of the process's first tk_decomp_create
 * (0 when it did not run). */
double tk_reduce_check_ms(void);

/* Multi-rank waits (the records exchange, tk_comm_allreduce_host, tk_ctx_sync, destroy) are
 * bounded by TKHIP_WAIT_S seconds (default 120): on expiry the call returns TK_ERR_RCCL naming
 * the record slot / step it waited for and RCCL's asynchronous error state, and the context
 * is marked unusable (later collectives fail at once; its device buffers are left to process
 * exit, since a collective may still be running).  The exchange schedule -- which record slots
 * go through one all-reduce -- depends only on the call sequence and the group size agreed at
 * tk_decomp_create (TKHIP_XCH_GROUP, max over the ranks), never on rank-local state; create
 * also checks that every rank describes the same decomposition (d_total, kmax, method, n). */

/* Exp-sum-term split (more ranks than factors): a rank holding a REPLICA of
 * factors another rank owns runs the same steps (bitwise the same basis) but sends zero rows
 * into the records all-reduce, so every factor's record is counted once; at convergence each
 * replica forms its own slice of the t columns of X_s = V_s Y_s (tk_decomp_basis_mul with
 * Y_s[:, c0:c1]), i.e. basis_tensor_mul! (src/utils.jl:478-488) over the exponential-sum
 * terms of src/tensor_krylov_method.jl:10-34.  Call before tk_decomp_init; needs a handle
 * with a records exchange (TK_ERR_STATE otherwise).  replica = 0 is a no-op. */
tk_status tk_decomp_set_replica(tk_decomp* dc, int replica);

/* Per-factor record layout (doubles; m = tk_record_len(kmax)), written by every step:
 *   [0 .. kmax+1]        H[0..j+1, j] as computed by this step (rest 0)
 *   [kmax+2 .. 2kmax+3]  Gram row G[c, 0..c] = V[:,c]' V[:,0..c] of column c below
 *   [2kmax+4]            btilde[c] = <V[:,c], b_s>   (update_rhs!, src/utils.jl:466-476).
 *                        One-sweep Arnoldi handles (tk_decomp_arnoldi_sweeps == 1) form it
 *                        as norm(b_s) * <V[:,c], V[:,0]> (b_s = norm(b_s) V[:,0], so b_s is
 *                        not re-read); the other paths dot with b_s itself.  Equal in exact
 *                        arithmetic; they round differently (both O(eps) for c > 0).
 *   [2kmax+5]            c (column of the Gram row / btilde entry), -1 if none
 *   [2kmax+6]            beta = H[j+1, j] (after any re-orthogonalization)
 *   [2kmax+7]            loss (LanczosReorth: ||V[:,0..j+1]'V[:,0..j+1] - I||_F after TTR)
 *   [2kmax+8]            1.0 if LanczosReorth re-orthogonalized this step (MGS redo)
 *   [2kmax+9]            Gram tracked for this factor (1.0) or not (0.0)
 * Records are laid out [d_total][m]; slots of factors owned by other ranks are summed
 * in by the all-reduce (zero otherwise). */
int tk_record_len(int kmax);

/* initialize_decomp! + initialize_compressed_rhs (src/decompositions.jl:112-118,
 * src/utils.jl:456-464): V[:,0] = inv(norm(b)) .* b; record carries btilde[0] and
 * G[0,0].  rec_out: [d_total][m] or NULL (then nothing is synchronised). */
tk_status tk_decomp_init(tk_decomp* dc, double* rec_out);

/* orthonormalize!(td, k) for all of this rank's factors, k = j+1
 * (src/orthogonal_bases.jl:142-180 fan-out; per-factor steps :15-37 / :39-67 /
 * :98-139).  Must be called with j = 0, 1, ... in order.  The record of step j holds
 * H[0..j+1, j] and, for the fused pipeline, btilde[j] and G[j, 0..j] of column j.
 * rec_out NULL = asynchronous (records stay on the device; see tk_decomp_records). */
tk_status tk_decomp_step(tk_decomp* dc, int j, double* rec_out);

/* Enqueue steps j0 .. j1-1 back to back with no host synchronisation (the device
 * iteration of the driver loop, src/tensor_krylov_method.jl:63-66).  All three methods
 * run asynchronously: TK_LANCZOS_REORTH takes its loss check and MGS-redo decision on the
 * device (src/orthogonal_bases.jl:119-131). */
tk_status tk_decomp_sweep(tk_decomp* dc, int j0, int j1);

/* Write the last pending basis column V[:, j+1] (the fused pipeline defers it into
 * the next step); its btilde / Gram row go to the flush record.  rec_out may be NULL. */
tk_status tk_decomp_flush(tk_decomp* dc, double* rec_out);

/* Copy records of slots s0 .. s1-1 (slot 0 = init, slot j+1 = step j,
 * slot kmax+1 = last flush) to host out[(s1-s0)][d_total][m]. */
tk_status tk_decomp_records(tk_decomp* dc, int s0, int s1, double* out);

/* Copy V[:, c0 .. c0+nc-1] of local factor f (0-based within this rank) to host
 * (column-major n x nc).  Flushes a pending column first. */
tk_status tk_decomp_get_basis(tk_decomp* dc, int f, int c0, int nc, double* out);

/* orthogonality_loss's Gram matrix (src/orthogonal_bases.jl:231-257) of local factor f:
 * G = V[:, 0..k)' V[:, 0..k), k <= min(64, kmax+1), column-major k x k on the host (G NULL:
 * leave it on the device -- benchmarks), as ONE SYRK of the basis on v_mfma_f64_16x16x4f64
 * (the sum over the n rows runs in the matrix core; partials summed in a fixed order, so the
 * result is bitwise reproducible).  A pending column is flushed first when k includes it.
 * This is how a handle with a deferred Gram (tk_decomp_gram_deferred) provides the driver's
 * orthogonality_data of factor 1 (src/tensor_krylov_method.jl:103): orthogonality_data[k] =
 * norm(G[0..k, 0..k] - I) for every k from one G, instead of a Gram row in every step. */
tk_status tk_decomp_gram(tk_decomp* dc, int f, int k, double* G);
/* The same Gram launched AHEAD, asynchronously, over the longest prefix of columns that are
 * already written (no flush, so no record exchange: safe on one rank of many), when this rank
 * holds global factor 0 of a deferred-Gram handle (else nothing happens; *k_out = 0).
 * tk_solver_run calls it as soon as the last step of the loop is issued, so the SYRK runs right
 * behind the steps while the host evaluates the last iterations; a later tk_decomp_gram(dc, 0,
 * k, G) with k <= *k_out reads the leading k x k block of that result instead of launching
 * (columns 0..k-1 never change until the next tk_decomp_init, which drops it). */
tk_status tk_decomp_gram_ahead(tk_decomp* dc, int* k_out);
/* 1 when global factor 0's Gram rows are NOT carried in the step records (its record's
 * "tracked" field is 0) and orthogonality_data comes from tk_decomp_gram at the end: the
 * default for TK_ARNOLDI / TK_LANCZOS with kmax < 64 (the one-sweep Lanczos step reads no
 * basis row, so a per-step Gram row would stream the tracked factor's whole basis every step;
 * for Arnoldi the row's dots make the tracked factor the slowest rank at one factor per GPU).
 * TKHIP_GRAM=rows | deferred at create overrides it for TK_ARNOLDI / TK_LANCZOS;
 * TK_LANCZOS_REORTH (its loss check drives the redo) and track_all_gram keep rows. */
int tk_decomp_gram_deferred(tk_decomp* dc);

/* Launch streams of the one-sweep Arnoldi step: 2 when the local factors step as two groups,
 * each in its own launches on its own stream of the context (one group's launch drain and
 * reduce overlap the other's sweep), else 1.  Groups apply with nf >= 2 local factors, on a
 * single rank or under a records exchange whose steps signal through the signal word (both
 * groups' bookkeeping blocks count into it; slot guards are waited for on both streams);
 * TKHIP_FACTOR_GROUPS=1 at create keeps one stream.  Results are
 * bitwise those of one stream (every kernel is per factor). */
int tk_decomp_factor_groups(tk_decomp* dc);
/* 1 when V_s is kept in single-column tiles (the Gram-free one-sweep TensorLanczos: its step
 * reads one basis column and writes one, 40 bytes per row), 0 for paired columns; a layout
 * detail every reader of the basis (tk_decomp_get_basis, tk_decomp_basis_mul, tk_decomp_gram)
 * handles itself.  TKHIP_LANCZOS_SL=0 keeps the pairs. */
int tk_decomp_single_columns(tk_decomp* dc);

/* basis_tensor_mul! (src/utils.jl:478-488, called at src/tensor_krylov_method.jl:112):
 * X_s = V_s[:, 0..k-1] * Y_s for every local factor, on MFMA (v_mfma_f64_16x16x4).
 * Y: host [nf][t][k] (each Y_s column-major k x t).  X: host [nf][t][n] (column-major
 * n x t each) or NULL to leave the product on the device (benchmarks; on the device X_s
 * is tile-major like V_s: 256-row tiles, each tile's t columns of 256 rows contiguous).
 * A pending column is finalized first (as tk_decomp_flush, its record in the flush slot);
 * for TK_ARNOLDI with k <= the step count <= 64, in the same launch as the product: the
 * flush's register row of each basis tile also forms the product (FP64 FMAs, Y through the
 * scalar cache), so V is streamed once for both; otherwise (and with TKHIP_NO_FUSED_FLUSH=1)
 * the flush runs first and the product on v_mfma_f64_16x16x4f64. */
tk_status tk_decomp_basis_mul(tk_decomp* dc, int k, int t, const double* Y, double* X);

/* ---------------------------------------------------------------- timing hooks */
/* Device time (ms, total) and launch count of a kernel class recorded with HIP events on
 * the ctx stream since the last tk_timing_enable.  on = 1: classes 0 (one step group per
 * tk_decomp_step called outside a sweep), 5 (basis_mul), 6 (exchange) and 7 (one
 * tk_decomp_sweep: its step groups back to back); on = 2 adds per-kernel classes
 * 1 (first / one-sweep pass), 2 (second pass), 3 (finalize), 4 (reduce + post). */
tk_status tk_timing_enable(tk_ctx* ctx, int on);
tk_status tk_timing_read(tk_ctx* ctx, int cls, double* total_ms, long* launches);

/* ---------------------------------------------------------------- compressed side (host)
 * The k-sized per-iteration work of tensorkrylov! (no GPU needed).
 * Matrices are column-major; factor s's k x k block starts at s*k*k, its b~ at s*k, its
 * k x t Y_s at s*k*t. */

/* solve_compressed_system (src/tensor_krylov_method.jl:10-34, src/utils.jl:501-523):
 * lambda[j] = omega[j] / lmin and Y_s[:, j] = exp(-alpha[j]/lmin * first(H)) b~_s, where
 * first(H) = Symmetric(H1, :L) if `symmetric` (one eigendecomposition serves all t terms)
 * and the full H1 otherwise (Pade scaling-and-squaring exponential per term). */
tk_status tk_compressed_solve(int d, int k, const double* H1, int symmetric, const double* bt, int t,
                              const double* alpha, const double* omega, double lmin, double* lambda,
                              double* Y);

/* residualnorm! + compressed_residual (src/utils.jl:371-443, Lemma 3.4): H = the d k x k
 * minors, subdiag[s] = H_s[k+1, k].  Returns TK_BREAKDOWN (with *r_comp set) when the
 * compressed squared residual is negative, as the reference throws CompressedNormBreakdown. */
tk_status tk_residualnorm(int d, int k, int t, const double* H, const double* lambda, const double* Y,
                          const double* subdiag, const double* bt, double bnorm, double* r_comp,
                          double* r_norm);

/* ---------------------------------------------------------------- native iteration driver
 * The host side of tensorkrylov!'s loop (src/tensor_krylov_method.jl:63-118) in native code:
 * a tk_solver keeps the host mirror of H_s, b~_s and factor 1's Gram rows, applies step
 * records exactly as the reference mutates H (orthonormalize!, update_subdiagonals!,
 * LanczosReorth's zeroing, update_rhs!) and evaluates iteration k = compressed solve +
 * residualnorm! + orthogonality_loss(V_1, k).  The spectral / exp-sum data depend only on
 * A and tol and are passed per k at create: lmin[k-1] (lambda_min of the k x k minor times
 * d, src/eigenvalues.jl:353-370), rank[k-1] = t (0 = no tabulated rank: the loop stops
 * before k) and t coefficients alpha/omega per k, concatenated in k order
 * (src/approximation.jl:65-175). */
typedef struct tk_solver tk_solver;
tk_status tk_solver_create(int method, int d, int kmax, int symmetric, double b_norm, const double* lmin,
                           const int* rank, const double* alpha, const double* omega, tk_solver** out);
tk_status tk_solver_destroy(tk_solver* sv);
/* Apply the records [d][m] of ABI step j (j = -1: tk_decomp_init's record). */
tk_status tk_solver_apply(tk_solver* sv, int j, const double* rec);
/* Evaluate iteration k (records of steps < k applied): out4 = {r_comp, r_norm,
 * r_norm / norm(b), orthogonality loss of V_1}.  TK_BREAKDOWN as tk_residualnorm. */
tk_status tk_solver_evaluate(tk_solver* sv, int k, double* out4);
int tk_solver_rank(tk_solver* sv, int k);
/* lambda (t) and Y [d][t][k] of iteration k, which must be the last one evaluated (by
 * tk_solver_evaluate, or the iteration tk_solver_run ended on). */
tk_status tk_solver_solution(tk_solver* sv, int k, double* lambda_out, double* Y_out);
/* Host mirror: H [d][kmax+2][kmax+1] (row-major), b~ [d][kmax+1], Gram rows of factor 1
 * [(kmax+1)^2] (row c holds G[c, 0..c]); NULL outputs are skipped. */
tk_status tk_solver_state(tk_solver* sv, double* H_out, double* bt_out, double* gram0_out);
/* Diagnostic (bench.py --emulate-ranks): records of factors outside [first, first+nf) are
 * replaced, whenever records are applied, by those of a full run, records[slot][d][m]
 * (slot = j + 1, kmax + 2 slots), so one GPU holding one rank's factors drives the same
 * iterates as the whole job.  records = NULL removes the overlay. */
tk_status tk_solver_overlay(tk_solver* sv, int first, int nf, const double* records);
/* Start the native loop's evaluation threads ahead of tk_solver_run (the driver's setup): at
 * least nthreads workers, kept by the solver until tk_solver_destroy (a run needing more --
 * the agreed worker count -- starts the rest itself). */
tk_status tk_solver_prepare(tk_solver* sv, int nthreads);
/* The pipelined loop for k = kfirst .. kmax on a decomposition whose steps < kfirst-1 are
 * done and applied: enqueues steps up to `depth` ahead, applies each step's records in
 * order and evaluates up to `nthreads` iterations concurrently on host threads (each
 * iteration's evaluation reads only data that later steps do not touch, so every iterate
 * is bitwise the sequential loop's).  relres / projres / orth [kmax] receive the
 * reference's ConvergenceData entries (index k-1).  *outcome: 0 = no convergence through
 * *k_end, 1 = converged at *k_end (tk_solver_solution gives its y), 2 = compressed norm
 * breakdown at *k_end + 1 (src/tensor_krylov_method.jl:83-95).  Steps enqueued beyond
 * *k_end may still run; their results are not read. */
tk_status tk_solver_run(tk_solver* sv, tk_decomp* dc, double tol, int kfirst, int depth, int nthreads,
                        double* relres, double* projres, double* orth, int* k_end, int* outcome);
/* Evaluation split over the ranks of one node (the reference evaluates every
 * iteration itself, src/tensor_krylov_method.jl:72-103): after tk_solver_share, iteration k's
 * compressed solve + residual is evaluated by rank (k mod nranks) only, and every other rank
 * reads its (r_comp, r_norm, relres, orthogonality, status) from a node-local mailbox -- POSIX
 * shared memory /dev/shm/tkhip_ev_<key>, created by rank 0, unlinked as soon as every rank has
 * attached (so nothing is left behind).  Every rank holds the same host mirror (the records
 * all-reduce), so the result is bitwise what it would have computed, and convergence /
 * breakdown are decided at the same iteration on every rank.  Collective: every rank calls it
 * with the same key (e.g. derived from the RCCL unique id) and nranks; waits are bounded by
 * TKHIP_WAIT_S.  tk_solver_run splits only when every rank of the decomposition's exchange
 * shares (agreed at the run's start); on convergence at an iteration another rank evaluated,
 * the run evaluates it locally for tk_solver_solution.  nranks = 1 turns the split off. */
tk_status tk_solver_share(tk_solver* sv, const char* key, int nranks, int rank);
/* Diagnostic (bench.py --emulate-ranks): the split on one rank, with the results of the
 * iterations other ranks would own taken from `results` ([kmax][6], tk_solver_results of a
 * full run), each released no earlier than its record's arrival plus the evaluation time that
 * run measured for it.  nranks = 1 turns it off. */
tk_status tk_solver_share_emulated(tk_solver* sv, int nranks, int rank, const double* results);
/* Per iteration k (row k-1) of the last tk_solver_run: r_comp, r_norm, relres, orthogonality
 * loss, status (TK_OK / TK_BREAKDOWN), this rank's evaluation time in us (-1 if another rank
 * evaluated it); NaN rows for iterations the run did not consume.  out: [kmax][6]. */
tk_status tk_solver_results(tk_solver* sv, double* out);
/* tk_solver_evaluate under the split (a host-driven loop, one call per k in order on every
 * rank): the owner evaluates and posts, the others wait for its result; out4 and the status as
 * tk_solver_evaluate.  Without tk_solver_share it is tk_solver_evaluate. */
tk_status tk_solver_evaluate_shared(tk_solver* sv, int k, double* out4);
/* orthogonality_loss(V, k) = norm(V[:, 1:k]' V[:, 1:k] - I) for k = 1..K from ONE Gram matrix
 * G = V[:, 1:K]' V[:, 1:K] (K x K column-major, lower triangle read) into out[K]
 * (src/orthogonal_bases.jl:250-257, called per iteration at src/tensor_krylov_method.jl:103):
 * the squared loss grows by column k's diagonal and twice its off-diagonal squares, in the
 * order tk_solver_evaluate sums a tracked factor's Gram rows.  tk_solver_run fills orth[]
 * with it on the rank holding factor 1 of a deferred-Gram handle when the Gram launched
 * behind the last step (tk_decomp_gram_ahead) covers the iterations it ran; entries it
 * could not fill stay NaN. */
tk_status tk_orthogonality_losses(int K, const double* G, double* out);

#ifdef __cplusplus
}
#endif
#endif /* TK_H_ */
