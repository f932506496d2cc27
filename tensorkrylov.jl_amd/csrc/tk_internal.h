// tk_internal.h -- device-side descriptors shared by tk_kernels.hip and tk_abi.cpp.
#ifndef TK_INTERNAL_H_
#define TK_INTERNAL_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tk {

// Scalars kept per factor on the device (DFac::sc).
enum {
    SC_BETA = 0,      // beta of the last completed step (H[j+1, j])
    SC_INVBETA = 1,   // inv(beta)
    SC_BETAPREV = 2,  // Lanczos beta_{j-1} for a plain (non-fused) TTR step
    SC_INVB = 3,      // inv(norm(b))
    SC_BNORM = 4,     // norm(b)
    SC_REDO = 5,      // LanczosReorth: 1 when this step's loss check asks for the MGS redo
    SC_ALPHA = 6,     // one-sweep Lanczos: alpha of the last step (its pending column's w = u - alpha v)
    SC_COUNT = 8
};

// Sparse A_s on the device: CSR always; DIA (diagonal storage, ascending offsets,
// zero-padded) in addition when the matrix is banded with few, mostly full diagonals --
// then the SpMV has no index loads.  Both sum each row in ascending column order.
struct SpM {
    const int* rowptr;    // CSR (n+1)
    const int* col;       // (nnz) ascending within a row
    const double* val;    // (nnz)
    const int* doff;      // DIA offsets (ndiag), ascending
    const double* dval;   // DIA values [ndiag][dld]: dval[q*dld + r] = A[r, r + doff[q]]
    int ndiag;            // > 0: DIA is used
    int64_t dld;
    const double* dconst; // Toeplitz band: the one value of each diagonal (>= 4 entries)
    int toep;             // 1: every diagonal is constant and complete (dconst valid)
    // SELL-256: slice = one 256-row tile; entry q of row r at sptr[r/256] + q*256 + r%256
    const long long* sptr;  // (ntiles) slot offset of each slice
    const int* swidth;    // (ntiles) slice width = max row length in the slice
    const int* rowlen;    // (ntiles*256) row lengths (0 for padding rows)
    const int* scol;      // (slots) column, padded entries repeat the row index
    const double* sval;   // (slots) value, padded entries 0
    int sell;             // 1: SELL is used (when ndiag == 0)
    int64_t n;
};

// Per-factor device descriptor.  One array of these lives in device memory; kernels
// index it with blockIdx.y, so every launch covers all of this rank's factors.
struct DFac {
    SpM A;                // A_s
    double* V;            // basis, tile-major, paired columns (tk_kernels.hip header)
    const double* b;      // b_s (n)
    double* W;            // work vector (SpMV output / Lanczos v)
    double* U;            // work vector (w' / Lanczos u)
    double* P1;           // block partials [value][npart], first reduction of a step
    double* P2;           // block partials, second reduction
    double* RED1;         // reduced values of P1
    double* RED2;         // reduced values of P2
    double* sc;           // scalars (SC_*)
    double* h2;           // second-pass coefficients of the last Arnoldi step (kmax+2)
    double* g;            // Hbar * h2 (kmax+2)
    double* H;            // Hessenberg, column-major (kmax+2) x (kmax+1)
    double* lossrow;      // per column c: its share of ||V'V - I||_F^2 (LanczosReorth loss check)
    int track_gram;       // keep Gram rows for this factor
    int gidx;             // global factor index (record slot)
    // one-sweep Arnoldi (k_arn_d1, banded A_s only): lower/upper bandwidth, overlapping
    // row windows of stride 256 - 2(hl+hu), window count, partial blocks (a function of
    // n, hl, hu only)
    int hl, hu, nwin, npd;
    // one-sweep Lanczos without a Gram row (k_lan_1w): windows of LAN_RPT * 256 rows owning
    // all but hl + hu of them (one SpMV), their count (a function of n, hl, hu only)
    int nwl;
    // one-sweep Arnoldi: the even column written by the last even step (v_j, n rows); the
    // odd step after it stores the pair (v_{j-1}, v_j) once, so no column is written twice
    double* E;
    // CGS2 with one A_s shared by all local factors: their raw vectors U interleaved
    // (Uint[r * inf + ifs], shared by the group) feed one gather per nonzero for all factors
    // (k_spmv_mf), whose A U lands in AU; null otherwise
    double* Uint;
    double* AU;
    int ifs, inf;
    // one-sweep reduce: arrival counter of the step's value groups (the last one evaluates
    // the next step's scalars, red_d1_block)
    unsigned int* ctr;
    // one-sweep reduce, first level: each group's per-split sums ([group][split][16]) and the
    // group's arrival counter (the last split block of a group sums the splits in order)
    double* Q;
    unsigned int* ctrg;
    // fused one-sweep launches (the previous step's reduce in the leading blocks): the odd
    // steps' partials, and the step word the reducers publish and the window blocks wait for
    double* P1b;
    unsigned long long* rword;
    // records exchange: this factor's own exchange signal word, set to the step's KArgs::xval by
    // a plain store (host-resident signal memory: an atomic add there is a non-posted round trip
    // the launch waits for; with factor groups one shared count could also be reached with a
    // step of one group missing); null: an add to KArgs::xflag
    unsigned long long* xsig;
};

struct KArgs {
    int64_t n;        // rows
    int64_t ld;       // padded length of every n-vector (n rounded up to 256)
    int j;            // step (0-based column)
    int npart;        // partial blocks per factor (function of n only)
    int ntiles;       // ceil(n / 256)
    int kmax;
    int m;            // record length per factor
    double* rec;      // record slot base ([d_total][m])
    int fmt;          // storage common to all factors of the launch: 1 DIA, 2 SELL, 3 CSR, 0 mixed
    int gate;         // 1: a block does nothing unless its factor's SC_REDO flag is set
    int ubuf;         // one-sweep Arnoldi: 0 = the pending raw vector u is in U, 1 = in W
    unsigned long long* xflag;   // non-null: each k_post block adds 1 once its record is
                                 // written (signal memory the exchange stream waits on)
    double* hrec;                // non-null: the step's record slot in host-mapped memory
                                 // ([d_total][m]); k_post copies its row there ...
    unsigned long long* hdone;   // ... then stores `seq` to hdone[local factor] (host-mapped)
    unsigned long long seq;
    unsigned long long xval;     // exchange signal of this step (per-factor words, DFac::xsig): the
                                 // value its k_post / bookkeeping block stores (monotonic per handle)
    int ecol;         // flush of the one-sweep pending column: this column (j) is in DFac::E, not V (-1: none)
    int mfs;          // CGS2 pass 1: A U comes from DFac::AU (k_spmv_mf ran), not from its own gathers
    int sl;           // 1: V in single-column tiles (column c of a tile at c * 256 doubles, row
                      // stride 8 B) -- the Gram-free one-sweep TensorLanczos, whose step reads one
                      // column and writes one; 0: paired columns (tk_kernels.hip header)
    int red;          // fused one-sweep launch: its leading blocks reduce step j-1's partials
    int redmm;        // ... with the memory-model hand-off (red_mm())
    unsigned long long wseq;   // ... and publish this in each factor's step word (DFac::rword)
    unsigned int* werr;        // ... a wait that gave up sets this (host-mapped, the context's)
    unsigned int wspin;        // ... polls before a wait gives up (2^22; a test build may lower it)
    // one-sweep Arnoldi, one stream (no factor groups): the step's reduce is a plain reduction and
    // the windows evaluate the next step's scalars (d1_scalars); 0: the reduce's last block does
    // and stores them (with two group streams that reduce hides behind the other group's sweep)
    int wsc;
    int pgrp;         // one-sweep Arnoldi, factor groups without fused launches: the window partials
                      // in window-major groups (D1G) and their reduce red_d1_block; 0: value-major
};

// One-sweep Arnoldi steps j <= D1_JMAX (the j basis columns it reads fit the register
// row); later steps of the same decomposition run as CGS2.
constexpr int D1_JMAX = 64;
// the one-sweep Arnoldi runs steps j <= ARN_D1_JMAX: its last step is odd, so leaving the
// range never leaves an even column in DFac::E (the CGS2 kernels read V only)
constexpr int ARN_D1_JMAX = 63;
// RED1 length: 3 kmax + 8 reduced values, plus the span one-sweep register rows read past
// the live coefficients (2 x 64 + 16)
#define RED1_LEN(kmax) (3 * (kmax) + 8 + 144)
// One-sweep Arnoldi partials (k_arn_d1 -> red_d1_block): window-major groups of D1G values, group
// g of window w at P1[(g * npd + w) * D1G + v % D1G] -- each window stores every group as one
// whole 128-byte line (16 lanes of one instruction) -- on factor groups over long grids
// (KArgs::pgrp); value-major P1[v * npd + w] elsewhere.  Both reduces sum in the same order
// (red_d1_block emulates red256_block's), so the layout never changes a bit of the results.
#define D1G 16
__host__ __device__ inline int d1_groups(int nv) { return (nv + D1G - 1) / D1G; }
// values the reduce of one-sweep Arnoldi step J - 1 sums (J = coefJ): c and q (J each), |u|^2,
// <u,z>, <v,v_0>, the Gram diagonal, and a tracked factor's Gram row (J - 1)
__host__ __device__ inline int d1_nv(int J, int track_gram) { return track_gram ? 3 * J + 3 : 2 * J + 4; }
// launch_reduce's coefJ for a one-sweep Lanczos step (k_lan_1s)
#define RED_LAN (-2)
// where a one-sweep step's reduced dots (3j+6 values) are followed by the next step's
// scalars (k_reduce256's last block): ib, gamma, beta, t1
#define D1S_IB 0
#define D1S_GAMMA 1
#define D1S_BETA 2
#define D1S_T1 3

// launchers (tk_kernels.hip)
void launch_mirror_records(const double* src, double* dst, int cnt, unsigned long long* done, int nslots,
                           unsigned long long seq, hipStream_t s);
void launch_delay_us(double us, hipStream_t s);   // test-only (TKHIP_TEST_XCH_DELAY_US)
// k_reduce256's hand-off form (0 relaxed, 1 memory model): process-wide, set before launches
int red_mm();
void set_red_mm(int on);
void launch_fin_vy(const DFac* F, int nf, const KArgs& a, const double* Y, double* X, int ldy, int t, int mode,
                   hipStream_t s);
void launch_init_a(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_init_b(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_arn_a1_plain(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_arn_a1_fused(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_arn_a2(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_arn_finalize(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_init_bd(const DFac* F, int nf, const KArgs& a, int npd, hipStream_t s);
void launch_arn_d1(const DFac* F, int nf, const KArgs& a, const KArgs& b, int npd, bool gram, bool vcache,
                   bool fuse, hipStream_t s);
void launch_lan_1s(const DFac* F, int nf, const KArgs& a, int npd, hipStream_t s);
// the gram-free one-sweep Lanczos step (k_lan_1w; npd = the largest DFac::nwl); b.j >= 0: the
// previous step's record mirror + signal ride in 8 leading blocks
void launch_lan_1w(const DFac* F, int nf, const KArgs& a, const KArgs& b, int npd, hipStream_t s);
// ... and its reduce: one 1024-thread block per factor ends the step (alpha, beta, record)
void launch_red_lan(const DFac* F, int nf, const KArgs& ax, hipStream_t s);
// rows per thread of k_lan_1w (its windows are LAN_RPT * 256 rows; 2: 67 us per C2 step
// against 71 at 4 and 77 at 8, profiles/r03/lan_rpt_ab.txt)
#ifndef TK_LAN_RPT
#define TK_LAN_RPT 2
#endif
constexpr int LAN_RPT = TK_LAN_RPT;
inline int lan_windows(int64_t n, int hl, int hu) {
    const int ws = LAN_RPT * 256 - hl - hu;
    return (int)((n + ws - 1) / ws);
}
void launch_spmv_mf(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_lan_l1_plain(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_lan_l1_fused(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_lan_d1(const DFac* F, int nf, const KArgs& a, hipStream_t s);   // j in 1..64
void launch_lan_l2(const DFac* F, int nf, const KArgs& a, hipStream_t s);
void launch_lan_finalize(const DFac* F, int nf, const KArgs& a, hipStream_t s);
// ungated write of the pending column j+1 for j + 1 <= 64 columns (mode 0 Arnoldi, 1 Lanczos):
// one partial per tile (reduce with npart = ntiles)
void launch_fin_d(const DFac* F, int nf, const KArgs& a, int mode, hipStream_t s);
// npart <= 0: each factor's own DFac::npd partials (one-sweep Arnoldi)
// the one-sweep Arnoldi step's reduce of step J - 1 over window-major partials (KArgs::pgrp,
// red_d1_block); npd: the launch's largest window count
void launch_red_d1(const DFac* F, int nf, int which, int J, int npd, hipStream_t s);
void launch_reduce(const DFac* F, int nf, int which, int nv, int npart, hipStream_t s, int gate = 0,
                   int coefJ = -1, const KArgs* ax = nullptr);
// post-processing (one 64-thread block per factor)
enum PostKind {
    POST_INIT_A = 0,
    POST_INIT_B = 1,
    POST_ARN = 2,        // after a2; fused flag in `flag`
    POST_ARN_FIN = 3,    // after arn_finalize (column j+1)
    POST_LAN = 4,        // after l2; fused flag in `flag`
    POST_LAN_FIN = 5,    // after lan_finalize (column j+1)
    POST_ARN_D = 6,      // after k_arn_d1 (one-sweep Arnoldi): H column j, c, beta, next h1
    POST_SIGNAL = 7      // only mirror the finished record to the host (LanczosReorth)
};
void launch_post(const DFac* F, int nf, const KArgs& a, int kind, int flag, int clear, hipStream_t s);
void launch_get_cols(const double* V, int64_t n, int kmax, int c0, int nc, double* out, int sl, hipStream_t s);
void launch_basis_mul(const DFac* F, int nf, const KArgs& a, const double* Y, double* X, int k,
                      int t, hipStream_t s);
void launch_spmv(const SpM& A, const double* x, double* y, hipStream_t s);
// G = V_f[:, 0..k)' V_f[:, 0..k) on MFMA (k <= 64), into scratch (gram_scratch_doubles(ntiles)):
// gram_values(k) results at scratch + gram_result_offset, layout of k_gram (tk_kernels.hip)
int gram_values(int k);
int gram_blocks(int ntiles);
size_t gram_scratch_doubles(int ntiles);
inline size_t gram_result_offset(int ntiles, int k) {
    return (size_t)(gram_blocks(ntiles) + 64) * gram_values(k);
}
void launch_gram(const DFac* F, int f, const KArgs& a, int k, double* scratch, hipStream_t s);
// the gram_values(k) results -> G (k x k, both triangles)
void gram_unpack(int k, const double* v, double* G);

// record field offsets (see include/tk.h)
__host__ __device__ inline int rec_len(int kmax) { return 2 * kmax + 10; }
__host__ __device__ inline int rec_gram(int kmax) { return kmax + 2; }
__host__ __device__ inline int rec_bt(int kmax) { return 2 * kmax + 4; }
__host__ __device__ inline int rec_col(int kmax) { return 2 * kmax + 5; }
__host__ __device__ inline int rec_beta(int kmax) { return 2 * kmax + 6; }
__host__ __device__ inline int rec_loss(int kmax) { return 2 * kmax + 7; }
__host__ __device__ inline int rec_flag(int kmax) { return 2 * kmax + 8; }
__host__ __device__ inline int rec_tracked(int kmax) { return 2 * kmax + 9; }

}  // namespace tk

#endif
