// tk_kernels.hip -- gfx950 (MI355X) kernels for the inner Krylov iteration of
// thbake/TensorKrylov.jl.  Written for CDNA4: 64-lane waves, 256-thread blocks,
// thread-per-row streaming of the column-major basis V (n x (kmax+1), ld = n rounded
// up to 256) with the row held in VGPRs, deterministic LDS-transpose block reductions,
// and f64 MFMA (v_mfma_f64_16x16x4_f64) for the tall-skinny V*Y product.
//
// Numerical scheme (DESIGN.md "Arnoldi step"): the reference's two-pass MGS
// (src/orthogonal_bases.jl:15-37) is computed as CGS2 -- h1 = V'w, w' = w - V h1,
// h2 = V'w', H[:,j] = h1 + h2, beta = sqrt(|w'|^2 - |h2|^2),
// v_{j+1} = (w' - V h2) * inv(beta) -- equal to MGS2 in exact arithmetic and within
// the parity tolerance in floating point (tests/test_gpu_parity.py).  The correction
// v_{j+1} is not written by a pass of its own: the next step's SpMV kernel writes it
// while it holds the same V rows in registers, applying A to w' and subtracting
// A V h2 = V Hbar h2 through the Arnoldi relation.  V is therefore streamed twice per
// step (the compulsory MGS2 traffic of SURVEY.md section 8d), not three times.
//
// Every reduction is fixed-order (per-block LDS transpose, then one wave per value
// over NPART block partials, NPART a function of n only), so results are bitwise
// reproducible run to run and independent of how the factors are split over GPUs.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "tk_internal.h"

namespace tk {

#define TPB 256          // threads per block == rows per tile
#define CH 16            // columns per block-reduction chunk
#define TSTR (TPB + 16)  // LDS row stride (doubles): the +32 dwords put the two 32-lane
                         // halves of a ds_read_b64 on disjoint banks

// ------------------------------------------------------------------ small helpers

// Julia's CSC scatter adds nz*x into y without FMA; keep the product and the sum
// separately rounded so the device SpMV matches it bit for bit.  (__dmul_rn/__dadd_rn
// are plain * and + in ROCm 7.2's headers, so contraction must be switched off with
// the pragma at every use site.)
__device__ __forceinline__ double mul_rn(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b) {
#pragma clang fp contract(off)
    return a + b;
}

// Accumulate, over the block's 256 rows, CH per-thread values x[0..CH) into acc[base..]
// (LDS).  Fixed order: lane (col*16+part) sums elements q*16+part, q ascending, of
// column col, then a 16-lane xor butterfly.
__device__ __forceinline__ void chunk_reduce(const double (&x)[CH], double* __restrict__ tr,
                                             double* __restrict__ acc, int base, bool first) {
    const int t = threadIdx.x;
#pragma unroll
    for (int c = 0; c < CH; ++c) tr[c * TSTR + t] = x[c];
    __syncthreads();
    const int col = t >> 4, part = t & 15;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += tr[col * TSTR + q * 16 + part];
    s += __shfl_xor(s, 8);
    s += __shfl_xor(s, 4);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 1);
    if (part == 0) acc[base + col] = first ? s : acc[base + col] + s;
    __syncthreads();
}

// Block-reduce one per-thread scalar into acc[base].
__device__ __forceinline__ void reduce_one(double y, double* tr, double* acc, int base, bool first) {
    const int t = threadIdx.x;
    double s = y;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((t & 63) == 0) tr[CH * TSTR - 4 + (t >> 6)] = s;
    __syncthreads();
    if (t == 0) {
        const double* w = tr + CH * TSTR - 4;
        const double tot = (w[0] + w[1]) + (w[2] + w[3]);
        acc[base] = first ? tot : acc[base] + tot;
    }
    __syncthreads();
}

// The first MAXC columns of this thread's row of V live in VGPRs; columns beyond
// MAXC (kmax > MAXC) are streamed from memory on each use.
template <int MAXC>
struct Row {
    double v[MAXC];
    __device__ __forceinline__ void load(const double* __restrict__ V, int64_t ld, int64_t r,
                                         int ncols, bool ok) {
#pragma unroll
        for (int c = 0; c < MAXC; ++c) v[c] = (ok && c < ncols) ? V[r + (int64_t)c * ld] : 0.0;
    }
};

// sum_c V[r, c] * h[c], c < ncols (h uniform, in global memory)
template <int MAXC>
__device__ __forceinline__ double row_dot(const Row<MAXC>& R, const double* __restrict__ V,
                                          int64_t ld, int64_t r, int ncols, bool ok,
                                          const double* __restrict__ h) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
        if (c < ncols) s += R.v[c] * h[c];
    for (int c = MAXC; c < ncols; ++c) s += (ok ? V[r + (int64_t)c * ld] : 0.0) * h[c];
    return s;
}

// Block-reduce x_c = V[r, c] * y, c < ncols, into acc[base + c] (acc entries up to
// base + roundup16(ncols) are written; later reduce_one calls may overwrite them).
template <int MAXC>
__device__ __forceinline__ void reduce_cols(const Row<MAXC>& R, const double* __restrict__ V,
                                            int64_t ld, int64_t r, int ncols, bool ok, double y,
                                            double* tr, double* acc, int base, bool first) {
#pragma unroll
    for (int c0 = 0; c0 < MAXC; c0 += CH) {
        if (c0 < ncols) {
            double x[CH];
#pragma unroll
            for (int q = 0; q < CH; ++q) x[q] = (c0 + q < ncols) ? R.v[c0 + q] * y : 0.0;
            chunk_reduce(x, tr, acc, base + c0, first);
        }
    }
    for (int c0 = MAXC; c0 < ncols; c0 += CH) {
        double x[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int c = c0 + q;
            x[q] = (ok && c < ncols) ? V[r + (int64_t)c * ld] * y : 0.0;
        }
        chunk_reduce(x, tr, acc, base + c0, first);
    }
}

// Streaming (no row cache) variant for kernels that touch V only for a Gram row.
__device__ __forceinline__ void reduce_cols_stream(const double* __restrict__ V, int64_t ld,
                                                   int64_t r, int ncols, bool ok, double y,
                                                   double* tr, double* acc, int base, bool first) {
    for (int c0 = 0; c0 < ncols; c0 += CH) {
        double x[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int c = c0 + q;
            x[q] = (ok && c < ncols) ? V[r + (int64_t)c * ld] * y : 0.0;
        }
        chunk_reduce(x, tr, acc, base + c0, first);
    }
}

__device__ __forceinline__ void zero_acc(double* acc, int lo, int hi) {
    for (int c = lo + threadIdx.x; c < hi; c += TPB) acc[c] = 0.0;
}

// Write the block's accumulated values acc[0..nv) to the partial buffer [value][npart].
__device__ __forceinline__ void store_partials(const double* acc, double* __restrict__ P,
                                               int npart, int nv) {
    __syncthreads();
    for (int c = threadIdx.x; c < nv; c += TPB) P[(int64_t)c * npart + blockIdx.x] = acc[c];
}

// CSR row sum in ascending column order, products and sums separately rounded.
__device__ __forceinline__ double spmv_row(const int* __restrict__ rowptr, const int* __restrict__ col,
                                           const double* __restrict__ val, const double* __restrict__ x,
                                           int64_t r) {
#pragma clang fp contract(off)
    double s = 0.0;
    const int p1 = rowptr[r + 1];
    for (int p = rowptr[r]; p < p1; ++p) s = add_rn(s, mul_rn(val[p], x[col[p]]));
    return s;
}
// Same, gathering fl(x[c] * scale) -- bitwise the stored Lanczos column -- or zeros.
__device__ __forceinline__ double spmv_row_scaled(const int* __restrict__ rowptr, const int* __restrict__ col,
                                                  const double* __restrict__ val, const double* __restrict__ x,
                                                  double scale, bool zero, int64_t r) {
#pragma clang fp contract(off)
    double s = 0.0;
    const int p1 = rowptr[r + 1];
    for (int p = rowptr[r]; p < p1; ++p) {
        const double xv = zero ? 0.0 : mul_rn(x[col[p]], scale);
        s = add_rn(s, mul_rn(val[p], xv));
    }
    return s;
}

#define KERNEL_PROLOGUE                                   \
    __shared__ double tr[CH * TSTR];                      \
    extern __shared__ __attribute__((aligned(16))) double acc[]; \
    const DFac& d = F[blockIdx.y];

#define TILE_LOOP                                                                   \
    bool first = true;                                                              \
    for (int tile = blockIdx.x; tile < a.ntiles; tile += a.npart, first = false) {  \
        const int64_t r = (int64_t)tile * TPB + threadIdx.x;                        \
        const bool ok = r < a.n;

// ------------------------------------------------------------------ init kernels

// P1 = [ sum b^2 ]
__global__ __launch_bounds__(TPB) void k_init_a(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    TILE_LOOP
        const double bv = ok ? d.b[r] : 0.0;
        reduce_one(bv * bv, tr, acc, 0, first);
    }
    store_partials(acc, d.P1, a.npart, 1);
}

// V[:,0] = inv(norm(b)) .* b  (src/decompositions.jl:112-118);  P1 = [<v0,b>, <v0,v0>]
__global__ __launch_bounds__(TPB) void k_init_b(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    const double inv = d.sc[SC_INVB];
    TILE_LOOP
        const double bv = ok ? d.b[r] : 0.0;
        const double v0 = inv * bv;
        if (ok) d.V[r] = v0;
        reduce_one(v0 * bv, tr, acc, 0, first);
        reduce_one(v0 * v0, tr, acc, 1, first);
    }
    store_partials(acc, d.P1, a.npart, 2);
}

// ------------------------------------------------------------------ Arnoldi (CGS2)

// First pass, v_j stored:  W = A v_j;  P1 = [ <V[:,c], W>, c = 0..j ].
template <int MAXC>
__global__ __launch_bounds__(TPB) void k_arn_a1_plain(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    const int j = a.j, nc = j + 1;
    const double* vj = d.V + (int64_t)j * a.ld;
    TILE_LOOP
        Row<MAXC> R;
        R.load(d.V, a.ld, r, nc, ok);
        const double w = ok ? spmv_row(d.rowptr, d.col, d.val, vj, r) : 0.0;
        if (ok) d.W[r] = w;
        reduce_cols(R, d.V, a.ld, r, nc, ok, w, tr, acc, 0, first);
    }
    store_partials(acc, d.P1, a.npart, nc);
}

// First pass of step j fused with writing the pending column v_j of step j-1:
//   v_j = (U - V[:,0..j) h2) * inv_beta                     -> V[:, j]
//   W   = (A U - V[:,0..j) g[0..j) - g[j] v_j) * inv_beta    (= A v_j, Arnoldi relation)
//   P1  = [ <V[:,c],W> (c<j), <v_j,W> | gram <V[:,c],v_j> (c<j), <v_j,v_j> | <v_j,b> ]
template <int MAXC>
__global__ __launch_bounds__(TPB) void k_arn_a1_fused(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    const int j = a.j;
    const double inv_beta = d.sc[SC_INVBETA];
    const double gj = d.g[j];
    const bool gram = d.track_gram != 0;
    double* vj_out = d.V + (int64_t)j * a.ld;
    TILE_LOOP
        Row<MAXC> R;
        R.load(d.V, a.ld, r, j, ok);
        const double up = ok ? d.U[r] : 0.0;
        const double vj = ok ? (up - row_dot(R, d.V, a.ld, r, j, ok, d.h2)) * inv_beta : 0.0;
        const double au = ok ? spmv_row(d.rowptr, d.col, d.val, d.U, r) : 0.0;
        const double w = ok ? (au - row_dot(R, d.V, a.ld, r, j, ok, d.g) - gj * vj) * inv_beta : 0.0;
        if (ok) {
            vj_out[r] = vj;
            d.W[r] = w;
        }
        reduce_cols(R, d.V, a.ld, r, j, ok, w, tr, acc, 0, first);
        reduce_one(vj * w, tr, acc, j, first);
        if (gram) {
            reduce_cols(R, d.V, a.ld, r, j, ok, vj, tr, acc, j + 1, first);
            reduce_one(vj * vj, tr, acc, 2 * j + 1, first);
        }
        reduce_one(ok ? vj * d.b[r] : 0.0, tr, acc, 2 * j + 2, first);
    }
    if (!gram) zero_acc(acc, j + 1, 2 * j + 2);
    store_partials(acc, d.P1, a.npart, 2 * j + 3);
}

// Second pass: U = W - V[:,0..j] h1;  P2 = [ <V[:,c],U> (c<=j), <U,U> ].
template <int MAXC>
__global__ __launch_bounds__(TPB) void k_arn_a2(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    const int j = a.j, nc = j + 1;
    TILE_LOOP
        Row<MAXC> R;
        R.load(d.V, a.ld, r, nc, ok);
        const double w = ok ? d.W[r] : 0.0;
        const double u = ok ? (w - row_dot(R, d.V, a.ld, r, nc, ok, d.RED1)) : 0.0;
        if (ok) d.U[r] = u;
        reduce_cols(R, d.V, a.ld, r, nc, ok, u, tr, acc, 0, first);
        reduce_one(u * u, tr, acc, nc, first);
    }
    store_partials(acc, d.P2, a.npart, nc + 1);
}

// Write the pending column j+1 with no following step:
//   v = (U - V[:,0..j] h2) * inv_beta;  P1 = [ gram <V[:,c],v> (c<=j), <v,v>, <v,b> ]
template <int MAXC>
__global__ __launch_bounds__(TPB) void k_arn_finalize(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    const int j = a.j, nc = j + 1;
    const double inv_beta = d.sc[SC_INVBETA];
    double* vout = d.V + (int64_t)(j + 1) * a.ld;
    TILE_LOOP
        Row<MAXC> R;
        R.load(d.V, a.ld, r, nc, ok);
        const double up = ok ? d.U[r] : 0.0;
        const double v = ok ? (up - row_dot(R, d.V, a.ld, r, nc, ok, d.h2)) * inv_beta : 0.0;
        if (ok) vout[r] = v;
        reduce_cols(R, d.V, a.ld, r, nc, ok, v, tr, acc, 0, first);
        reduce_one(v * v, tr, acc, nc, first);
        reduce_one(ok ? v * d.b[r] : 0.0, tr, acc, nc + 1, first);
    }
    store_partials(acc, d.P1, a.npart, nc + 2);
}

// ------------------------------------------------------------------ Lanczos (TTR)

// Plain, v_j stored (src/orthogonal_bases.jl:45-50):
//   U = A v_j - beta_{j-1} v_{j-1};  P1 = [ <U, v_j> ]
__global__ __launch_bounds__(TPB) void k_lan_l1_plain(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    const int j = a.j;
    const double* vj = d.V + (int64_t)j * a.ld;
    const double* vp = d.V + (int64_t)(j > 0 ? j - 1 : 0) * a.ld;
    const double bp = j > 0 ? d.sc[SC_BETAPREV] : 0.0;
    TILE_LOOP
        double u = 0.0, v = 0.0;
        if (ok) {
            const double av = spmv_row(d.rowptr, d.col, d.val, vj, r);
            const double prev = j > 0 ? vp[r] : 0.0;
            u = av - bp * prev;
            v = vj[r];
            d.U[r] = u;
        }
        reduce_one(u * v, tr, acc, 0, first);
    }
    store_partials(acc, d.P1, a.npart, 1);
}

// Fused: pending v_j = (beta == 0 ? 0 : inv(beta) .* W) (src/orthogonal_bases.jl:59) is
// written while  U = A v_j - beta v_{j-1};
//   P1 = [ <U,v_j>, <v_j,b> | gram <V[:,c],v_j> (c<j), <v_j,v_j> ]
__global__ __launch_bounds__(TPB) void k_lan_l1_fused(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    const int j = a.j;
    const double beta = d.sc[SC_BETA];
    const double inv_beta = d.sc[SC_INVBETA];
    const bool zero = (beta == 0.0);
    const double* vp = d.V + (int64_t)(j - 1) * a.ld;
    double* vj_out = d.V + (int64_t)j * a.ld;
    const bool gram = d.track_gram != 0;
    TILE_LOOP
        double u = 0.0, vj = 0.0, bv = 0.0;
        if (ok) {
            vj = zero ? 0.0 : mul_rn(d.W[r], inv_beta);
            const double av = spmv_row_scaled(d.rowptr, d.col, d.val, d.W, inv_beta, zero, r);
            u = av - beta * vp[r];
            vj_out[r] = vj;
            d.U[r] = u;
            bv = d.b[r];
        }
        reduce_one(u * vj, tr, acc, 0, first);
        reduce_one(vj * bv, tr, acc, 1, first);
        if (gram) {
            reduce_cols_stream(d.V, a.ld, r, j, ok, vj, tr, acc, 2, first);
            reduce_one(vj * vj, tr, acc, 2 + j, first);
        }
    }
    if (!gram) zero_acc(acc, 2, 3 + j);
    store_partials(acc, d.P1, a.npart, j + 3);
}

// W = U - alpha v_j (src/orthogonal_bases.jl:53);  P2 = [ <W,W> ]
__global__ __launch_bounds__(TPB) void k_lan_l2(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    const int j = a.j;
    const double alpha = d.RED1[0];
    const double* vj = d.V + (int64_t)j * a.ld;
    TILE_LOOP
        double w = 0.0;
        if (ok) {
            w = d.U[r] - alpha * vj[r];
            d.W[r] = w;
        }
        reduce_one(w * w, tr, acc, 0, first);
    }
    store_partials(acc, d.P2, a.npart, 1);
}

// Write pending column j+1 = (beta == 0 ? 0 : inv(beta) .* W);
//   P1 = [ <v,b> | gram <V[:,c],v> (c<=j), <v,v> ]
__global__ __launch_bounds__(TPB) void k_lan_finalize(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    const int j = a.j, nc = j + 1;
    const double beta = d.sc[SC_BETA];
    const double inv_beta = d.sc[SC_INVBETA];
    const bool zero = (beta == 0.0);
    double* vout = d.V + (int64_t)(j + 1) * a.ld;
    const bool gram = d.track_gram != 0;
    TILE_LOOP
        double v = 0.0, bv = 0.0;
        if (ok) {
            v = zero ? 0.0 : mul_rn(d.W[r], inv_beta);
            vout[r] = v;
            bv = d.b[r];
        }
        reduce_one(v * bv, tr, acc, 0, first);
        if (gram) {
            reduce_cols_stream(d.V, a.ld, r, nc, ok, v, tr, acc, 1, first);
            reduce_one(v * v, tr, acc, 1 + nc, first);
        }
    }
    if (!gram) zero_acc(acc, 1, 2 + nc);
    store_partials(acc, d.P1, a.npart, nc + 2);
}

// ------------------------------------------------------------------ reductions

// RED[c] = sum_b P[c*npart + b]: one wave per value, fixed order.
__global__ __launch_bounds__(64) void k_reduce(const DFac* __restrict__ F, int which, int nv, int npart) {
    const DFac& d = F[blockIdx.y];
    const int c = blockIdx.x;
    if (c >= nv) return;
    const double* P = (which == 1 ? d.P1 : d.P2) + (int64_t)c * npart;
    double s = 0.0;
    for (int b = threadIdx.x; b < npart; b += 64) s += P[b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (threadIdx.x == 0) (which == 1 ? d.RED1 : d.RED2)[c] = s;
}

// ------------------------------------------------------------------ post-processing
// One 64-thread block per factor: turns reduced values into H / beta / records.

__device__ __forceinline__ void put_gram(double* rec, int kmax, int c, const double* row, double bt,
                                         int tracked) {
    if (tracked)
        for (int i = threadIdx.x; i <= c; i += 64) rec[rec_gram(kmax) + i] = row[i];
    if (threadIdx.x == 0) {
        rec[rec_bt(kmax)] = bt;
        rec[rec_col(kmax)] = (double)c;
        rec[rec_tracked(kmax)] = tracked ? 1.0 : 0.0;
    }
}

__global__ __launch_bounds__(64) void k_post(const DFac* __restrict__ F, KArgs a, int kind, int flag) {
    const DFac& d = F[blockIdx.x];
    const int j = a.j, kmax = a.kmax, KP = kmax + 2;
    double* rec = a.rec + (int64_t)d.gidx * a.m;
    const int t = threadIdx.x;
    if (kind == POST_INIT_A) {
        if (t == 0) {
            const double nrm = sqrt(d.RED1[0]);
            d.sc[SC_BNORM] = nrm;
            d.sc[SC_INVB] = 1.0 / nrm;
        }
        return;
    }
    if (kind == POST_INIT_B) {
        put_gram(rec, kmax, 0, d.RED1 + 1, d.RED1[0], d.track_gram);
        return;
    }
    if (kind == POST_ARN) {
        // RED1 = [h1 (j+1) | gram_j (j+1) | bt_j] (gram/bt only when fused), RED2 = [h2 (j+1) | s]
        double* Hc = d.H + (int64_t)j * KP;
        for (int i = t; i <= j; i += 64) {
            Hc[i] = d.RED1[i] + d.RED2[i];
            d.h2[i] = d.RED2[i];
            rec[i] = Hc[i];
        }
        __shared__ double part[64];
        double hh = 0.0;
        for (int i = t; i <= j; i += 64) hh += d.RED2[i] * d.RED2[i];
        part[t] = hh;
        __syncthreads();
        if (t == 0) {
            double s2 = 0.0;
            for (int i = 0; i < 64; ++i) s2 += part[i];
            double bsq = d.RED2[j + 1] - s2;
            const double beta = sqrt(bsq > 0.0 ? bsq : 0.0);
            Hc[j + 1] = beta;
            rec[j + 1] = beta;
            rec[rec_beta(kmax)] = beta;
            d.sc[SC_BETA] = beta;
            d.sc[SC_INVBETA] = 1.0 / beta;
            d.sc[SC_BETAPREV] = beta;
        }
        __syncthreads();
        // g = Hbar[0..j+1, 0..j] * h2  (column i of Hbar has rows 0..i+1)
        for (int l = t; l <= j + 1; l += 64) {
            double s = 0.0;
            for (int i = (l > 0 ? l - 1 : 0); i <= j; ++i) s += d.H[(int64_t)i * KP + l] * d.RED2[i];
            d.g[l] = s;
        }
        if (flag) put_gram(rec, kmax, j, d.RED1 + j + 1, d.RED1[2 * j + 2], d.track_gram);
        else if (t == 0) rec[rec_col(kmax)] = -1.0;
        return;
    }
    if (kind == POST_ARN_FIN) {
        // RED1 = [gram_{j+1} (j+2) | bt]
        put_gram(rec, kmax, j + 1, d.RED1, d.RED1[j + 2], d.track_gram);
        return;
    }
    if (kind == POST_LAN) {
        // RED1 = [alpha | bt_j | gram_j (j+1)] (bt/gram only when fused), RED2 = [|w|^2]
        if (t == 0) {
            const double alpha = d.RED1[0];
            const double beta = sqrt(d.RED2[0]);
            rec[j] = alpha;
            rec[j + 1] = beta;
            rec[rec_beta(kmax)] = beta;
            d.sc[SC_BETA] = beta;
            d.sc[SC_INVBETA] = 1.0 / beta;
            d.sc[SC_BETAPREV] = beta;
        }
        if (flag) put_gram(rec, kmax, j, d.RED1 + 2, d.RED1[1], d.track_gram);
        else if (t == 0) rec[rec_col(kmax)] = -1.0;
        return;
    }
    if (kind == POST_LAN_FIN) {
        // RED1 = [bt | gram_{j+1} (j+2)]
        put_gram(rec, kmax, j + 1, d.RED1 + 1, d.RED1[0], d.track_gram);
        return;
    }
}

// ------------------------------------------------------------------ V * Y on MFMA

typedef double f64x4 __attribute__((ext_vector_type(4)));

// X[:, t0..t0+64) = V[:, 0..k) * Y[:, t0..t0+64) for one factor (blockIdx.y), Y
// column-major k x t.  Each wave computes 16-row strips for up to four 16-column
// tiles with v_mfma_f64_16x16x4_f64:
//   A = V[16 rows x 4 cols]  lane l: row l&15, col l>>4   (coalesced 128 B per column)
//   B = Y[4 x 16]            lane l: row l>>4, col l&15   (from LDS)
//   D                        lane l: row (l>>4) + 4i, col l&15
// k is walked in chunks of 64 staged through LDS.
__global__ __launch_bounds__(256) void k_basis_mul(const DFac* __restrict__ F, KArgs a,
                                                   const double* __restrict__ Yall,
                                                   double* __restrict__ Xall, int k, int t) {
    __shared__ double Ys[64 * 65];   // [col][kk] padded
    const int f = blockIdx.y;
    const DFac& d = F[f];
    const double* Y = Yall + (int64_t)f * k * t;
    double* X = Xall + (int64_t)f * a.ld * t;
    const int t0 = blockIdx.z * 64;
    const int tn = min(64, t - t0);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    f64x4 acc[4][4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[s][q] = (f64x4){0.0, 0.0, 0.0, 0.0};
    const int64_t rb = (int64_t)blockIdx.x * 256 + wave * 64;
    for (int k0 = 0; k0 < k; k0 += 64) {
        const int kn = min(64, k - k0);
        __syncthreads();
        for (int i = threadIdx.x; i < 64 * 64; i += 256) {
            const int kk = i & 63, tt = i >> 6;
            Ys[tt * 65 + kk] = (kk < kn && tt < tn) ? Y[(int64_t)(t0 + tt) * k + k0 + kk] : 0.0;
        }
        __syncthreads();
        const int kp = (kn + 3) & ~3;
        for (int kk = 0; kk < kp; kk += 4) {
            const int ka = kk + lk;
            double b0 = Ys[(0 + lr) * 65 + ka], b1 = Ys[(16 + lr) * 65 + ka];
            double b2 = Ys[(32 + lr) * 65 + ka], b3 = Ys[(48 + lr) * 65 + ka];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int64_t ra = rb + s * 16 + lr;
                const double av = (ra < a.n && ka < kn) ? d.V[ra + (int64_t)(k0 + ka) * a.ld] : 0.0;
                acc[s][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b0, acc[s][0], 0, 0, 0);
                if (tn > 16) acc[s][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b1, acc[s][1], 0, 0, 0);
                if (tn > 32) acc[s][2] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b2, acc[s][2], 0, 0, 0);
                if (tn > 48) acc[s][3] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b3, acc[s][3], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t rr = rb + s * 16 + lk + 4 * i;
            if (rr < a.n) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = q * 16 + lr;
                    if (c < tn) X[rr + (int64_t)(t0 + c) * a.ld] = acc[s][q][i];
                }
            }
        }
    }
}

// ------------------------------------------------------------------ plain SpMV (test hook)
__global__ __launch_bounds__(TPB) void k_spmv(const int* __restrict__ rowptr, const int* __restrict__ col,
                                              const double* __restrict__ val, const double* __restrict__ x,
                                              double* __restrict__ y, int64_t n) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r < n) y[r] = spmv_row(rowptr, col, val, x, r);
}

// ------------------------------------------------------------------ launchers

static size_t acc_bytes(int nv) { return (size_t)((nv + 32 + 15) & ~15) * sizeof(double); }

#define DISPATCH_MAXC(ncols, KERNEL, ...)                  \
    do {                                                   \
        if ((ncols) <= 16)                                 \
            hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__);   \
        else if ((ncols) <= 32)                            \
            hipLaunchKernelGGL(KERNEL<32>, __VA_ARGS__);   \
        else if ((ncols) <= 48)                            \
            hipLaunchKernelGGL(KERNEL<48>, __VA_ARGS__);   \
        else                                               \
            hipLaunchKernelGGL(KERNEL<64>, __VA_ARGS__);   \
    } while (0)

void launch_init_a(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_init_a, dim3(a.npart, nf), dim3(TPB), acc_bytes(1), s, F, a);
}
void launch_init_b(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_init_b, dim3(a.npart, nf), dim3(TPB), acc_bytes(2), s, F, a);
}
void launch_arn_a1_plain(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    DISPATCH_MAXC(a.j + 1, k_arn_a1_plain, dim3(a.npart, nf), dim3(TPB), acc_bytes(a.j + 1), s, F, a);
}
void launch_arn_a1_fused(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    DISPATCH_MAXC(a.j, k_arn_a1_fused, dim3(a.npart, nf), dim3(TPB), acc_bytes(2 * a.j + 3), s, F, a);
}
void launch_arn_a2(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    DISPATCH_MAXC(a.j + 1, k_arn_a2, dim3(a.npart, nf), dim3(TPB), acc_bytes(a.j + 2), s, F, a);
}
void launch_arn_finalize(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    DISPATCH_MAXC(a.j + 1, k_arn_finalize, dim3(a.npart, nf), dim3(TPB), acc_bytes(a.j + 3), s, F, a);
}
void launch_lan_l1_plain(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_lan_l1_plain, dim3(a.npart, nf), dim3(TPB), acc_bytes(1), s, F, a);
}
void launch_lan_l1_fused(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_lan_l1_fused, dim3(a.npart, nf), dim3(TPB), acc_bytes(a.j + 3), s, F, a);
}
void launch_lan_l2(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_lan_l2, dim3(a.npart, nf), dim3(TPB), acc_bytes(1), s, F, a);
}
void launch_lan_finalize(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_lan_finalize, dim3(a.npart, nf), dim3(TPB), acc_bytes(a.j + 3), s, F, a);
}
void launch_reduce(const DFac* F, int nf, int which, int nv, int npart, hipStream_t s) {
    hipLaunchKernelGGL(k_reduce, dim3(nv, nf), dim3(64), 0, s, F, which, nv, npart);
}
void launch_post(const DFac* F, int nf, const KArgs& a, int kind, int flag, hipStream_t s) {
    hipLaunchKernelGGL(k_post, dim3(nf), dim3(64), 0, s, F, a, kind, flag);
}
void launch_basis_mul(const DFac* F, int nf, const KArgs& a, const double* Y, double* X, int k,
                      int t, hipStream_t s) {
    const int nb = (int)((a.n + 255) / 256);
    const int nz = (t + 63) / 64;
    hipLaunchKernelGGL(k_basis_mul, dim3(nb, nf, nz), dim3(256), 0, s, F, a, Y, X, k, t);
}
void launch_spmv(const int* rowptr, const int* col, const double* val, const double* x, double* y,
                 int64_t n, hipStream_t s) {
    const int nb = (int)((n + TPB - 1) / TPB);
    hipLaunchKernelGGL(k_spmv, dim3(nb), dim3(TPB), 0, s, rowptr, col, val, x, y, n);
}

}  // namespace tk
