// tk_kernels.hip -- gfx950 (MI355X) kernels for the inner Krylov iteration of
// thbake/TensorKrylov.jl.
//
// Layout (DESIGN.md "Data layout in HBM"): the basis V_s of every factor is stored
// TILE-MAJOR with PAIRED COLUMNS: rows are cut into 256-row tiles; a tile holds its
// KCP = kmax+1 rounded up to even columns contiguously, as column pairs, element (r, c) at
//   (r/256)*256*KCP + (c/2)*512 + (r%256)*2 + c%2.
// A 256-thread block owns one tile at a time; thread t keeps its row V[r, 0..ncols) in
// VGPRs, loaded two columns per buffer_load_dwordx4 (1 KiB per wave instruction; measured
// 6.0 TB/s vs 5.6 with one column per dwordx2, tools/bwprobe.hip) whose hardware range
// check (num_records = whole column pairs from the tile base) zero-fills the pairs a step
// does not use; the odd column of a half-used pair is cleared in registers.  All
// n-length vectors are padded to whole tiles (zeros).
// The Gram-free one-sweep TensorLanczos (KArgs::sl) keeps the same tiles with SINGLE
// columns instead, element (r, c) at (r/256)*256*KCP + c*256 + r%256: its step reads one
// column and writes one, and a pair layout makes that 48 bytes per row instead of 40 (half
// a pair read for the previous column, the even column's round trip through E).  The
// readers of a whole basis (V*Y, the Gram, the flush) take both layouts.
//
// Numerical scheme (DESIGN.md "Arnoldi step"): the reference's two-pass MGS
// (src/orthogonal_bases.jl:15-37) is computed as CGS2 -- h1 = V'w, w' = w - V h1,
// h2 = V'w', H[:,j] = h1 + h2, beta = sqrt(|w'|^2 - |h2|^2),
// v_{j+1} = (w' - V h2) * inv(beta) -- equal to MGS2 in exact arithmetic and within the
// parity tolerance in floating point (tests/test_gpu_parity.py).  v_{j+1} is not
// written by a pass of its own: the next step's SpMV kernel writes it while it holds
// the same V rows in registers, applying A to w' and subtracting A V h2 = V Hbar h2
// through the Arnoldi relation.  V is streamed twice per step (the compulsory MGS2
// traffic of SURVEY.md section 8d).
//
// Every reduction is fixed-order (LDS transpose + DPP row sums per block, then one
// wave per value over NPART block partials, NPART a function of n only): results are
// bitwise reproducible and independent of how the factors are split over GPUs.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "tk_internal.h"

namespace tk {

#define TPB 256          // threads per block == rows per tile
#define CH 16            // values per block-reduction chunk
#define TSTR (TPB + 16)  // LDS stride (doubles) of the transpose buffer
// Occupancy of the streaming pass kernels (waves per SIMD, by register-row width): the
// compiler's own choice left 40/56-column rows at one wave less than their registers
// allow; these limits are the largest that compile without spills.
#define OCC_WAVES(L4, L3) (MAXC <= (L4) ? 4 : (MAXC <= (L3) ? 3 : 2))
// SpMV-fused kernels: the gather formats need more registers
// (6 = SPM_PRE: no gathers, the register budget of the second pass)
#define A1_L4(F) ((F) == 1 || (F) == 3 || (F) == 4 || (F) == 5 ? 40 : ((F) == 2 ? 24 : ((F) == 6 ? 32 : 16)))
#define A1_L3(F) ((F) == 1 || (F) == 3 || (F) == 4 || (F) == 5 ? 56 : ((F) == 2 ? 40 : ((F) == 6 ? 48 : 32)))
#define OCC_ATTR(L4, L3) __attribute__((amdgpu_waves_per_eu(OCC_WAVES(L4, L3), OCC_WAVES(L4, L3))))
#ifndef TK_A1_SCALAR
#define TK_A1_SCALAR 1
#endif
#ifndef TK_A2_SCALAR
#define TK_A2_SCALAR 0
#endif
#define COEF_TAIL 16     // h2/g hold kmax+2+COEF_TAIL doubles: register rows may read past kmax+1
#define COEF_PAD(kmax) ((kmax) + 2 > 64 ? (kmax) + 2 : 64)   // LDS coefficient array length

typedef __amdgpu_buffer_rsrc_t rsrc_t;
#define GP(T, p) ((__attribute__((address_space(1))) T*)(p))
// constant address space: wave-uniform reads of data no kernel writes while it runs
// (coefficient vectors produced by the previous launch) compile to scalar loads
#define CP4(p) ((const __attribute__((address_space(4))) double*)(p))

// ------------------------------------------------------------------ primitives

__device__ __forceinline__ rsrc_t mkrsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
// V is streamed once per pass and never re-read from cache within a step: non-temporal
// loads (aux = 2, `nt`) measured 3-5 % faster than the default policy (tools/bwprobe.hip).
#ifndef TK_V_AUX
#define TK_V_AUX 2
#endif
__device__ __forceinline__ double bld(rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, TK_V_AUX));
}

typedef double d2_t __attribute__((ext_vector_type(2)));
template <int AUX = TK_V_AUX>
__device__ __forceinline__ d2_t bld2(rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(d2_t, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}
// Paired-column tile layout: element offset of (row t, column c) inside a tile, byte
// offset of column c relative to thread t's pair base (t*16), tile stride, and the
// range-check size that admits columns [0, nc).
__device__ __forceinline__ int64_t vofs(int c, int t) { return ((int64_t)(c >> 1) * TPB + t) * 2 + (c & 1); }
__device__ __forceinline__ uint32_t cofs(int c) { return (uint32_t)(c >> 1) * (TPB * 16) + (uint32_t)(c & 1) * 8; }
__host__ __device__ __forceinline__ int kcp(int kmax) { return (kmax + 2) & ~1; }
__device__ __forceinline__ uint32_t vrange(int nc) { return (uint32_t)((nc + 1) >> 1) * (TPB * 16); }
// single-column tiles (KArgs::sl): element offset of (row t, column c), byte offset of column c
// relative to thread t's base (t*8); vrange covers them too (nc*256*8 <= its pair bytes)
__device__ __forceinline__ int64_t svofs(int c, int t) { return (int64_t)c * TPB + t; }
__device__ __forceinline__ uint32_t sofs(int c) { return (uint32_t)c * (TPB * 8); }

// Julia's CSC scatter adds nz*x into y without FMA; keep products and sums separately
// rounded so the device SpMV equals it bit for bit (__dmul_rn/__dadd_rn are plain
// * and + in ROCm 7.2's headers, so contraction is switched off explicitly).
__device__ __forceinline__ double mul_rn(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b) {
#pragma clang fp contract(off)
    return a + b;
}
__device__ __forceinline__ double sub_rn_(double a, double b) {
#pragma clang fp contract(off)
    return a - b;
}

// DPP row rotate (16-lane rows) of a double.
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
// Sum over each 16-lane row; every lane of the row ends with its row's total.
__device__ __forceinline__ double row16_sum(double s) {
    s += dpp<0x128>(s);   // row_ror:8
    s += dpp<0x124>(s);   // row_ror:4
    s += dpp<0x122>(s);   // row_ror:2
    s += dpp<0x121>(s);   // row_ror:1
    return s;
}
// lane 0's value in every lane (the rotations leave each lane its own rounding of the total)
__device__ __forceinline__ double lane0(double x) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), 0),
                            __builtin_amdgcn_readlane(__double2loint(x), 0));
}
// A one-sweep Arnoldi step's scalars from the previous step's reduced dots (RED1 = c [0,J) |
// q [J,2J) | |u|^2 | <u,z> ..., J <= 64): beta = sqrt(|u|^2 - |c|^2), ib = 1/beta,
// t1 = (<u,z> - c.q) ib (gamma = t1 ib, the coefficient of v_J in u_{J+1}).  One full wave,
// lane l holding c[l], q[l] (zero for l >= J), a fixed-order butterfly and lane 0's sums: every
// caller -- each window block of k_arn_d1 and the step's bookkeeping -- gets the same bits, so
// no block has to hand them to the others (round 5: the reduce is a plain reduction).
__device__ __forceinline__ void d1_scalars(double c0, double q0, double uu, double uz, double& beta, double& ib,
                                           double& t1) {
#pragma clang fp contract(off)
    double cc = c0 * c0, cq = c0 * q0;
    cc = row16_sum(cc);
    cc += __shfl_xor(cc, 16);
    cc += __shfl_xor(cc, 32);
    cq = row16_sum(cq);
    cq += __shfl_xor(cq, 16);
    cq += __shfl_xor(cq, 32);
    cc = lane0(cc);
    cq = lane0(cq);
    const double bsq = uu - cc;
    beta = sqrt(bsq > 0.0 ? bsq : 0.0);
    ib = 1.0 / beta;
    t1 = (uz - cq) * ib;
}

// Reduce-scatter over each 16-lane row: lane l returns the sum over its row's 16 lanes of
// x[l & 15].  Four exchange steps (partners l^8 by row_ror:8, l^7 by row_half_mirror, l^2
// and l^1 by quad_perm); at each a lane keeps the half of its values selected by one
// bit of its index and adds the partner's copy of that half.  Fixed order, no LDS.
__device__ __forceinline__ double rs16(const double (&x)[16]) {
    const int l = threadIdx.x & 15;
    const bool b3 = l & 8, b2 = l & 4, b1 = l & 2, b0 = l & 1;
    double y[8], z[4], w[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) y[i] = (b3 ? x[8 + i] : x[i]) + dpp<0x128>(b3 ? x[i] : x[8 + i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = (b2 ? y[4 + i] : y[i]) + dpp<0x141>(b2 ? y[i] : y[4 + i]);
#pragma unroll
    for (int i = 0; i < 2; ++i) w[i] = (b1 ? z[2 + i] : z[i]) + dpp<0x4E>(b1 ? z[i] : z[2 + i]);
    return (b0 ? w[1] : w[0]) + dpp<0xB1>(b0 ? w[0] : w[1]);
}

// Reduce-scatter over the whole wave: lane l returns the sum over all 64 lanes of
// x[(l >> 2) & 15] (lanes 4v..4v+3 hold value v, bitwise equal).  The two cross-row steps
// are v_permlane32_swap / v_permlane16_swap half exchanges (gfx950): with vdst = the half the
// lower rows keep and src = the half the upper rows keep, one swap per dword leaves every
// lane with its own and its partner's copy of the half it keeps -- no select.  Then
// row_ror:8 and row_half_mirror halve the last four values (as rs16) and two quad_perm
// all-reduce steps finish.  Fixed order; 63 VALU per 16 values against rs16's 105.
__device__ __forceinline__ double swap_add32(double a, double b) {   // lanes < 32: a, else b
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    const double na = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
    const double nb = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
    return na + nb;
}
__device__ __forceinline__ double swap_add16(double a, double b) {   // even rows: a, odd: b
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    const double na = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
    const double nb = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
    return na + nb;
}
// The half exchange itself: vd = (lanes < 32: a, else the partner's b), vs = (lanes < 32:
// the partner's a, else b).
__device__ __forceinline__ void swap32(double a, double b, double& vd, double& vs) {
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    vd = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
    vs = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
}
// rs64 after its first (cross-half) step: y[i] holds value i + 8 [lane >= 32]
__device__ __forceinline__ double rs64_tail(const double (&y)[8]) {
    const int l = threadIdx.x & 15;
    const bool b3 = l & 8, b2 = l & 4;
    double z[4], w[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = swap_add16(y[i], y[4 + i]);   // + 4 [odd row]
#pragma unroll
    for (int i = 0; i < 2; ++i) w[i] = (b3 ? z[2 + i] : z[i]) + dpp<0x128>(b3 ? z[i] : z[2 + i]);
    double s = (b2 ? w[1] : w[0]) + dpp<0x141>(b2 ? w[0] : w[1]);
    s += dpp<0x4E>(s);   // quad_perm [2,3,0,1]
    s += dpp<0xB1>(s);   // quad_perm [1,0,3,2]
    return s;
}
__device__ __forceinline__ double rs64(const double (&x)[16]) {
    const int l = threadIdx.x & 15;
    const bool b3 = l & 8, b2 = l & 4;
    double y[8], z[4], w[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) y[i] = swap_add32(x[i], x[8 + i]);   // value i + 8 [lane >= 32]
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = swap_add16(y[i], y[4 + i]);   // + 4 [odd row]
#pragma unroll
    for (int i = 0; i < 2; ++i) w[i] = (b3 ? z[2 + i] : z[i]) + dpp<0x128>(b3 ? z[i] : z[2 + i]);
    double s = (b2 ? w[1] : w[0]) + dpp<0x141>(b2 ? w[0] : w[1]);
    s += dpp<0x4E>(s);   // quad_perm [2,3,0,1]
    s += dpp<0xB1>(s);   // quad_perm [1,0,3,2]
    return s;
}

// Accumulate CH per-thread values x[0..CH) over the block's 256 rows into
// acc[base .. base+CH) (LDS).  Fixed order: lane (col*16+part) sums rows q*16+part of
// column col (q ascending), then a DPP row sum.
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
    s = row16_sum(s);
    if (part == 0) acc[base + col] = first ? s : acc[base + col] + s;
    __syncthreads();
}

// Row of V held in VGPRs: v[c] = V[r, c] for c < MAXC, zero for c >= nc (pairs beyond
// the resource's range read as zero; the odd half of the last pair is cleared here).
// `last` = V[r, nc-1], the newest column, picked while loading (a second load of it would
// miss the cache: V loads are non-temporal).
template <int MAXC>
struct Row {
    static_assert(MAXC % 2 == 0, "register rows hold whole column pairs");
    double v[MAXC];
    double last;
    __device__ __forceinline__ void load(rsrc_t tile, uint32_t toff, int nc) {
        last = 0.0;
#pragma unroll
        for (int p = 0; p < MAXC / 2; ++p) {
            const d2_t x = bld2(tile, toff + (uint32_t)p * (TPB * 16));
            v[2 * p] = x.x;
            v[2 * p + 1] = 2 * p + 1 < nc ? x.y : 0.0;
            last = 2 * p == nc - 1 ? x.x : (2 * p + 1 == nc - 1 ? x.y : last);
        }
        if (nc > MAXC) last = bld(tile, toff + cofs(nc - 1));
    }
    // single-column tiles (toff = t*8): columns past nc get an offset beyond the resource
    __device__ __forceinline__ void load_sl(rsrc_t tile, uint32_t toff, int nc) {
#pragma unroll
        for (int c = 0; c < MAXC; ++c) v[c] = bld(tile, c < nc ? toff + sofs(c) : 0x80000000u);
        last = nc <= MAXC ? 0.0 : bld(tile, toff + sofs(nc - 1));
#pragma unroll
        for (int c = 0; c < MAXC; ++c) last = c == nc - 1 ? v[c] : last;
    }
    // Column c (MAXC - 8 <= c < MAXC, or MAXC == 8; wave-uniform; loaded as zero) := x, and
    // `last` := x.  Masked adds, not a conditional store: that one the compiler merged into
    // a dynamically indexed store and moved the whole row to scratch.
    __device__ __forceinline__ void set_col(int c, double x) {
        constexpr int C0 = MAXC > 8 ? MAXC - 8 : 0;
        const uint64_t xb = __builtin_bit_cast(uint64_t, x);
#pragma unroll
        for (int q = C0; q < MAXC; ++q)
            v[q] += __builtin_bit_cast(double, xb & (0ull - (uint64_t)(q == c)));
        last = x;
    }
    // Same as load through a resource over the factor's whole basis (rows of two tiles in
    // one wave): pairs past nc get an offset beyond the resource, like rows outside the
    // basis (toff >= 2^31): every such load returns zero.  The caller sizes the row to the
    // step (MAXC - 8 <= nc <= MAXC, or MAXC == 8): only the last four pairs need the uniform
    // column checks, and `last` is one of their columns.
    // loadm for an even nc: whole pairs only, no selects on the loaded values (a uniform
    // select there made the compiler wait for the row before its next loads); `last` unset
    // AUX: the load's cache policy (k_arn_d1: nt, or the default policy while the rank's
    // per-step working set fits the Infinity Cache)
    template <int PLO = 0, int AUX = TK_V_AUX>   // pairs below PLO are not loaded (k_arn_d1 keeps them in LDS)
    __device__ __forceinline__ void loadm_even(rsrc_t basis, uint32_t toff, int nc) {
        constexpr int P0 = MAXC / 2 - 4;
#pragma unroll
        for (int p = PLO; p < MAXC / 2; ++p) {
            const uint32_t off = (p < P0 || 2 * p < nc) ? toff + (uint32_t)p * (TPB * 16) : 0x80000000u;
            const d2_t x = bld2<AUX>(basis, off);
            v[2 * p] = x.x;
            v[2 * p + 1] = x.y;
        }
    }
    __device__ __forceinline__ void loadm(rsrc_t basis, uint32_t toff, int nc) {
        constexpr int P0 = MAXC / 2 - 4;
        last = 0.0;
#pragma unroll
        for (int p = 0; p < MAXC / 2; ++p) {
            // pairs past nc: an offset beyond the resource (the load returns zero, no branch --
            // a branch around the load made the compiler wait for every load at its join)
            const uint32_t off = (p < P0 || 2 * p < nc) ? toff + (uint32_t)p * (TPB * 16) : 0x80000000u;
            const d2_t x = bld2(basis, off);
            v[2 * p] = x.x;
            v[2 * p + 1] = (p < P0 || 2 * p + 1 < nc) ? x.y : 0.0;
            if (p >= P0) last = 2 * p == nc - 1 ? x.x : (2 * p + 1 == nc - 1 ? x.y : last);
        }
    }
};

// Store V[r, c] as a whole 16-byte column pair (`other` = the pair's other column): a lone
// 8-byte store would leave half-written 32-byte sectors behind.
__device__ __forceinline__ void st_pair(double* V, int64_t tile_base, int c, int t, double v, double other) {
    const d2_t x = (c & 1) ? (d2_t){other, v} : (d2_t){v, other};
    GP(d2_t, V + tile_base + vofs(c & ~1, t))[0] = x;
}

// The one-sweep Arnoldi step's outputs -- u, v_j, the window partials -- are read by the next
// launches, not by this one: stored write-through (sc1), they leave no dirty lines in the XCD
// L2s for the kernel boundary's writeback to drain (a boundary costs ~1.7 us + dirty bytes /
// 6 TB/s, /opt/skills/guides/MI355X_MICROARCH.md "boundary"; plain stores keep the line dirty
// in L2, sc1 stores drop it, "stores of each flavour").  Measured (profiles/r03/wt_ab.txt):
// k_arn_d1 at one factor per GPU 2 us faster per step, neutral at 8 factors; k_lan_1w's
// 8-byte stores 10 % slower write-through, so it keeps plain stores.  TK_WT=0: plain.
#ifndef TK_WT
#define TK_WT 1
#endif
// k_reduce256's hand-off of the reduced values to the block that evaluates the next step's
// scalars: 0 = agent-scope relaxed atomics with the store's completion awaited before the
// arrival add (measured correct on gfx950), 1 = a release/acquire add + acquire fence (the
// HIP memory model's own guarantee)
#ifndef TK_RED_MM
#define TK_RED_MM 0
#endif
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_wt(double* p, int64_t i, double v) {
#if TK_WT
    __hip_atomic_store(GP(double, p) + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    GP(double, p)[i] = v;
#endif
}
// column pair (c & ~1, c | 1) of the row at byte offset toff of the basis resource
__device__ __forceinline__ void st_pair_wt(rsrc_t basis, uint32_t toff, int c, double v, double other) {
    const d2_t x = (c & 1) ? (d2_t){other, v} : (d2_t){v, other};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, x), basis, toff + (uint32_t)(c >> 1) * (TPB * 16), 0,
                                           TK_WT ? 16 : 0);
}

// sum_c V[r,c] * h[c] for c < nc.  SCALAR: h is a global coefficient array read with
// wave-uniform addresses through the constant address space (scalar loads, many in
// flight); otherwise h is an LDS copy (broadcast reads).  Entries past nc are finite
// (zeroed at init or earlier coefficients) and meet R.v[c] == 0.
// Two accumulators (even / odd columns, summed at the end) halve the dependent FMA chain;
// the split depends on the column index only, so any register-row width gives the same
// value (the zero columns past nc add exact zeros).
template <int MAXC, bool SCALAR>
__device__ __forceinline__ double row_dot(const Row<MAXC>& R, rsrc_t tile, uint32_t toff, int nc,
                                          const double* __restrict__ h) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int c = 0; c < MAXC; c += 2) {
        s0 += R.v[c] * (SCALAR ? CP4(h)[c] : h[c]);
        s1 += R.v[c + 1] * (SCALAR ? CP4(h)[c + 1] : h[c + 1]);
    }
    for (int c = MAXC; c < nc; ++c) {
        const double x = bld(tile, toff + cofs(c)) * (SCALAR ? CP4(h)[c] : h[c]);
        if (c & 1) s1 += x;
        else s0 += x;
    }
    return s0 + s1;
}
// Two row dots at once (four independent chains), each bitwise equal to row_dot.
template <int MAXC>
__device__ __forceinline__ void row_dot2(const Row<MAXC>& R, const double* __restrict__ h,
                                         const double* __restrict__ g, double& sh, double& sg) {
    double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
    uint64_t ph = (uint64_t)h, pg = (uint64_t)g;
#pragma unroll
    for (int c0 = 0; c0 < MAXC; c0 += 8) {
        // the next 8 coefficients of each vector are loaded (scalar) only after the
        // previous ones were used: bounded SGPR live range, no spills
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" : "+s"(ph), "+s"(pg) : "v"(a0), "v"(b0));
        const double* hh = (const double*)ph;
        const double* gg = (const double*)pg;
#pragma unroll
        for (int c = c0; c < c0 + 8; c += 2) {
            a0 += R.v[c] * CP4(hh)[c];
            a1 += R.v[c + 1] * CP4(hh)[c + 1];
            b0 += R.v[c] * CP4(gg)[c];
            b1 += R.v[c + 1] * CP4(gg)[c + 1];
        }
    }
    sh = a0 + a1;
    sg = b0 + b1;
}
// Same, with the coefficients in lanes (lane l holds h[l], g[l]; l < 64 covers MAXC), read
// column by column with v_readlane into SGPRs: the fused launch's coefficients, produced
// inside the same launch, come through sc1 vector loads instead of the scalar cache.
template <int MAXC>
__device__ __forceinline__ void row_dot2_rl(const Row<MAXC>& R, double hl, double gl, double& sh, double& sg) {
    static_assert(MAXC <= 64, "one coefficient per lane");
    double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
    const int hlo = __double2loint(hl), hhi = __double2hiint(hl), glo = __double2loint(gl), ghi = __double2hiint(gl);
#pragma unroll
    for (int c = 0; c < MAXC; c += 2) {
        const double h0 = __hiloint2double(__builtin_amdgcn_readlane(hhi, c), __builtin_amdgcn_readlane(hlo, c));
        const double h1 = __hiloint2double(__builtin_amdgcn_readlane(hhi, c + 1), __builtin_amdgcn_readlane(hlo, c + 1));
        const double g0 = __hiloint2double(__builtin_amdgcn_readlane(ghi, c), __builtin_amdgcn_readlane(glo, c));
        const double g1 = __hiloint2double(__builtin_amdgcn_readlane(ghi, c + 1), __builtin_amdgcn_readlane(glo, c + 1));
        a0 += R.v[c] * h0;
        a1 += R.v[c + 1] * h1;
        b0 += R.v[c] * g0;
        b1 += R.v[c + 1] * g1;
    }
    sh = a0 + a1;
    sg = b0 + b1;
}
// an agent-scope (sc1) load: another CU's in-launch store drained to the device level is seen
__device__ __forceinline__ double ld_ag(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Fused one-sweep launch: one lane polls the factor's step word (sc1 loads, s_sleep between)
// until the in-launch reducers publish `want`; the block's waves pass a barrier after it.
// Bounded: after `spin` polls (2^22) the context's error word is set -- every host call that
// hands results out after a sync then returns TK_ERR_INTERNAL -- and the block goes on: a
// result would be wrong, but nothing hangs.
// mm (the memory-model hand-off, red_mm()): the reducers' last block stores the word with
// release; every wave then takes an agent-scope acquire fence after the barrier, so the
// values it loads next are ordered after the word (a relaxed poll that reads a release store,
// then an acquire fence, synchronizes with it).  Without mm the measured relaxed form: sc1
// stores drained before the word, sc1 loads after it.
__device__ __forceinline__ void fuse_wait(const unsigned long long* word, unsigned long long want, unsigned int* err,
                                          unsigned spin, int mm) {
    if (threadIdx.x == 0) {
        unsigned spins = 0;
        while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
            if (++spins > spin) {
                if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    if (mm) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}
// Same with both coefficient vectors staged in LDS (broadcast ds_read_b128), same order;
// coefficient reads in groups of GRP columns (register pressure).
template <int MAXC, int GRP = 8>
__device__ __forceinline__ void row_dot2_lds(const Row<MAXC>& R, const double* __restrict__ h,
                                             const double* __restrict__ g, double& sh, double& sg) {
    double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
#pragma unroll
    for (int c0 = 0; c0 < MAXC; c0 += GRP) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = c0; c < c0 + GRP; c += 2) {
            const d2_t hv = *(const d2_t*)(h + c);
            const d2_t gv = *(const d2_t*)(g + c);
            a0 += R.v[c] * hv.x;
            a1 += R.v[c + 1] * hv.y;
            b0 += R.v[c] * gv.x;
            b1 += R.v[c + 1] * gv.y;
        }
    }
    sh = a0 + a1;
    sg = b0 + b1;
}

// Block-reduce V[r,i]*y for i < lim (lim == the row's loaded column count, so R.v[i]
// is zero beyond it) into acc[base .. base+lim).  Entries up to base+roundup16(lim)
// receive zeros (callers reduce extra scalars into them afterwards).  MAXC need not be a
// multiple of CH: the rest of the last register chunk is streamed (range-checked zeros).
template <int MAXC>
__device__ __forceinline__ void reduce_row(const Row<MAXC>& R, rsrc_t tile, uint32_t toff, int lim,
                                           double y, double* tr, double* acc, int base, bool first) {
    constexpr int MR = (MAXC + CH - 1) / CH * CH;
#pragma unroll
    for (int c0 = 0; c0 < MR; c0 += CH) {
        if (c0 < lim) {
            double x[CH];
#pragma unroll
            for (int q = 0; q < CH; ++q)
                x[q] = (c0 + q < MAXC ? R.v[c0 + q < MAXC ? c0 + q : 0]
                                      : (c0 + q < lim ? bld(tile, toff + cofs(c0 + q)) : 0.0)) * y;
            chunk_reduce(x, tr, acc, base + c0, first);
        }
    }
    for (int c0 = MR; c0 < lim; c0 += CH) {
        double x[CH];
#pragma unroll
        for (int q = 0; q < CH; q += 2) {
            const d2_t p = bld2(tile, toff + cofs(c0 + q));
            x[q] = (c0 + q < lim ? p.x : 0.0) * y;
            x[q + 1] = (c0 + q + 1 < lim ? p.y : 0.0) * y;
        }
        chunk_reduce(x, tr, acc, base + c0, first);
    }
}

// Same without a register row (streams V[r, 0..lim) from the tile; the tile resource
// must admit the pairs of exactly lim columns).
__device__ __forceinline__ void reduce_stream(rsrc_t tile, uint32_t toff, int lim, double y, double* tr,
                                              double* acc, int base, bool first) {
    for (int c0 = 0; c0 < lim; c0 += CH) {
        double x[CH];
#pragma unroll
        for (int q = 0; q < CH; q += 2) {
            const d2_t p = bld2(tile, toff + cofs(c0 + q));
            x[q] = p.x * y;
            x[q + 1] = (c0 + q + 1 < lim ? p.y : 0.0) * y;
        }
        chunk_reduce(x, tr, acc, base + c0, first);
    }
}

// Block-reduce NE per-thread scalars into acc[base .. base+NE): DPP row sums, then the
// 16 row totals of each value summed in fixed order by one thread.
template <int NE>
__device__ __forceinline__ void reduce_scalars(const double* e, double* tr, double* acc, int base,
                                               bool first) {
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const double s = row16_sum(e[k]);
        if ((t & 15) == 0) tr[k * 16 + (t >> 4)] = s;
    }
    __syncthreads();
    if (t < NE) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) s += tr[t * 16 + q];
        acc[base + t] = first ? s : acc[base + t] + s;
    }
    __syncthreads();
}

// Block partials -> global [value][npart]
__device__ __forceinline__ void store_partials(const double* acc, double* P, int npart, int nv) {
    __syncthreads();
    for (int c = threadIdx.x; c < nv; c += TPB) GP(double, P)[(int64_t)c * npart + blockIdx.x] = acc[c];
}


// Copy nc coefficients from global to LDS, zero-padded to `pad` entries (caller syncs).
__device__ __forceinline__ void stage(double* dst, const double* src, int nc, int pad) {
    const int m = nc > pad ? nc : pad;
    for (int c = threadIdx.x; c < m; c += TPB) dst[c] = c < nc ? GP(const double, src)[c] : 0.0;
}

__device__ __forceinline__ double ld(const double* p, int64_t i) { return GP(const double, p)[i]; }
__device__ __forceinline__ void st(double* p, int64_t i, double v) { GP(double, p)[i] = v; }
// X_s = V_s Y_s (written once, read by the host copy-out): streaming stores
#ifndef TK_X_NT
#define TK_X_NT 1
#endif
__device__ __forceinline__ void st_x(double* p, int64_t i, double v) {
#if TK_X_NT
    __builtin_nontemporal_store(v, &GP(double, p)[i]);
#else
    GP(double, p)[i] = v;
#endif
}

// y[r] = sum over row r of A, terms in ascending column order, products and sums
// separately rounded (Julia's CSC scatter order).  x(c) supplies the vector entry.
// FMT: SPM_DIA / SPM_SELL / SPM_CSR fixes the storage at compile time (fewer live
// registers in the fused kernels); SPM_ANY decides at run time.
enum { SPM_ANY = 0, SPM_DIA = 1, SPM_SELL = 2, SPM_CSR = 3, SPM_DIAN = 4, SPM_DIAT = 5,
       SPM_PRE = 6 };   // SPM_PRE: CGS2 pass 1 reads A U from DFac::AU (k_spmv_mf ran), no SpMV
template <int FMT, class XF>
__device__ __forceinline__ double spmv(const SpM& A, int64_t r, XF x) {
#pragma clang fp contract(off)
    double s = 0.0;
    if (FMT == SPM_DIA || FMT == SPM_DIAT) {
        // at most 4 diagonals (the gallery's tridiagonal / convection-diffusion bands); the
        // device arrays hold at least 4 rows (zero padding, offset 0), so every load is
        // issued up front from clamped indices and the terms are then summed in order --
        // one memory round trip instead of one per diagonal.
        double vv[4], xx[4];
        bool in[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q < 3 || q < A.ndiag) {
                const int64_t c = r + GP(const int, A.doff)[q];
                in[q] = q < A.ndiag && c >= 0 && c < A.n;
                const int64_t cc = c < 0 ? 0 : (c >= A.n ? A.n - 1 : c);
                vv[q] = FMT == SPM_DIAT ? CP4(A.dconst)[q] : ld(A.dval, (int64_t)q * A.dld + r);
                xx[q] = x(cc);
            } else {
                in[q] = false;
                vv[q] = xx[q] = 0.0;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (in[q]) s = add_rn(s, mul_rn(vv[q], xx[q]));
    } else if (FMT == SPM_DIAN || (FMT == SPM_ANY && A.ndiag > 0)) {
        for (int q = 0; q < A.ndiag; ++q) {
            const int64_t c = r + GP(const int, A.doff)[q];
            const double v = ld(A.dval, (int64_t)q * A.dld + r);
            if (c >= 0 && c < A.n) s = add_rn(s, mul_rn(v, x(c)));
        }
    } else if (FMT == SPM_SELL || (FMT == SPM_ANY && A.sell)) {
        const int64_t t = r >> 8;
        const int l = (int)(r & 255);
        const int64_t base = GP(const long long, A.sptr)[t];
        const int w = GP(const int, A.swidth)[t];
        const int len = GP(const int, A.rowlen)[r];
        for (int q = 0; q < w; ++q) {
            const int64_t e = base + (int64_t)q * TPB + l;
            if (q < len) s = add_rn(s, mul_rn(ld(A.sval, e), x((int64_t)GP(const int, A.scol)[e])));
        }
    } else {
        const int p0 = GP(const int, A.rowptr)[r], p1 = GP(const int, A.rowptr)[r + 1];
        for (int p = p0; p < p1; ++p) s = add_rn(s, mul_rn(ld(A.val, p), x((int64_t)GP(const int, A.col)[p])));
    }
    return s;
}


// Shared prologue: descriptor, LDS, tile loop.  Rows r >= n are padding (all inputs
// zero there); `ok` guards only the SpMV and the stored scalars.
#define KERNEL_PROLOGUE                                                \
    __shared__ double tr[CH * TSTR];                                   \
    extern __shared__ __attribute__((aligned(16))) double lds[];       \
    const DFac& d = F[blockIdx.y];                                     \
    if (a.gate && ld(d.sc, SC_REDO) == 0.0) return;                    \
    const int64_t TS = (int64_t)TPB * kcp(a.kmax);                     \
    (void)TS;

#define TILE_LOOP                                                                  \
    bool first = true;                                                             \
    for (int tile = blockIdx.x; tile < a.ntiles; tile += a.npart, first = false) { \
        const int64_t r = (int64_t)tile * TPB + threadIdx.x;                       \
        const bool ok = r < a.n;                                                   \
        const double* Vt = d.V + (int64_t)tile * TS;                               \
        const uint32_t toff = threadIdx.x * 16u;                                   \
        (void)Vt; (void)toff; (void)ok;

// ------------------------------------------------------------------ init kernels

// P1 = [ sum b^2 ]
__global__ __launch_bounds__(TPB) void k_init_a(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    double* acc = lds;
    TILE_LOOP
        const double bv = ld(d.b, r);
        const double e[1] = {bv * bv};
        reduce_scalars<1>(e, tr, acc, 0, first);
    }
    store_partials(acc, d.P1, a.npart, 1);
}

// V[:,0] = inv(norm(b)) .* b  (src/decompositions.jl:112-118);  P1 = [<v0,b>, <v0,v0>]
__global__ __launch_bounds__(TPB) void k_init_b(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    double* acc = lds;
    const double inv = ld(d.sc, SC_INVB);
    TILE_LOOP
        const double bv = ld(d.b, r);
        const double v0 = inv * bv;
        st_pair(d.V, (int64_t)tile * TS, 0, threadIdx.x, v0, 0.0);   // column 1 not yet written
        if (d.Uint) st(d.U, r, v0);   // (shared A_s: step 0's A v0 from k_spmv_mf, which reads U)
        const double e[2] = {v0 * bv, v0 * v0};
        reduce_scalars<2>(e, tr, acc, 0, first);
    }
    store_partials(acc, d.P1, a.npart, 2);
}

// ------------------------------------------------------------------ one A_s, many factors
// The CGS2 first pass of factors sharing one A_s (the C3 gallery: five factors, one random
// sparse matrix) is bound by its random gathers of U: ~15 distinct cache lines per row per
// factor move from L2 to L1 for 8 useful bytes each.  With the factors' U rows interleaved
// (Uint[r][f], k_ilv) one gather per nonzero fetches the entries of
// every factor, and k_spmv_mf writes each factor's A U with the same products and sums in the
// same order as its own SpMV would (bitwise the same), which pass 1 then reads as one more
// streamed vector.  F[0] carries the group's Uint (all factors' descriptors point to it).
// Uint rows are padded to ilv_pitch(nf) doubles (a power of two: one aligned 16..64-byte
// piece per row, read as 16-byte loads).
__host__ __device__ inline int ilv_pitch(int nf) { return nf <= 2 ? 2 : (nf <= 4 ? 4 : 8); }
// One 256-row tile per block (ld_ is a multiple of 256): the factors' entries are transposed
// through LDS so every wave store writes 1 KiB of contiguous Uint (row-strided 16-byte
// stores left each line to be completed by four separate instructions; k_arn_a2 storing each
// factor's 8-byte piece of every row cost that pass 10-50 %, one block walking all factors of
// a tile cost it more)
__global__ __launch_bounds__(TPB) void k_ilv(const DFac* __restrict__ F, int nf, int64_t ld_) {
    __shared__ double tl[TPB * 9];   // row pitch 9: the transposing writes are conflict-free
    const int64_t r0 = (int64_t)blockIdx.x * TPB;
    const int t = threadIdx.x;
    double* Ui = F[0].Uint;
    const int p = ilv_pitch(nf);
    double u[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) u[f] = f < nf ? ld(F[f < nf ? f : 0].U, r0 + t) : 0.0;
#pragma unroll
    for (int f = 0; f < 8; ++f)
        if (f < p) tl[t * 9 + f] = u[f];
    __syncthreads();
    const int nch = TPB * p / 2;   // 16-byte pieces of the tile's Uint rows
    auto* out = GP(d2_t, Ui + r0 * p);
    for (int c = t; c < nch; c += TPB) {
        const int e = 2 * c, row = e / p, col = e - row * p;
        out[c] = (d2_t){tl[row * 9 + col], tl[row * 9 + col + 1]};
    }
}
// Four lanes per row (tools/gatherprobe.hip: one thread per row with three 16-byte gathers
// per nonzero ran at 0.88 of the pattern's random-gather ceiling, four lanes at 0.98): lane p
// of a row's quad gathers piece p (16 bytes, factors 2p and 2p+1) of the row's Uint entry, so a
// wave instruction touches 16 rows' 64-byte pieces instead of 64 rows' -- and sums its two
// factors in the row's order (ascending column, products and sums rounded apart: bitwise the
// per-factor SpMV).  64 rows per 256-thread block.
template <int FMT, int NFM>
__global__ __launch_bounds__(TPB) void k_spmv_mf(const DFac* __restrict__ F, int nf, KArgs a) {
#pragma clang fp contract(off)
    constexpr int NP = NFM <= 2 ? 2 : (NFM <= 4 ? 4 : 8);   // = ilv_pitch(NFM)
    constexpr int NQ = (NFM + 1) / 2;                        // lanes of a quad with factors
    const int p = threadIdx.x & 3;
    const int64_t r = (int64_t)blockIdx.x * (TPB / 4) + (threadIdx.x >> 2);
    if (r >= a.ld) return;
    const DFac& d0 = F[0];
    const double* Ui = d0.Uint;
    double s0 = 0.0, s1 = 0.0;
    if (r < a.n && p < NQ) {
        auto acc = [&](double v, int64_t c) {
            const d2_t x = GP(const d2_t, Ui + c * NP)[p];
            s0 = add_rn(s0, mul_rn(v, x.x));
            s1 = add_rn(s1, mul_rn(v, x.y));
        };
        const SpM& A = d0.A;
        if (FMT == SPM_SELL) {
            const int64_t t = r >> 8;
            const int l = (int)(r & 255);
            const int64_t base = GP(const long long, A.sptr)[t];
            const int w = GP(const int, A.swidth)[t];
            const int len = GP(const int, A.rowlen)[r];
            // slots in groups of SG: their indices and values, then their gathers, in flight
            // together before the products are summed in order
            constexpr int SG = 4;
            for (int q0 = 0; q0 < w; q0 += SG) {
                int64_t cc[SG];
                double vv[SG];
#pragma unroll
                for (int g = 0; g < SG; ++g) {
                    const int64_t e = base + (int64_t)(q0 + g) * TPB + l;
                    const bool in = q0 + g < len;
                    cc[g] = in ? (int64_t)GP(const int, A.scol)[e] : -1;
                    vv[g] = in ? ld(A.sval, e) : 0.0;
                }
                d2_t x[SG];
#pragma unroll
                for (int g = 0; g < SG; ++g)
                    x[g] = cc[g] >= 0 ? GP(const d2_t, Ui + cc[g] * NP)[p] : (d2_t){0.0, 0.0};
#pragma unroll
                for (int g = 0; g < SG; ++g)
                    if (cc[g] >= 0) {
                        s0 = add_rn(s0, mul_rn(vv[g], x[g].x));
                        s1 = add_rn(s1, mul_rn(vv[g], x[g].y));
                    }
            }
        } else {
            const int p0 = GP(const int, A.rowptr)[r], p1 = GP(const int, A.rowptr)[r + 1];
            for (int q = p0; q < p1; ++q) acc(ld(A.val, q), (int64_t)GP(const int, A.col)[q]);
        }
    }
    if (p < NQ) {
        st(F[2 * p].AU, r, s0);
        if (2 * p + 1 < NFM) st(F[2 * p + 1 < NFM ? 2 * p + 1 : 0].AU, r, s1);
    }
}

// ------------------------------------------------------------------ Arnoldi (CGS2)

// First pass, v_j stored:  W = A v_j;  P1 = [ <V[:,c], W>, c = 0..j ].
template <int MAXC, int FMT>
__global__ __launch_bounds__(TPB) OCC_ATTR(A1_L4(FMT), A1_L3(FMT)) void k_arn_a1_plain(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    double* acc = lds;
    const int j = a.j, nc = j + 1;
    TILE_LOOP
        const rsrc_t tv = mkrsrc(Vt, vrange(nc));
        Row<MAXC> R;
        R.load(tv, toff, nc);
        const double* Vg = d.V;
        double w = 0.0;
        if constexpr (FMT == SPM_PRE) w = ok ? ld(d.AU, r) : 0.0;   // (A v_j from k_spmv_mf)
        else w = ok ? spmv<FMT>(d.A, r, [=](int64_t c) { return ld(Vg, (c >> 8) * TS + vofs(j, (int)(c & 255))); }) : 0.0;
        st(d.W, r, w);
        reduce_row<MAXC>(R, tv, toff, nc, w, tr, acc, 0, first);
    }
    store_partials(acc, d.P1, a.npart, nc);
}

// First pass of step j fused with writing the pending column v_j of step j-1:
//   v_j = (U - V[:,0..j) h2) * inv_beta                     -> V[:, j]
//   W   = (A U - V[:,0..j) g[0..j) - g[j] v_j) * inv_beta    (= A v_j, Arnoldi relation)
//   P1  = [ <V[:,c],W> (c<j), <v_j,W> ]
template <int MAXC, int FMT>
__global__ __launch_bounds__(TPB) OCC_ATTR(A1_L4(FMT), A1_L3(FMT)) void k_arn_a1_fused(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    const int j = a.j;
    constexpr bool SC = TK_A1_SCALAR;
    const int CP = COEF_PAD(a.kmax);
    const double* h2 = d.h2;
    const double* g = d.g;            // g[j] read separately
    double* acc = lds + (SC ? 0 : 2 * CP);
    if (!SC) {
        stage(lds, d.h2, j, CP);
        stage(lds + CP, d.g, j, CP);
        __syncthreads();
        h2 = lds;
        g = lds + CP;
    }
    const double inv_beta = ld(d.sc, SC_INVBETA);
    const double gj = ld(d.g, j);
    TILE_LOOP
        const rsrc_t tv = mkrsrc(Vt, vrange(j));
        Row<MAXC> R;
        R.load(tv, toff, j);
        const double* Ug = d.U;
        double au = 0.0;
        if constexpr (FMT == SPM_PRE) au = ok ? ld(d.AU, r) : 0.0;
        else au = ok ? spmv<FMT>(d.A, r, [=](int64_t c) { return ld(Ug, c); }) : 0.0;
        const double up = ld(d.U, r);
        const double vj = ok ? (up - row_dot<MAXC, SC>(R, tv, toff, j, h2)) * inv_beta : 0.0;
        const double w = ok ? (au - row_dot<MAXC, SC>(R, tv, toff, j, g) - gj * vj) * inv_beta : 0.0;
        st_pair(d.V, (int64_t)tile * TS, j, threadIdx.x, vj, (j & 1) ? R.last : 0.0);
        st(d.W, r, w);
        reduce_row<MAXC>(R, tv, toff, j, w, tr, acc, 0, first);
        const double e1[1] = {vj * w};
        reduce_scalars<1>(e1, tr, acc, j, first);
    }
    store_partials(acc, d.P1, a.npart, j + 1);
}

// Second pass: U = W - V[:,0..j] h1, plus update_rhs! and the Gram row of column j
// (both need only V[r, 0..j], already in registers):
//   P2 = [ <V[:,c],U> (c<=j), <U,U>, <v_j,b> | gram <V[:,c],v_j> (c<=j) ]
template <int MAXC>
__global__ __launch_bounds__(TPB) OCC_ATTR(32, 48) void k_arn_a2(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    const int j = a.j, nc = j + 1;
    constexpr bool SC = TK_A2_SCALAR;
    const int CP = COEF_PAD(a.kmax);
    const double* h1 = d.RED1;
    double* acc = lds + (SC ? 0 : CP);
    if (!SC) {
        stage(lds, d.RED1, nc, CP);
        __syncthreads();
        h1 = lds;
    }
    const bool gram = d.track_gram != 0;
    TILE_LOOP
        const rsrc_t tv = mkrsrc(Vt, vrange(nc));
        Row<MAXC> R;
        R.load(tv, toff, nc);
        const double vj = R.last;
        const double w = ld(d.W, r);
        const double u = ok ? (w - row_dot<MAXC, SC>(R, tv, toff, nc, h1)) : 0.0;
        st(d.U, r, u);
        reduce_row<MAXC>(R, tv, toff, nc, u, tr, acc, 0, first);
        const double e[2] = {u * u, vj * ld(d.b, r)};
        reduce_scalars<2>(e, tr, acc, nc, first);
        if (gram) reduce_row<MAXC>(R, tv, toff, nc, vj, tr, acc, nc + 2, first);
    }
    store_partials(acc, d.P2, a.npart, gram ? 2 * nc + 2 : nc + 2);
}

// Write the pending column j+1 with no following step (U or W per a.ubuf: W after an
// even one-sweep step):
//   v = (U - V[:,0..j] h2) * inv_beta;  P1 = [ gram <V[:,c],v> (c<=j), <v,v>, <v,b> ]
template <int MAXC>
__global__ __launch_bounds__(TPB) OCC_ATTR(32, 48) void k_arn_finalize(const DFac* __restrict__ F, KArgs a) {
    KERNEL_PROLOGUE
    const int j = a.j, nc = j + 1;
    constexpr bool SC = TK_A2_SCALAR;
    const int CP = COEF_PAD(a.kmax);
    const double* h2 = d.h2;
    double* acc = lds + (SC ? 0 : CP);
    if (!SC) {
        stage(lds, d.h2, nc, CP);
        __syncthreads();
        h2 = lds;
    }
    const double inv_beta = ld(d.sc, SC_INVBETA);
    TILE_LOOP
        const rsrc_t tv = mkrsrc(Vt, vrange(nc));
        Row<MAXC> R;
        R.load(tv, toff, nc);
        const double up = ld(a.ubuf ? d.W : d.U, r);
        const double v = ok ? (up - row_dot<MAXC, SC>(R, tv, toff, nc, h2)) * inv_beta : 0.0;
        st_pair(d.V, (int64_t)tile * TS, j + 1, threadIdx.x, v, ((j + 1) & 1) ? R.last : 0.0);
        reduce_row<MAXC>(R, tv, toff, nc, v, tr, acc, 0, first);
        const double e[2] = {v * v, v * ld(d.b, r)};
        reduce_scalars<2>(e, tr, acc, nc, first);
    }
    store_partials(acc, d.P1, a.npart, nc + 2);
}

// ------------------------------------------------------------------ Arnoldi, one sweep per step
// CGS2 with the reorthogonalization delayed by one step: step j
// streams V[:, 0..j) ONCE.  Entering step j the device holds the raw vector u_j (once
// orthogonalized, in U or W), its reorthogonalization coefficients c = h2[0..j) and
// inv_beta, and h1 = g[0..j] (projection of A v_j on V[:, 0..j]).  Per row:
//   v_j     = (u_j - V[:,0..j) c) * inv_beta                      -> V[:, j]
//   u_{j+1} = A v_j - V[:,0..j) h1[0..j) - h1[j] v_j               -> the other buffer
//   z       = A u_{j+1}
//   P1 = [ <V[:,c],u> (c<j) | <V[:,c],z> (c<j) | <v_j,u>, <v_j,z>, <u,u>, <u,z>, <v_j,v_0>,
//          <v_j,v_j> | gram <V[:,c],v_j> (c<j) ]       (<v_j,b> = norm(b) <v_j,v_0> in the post)
// Both SpMVs read their vector from LDS, so each block works on an overlapping window of
// 256 rows and owns the middle 256 - 2(hl+hu) of them: v_j is valid on the whole window,
// u on all but hl/hu rows at its edges, z on all but 2hl/2hu -- the owned rows.  Halo rows
// are recomputed from the same data in the same order as by their owner, so every block
// sees bitwise the owner's values.  Only banded storage (hl, hu <= 4) takes this path.
__device__ __forceinline__ int clamp_row(int64_t i) { return i < 0 ? 0 : (i >= TPB ? TPB - 1 : (int)i); }


// fused flush + V*Y (k_fin_vy): 4 waves per SIMD up to this register-row width (56 spills to
// scratch at 4), Y coefficient reads from LDS in groups of this many columns
#ifndef TK_VY_OCC4
#define TK_VY_OCC4 48
#endif
#ifndef TK_VY_GRP
#define TK_VY_GRP 8
#endif
// occupancy by register-row width (measured at C2: 4 waves/SIMD up to 32 columns, 3 up
// to 56; 40 columns at 4 waves spill)
#ifndef TK_D1_L4
#define TK_D1_L4 40
#endif
#ifndef TK_D1_L3
#define TK_D1_L3 56
#endif
// Column dots: each wave reduce-scatters its products over all 64 lanes (rs64; the 16 values
// of a chunk land in 4 lanes) and every fourth lane adds its result into a private LDS slot --
// no barrier; the slots are combined once, at the end.  Chunk k < NUZ holds columns
// 8k..8k+7 times (u, z) interleaved, chunk NUZ the six scalars, chunks NUZ+1.. the Gram row
// (16 columns each).  acc[chunk][64]: slot = (wave p, value s).
#define D1_ACC_Y(k, y)                                                                  \
    do {                                                                                \
        const double r_ = rs64_tail(y);                                                 \
        if ((t & 3) == 0) acc[(k) * 64 + (t >> 6) * 16 + ((t >> 2) & 15)] += r_;        \
    } while (0)
#define D1_ACC(k, x)                                                                    \
    do {                                                                                \
        const double r_ = rs64(x);                                                      \
        if ((t & 3) == 0) acc[(k) * 64 + (t >> 6) * 16 + ((t >> 2) & 15)] += r_;        \
    } while (0)
#define D1_NP 4
#define D1_CHW 64
#define D1_PART(k, p, sl) acc[(k) * 64 + (p) * 16 + (sl)]
#if TK_D1_TRACE
// diagnostic builds only (tools/build_variant.sh NAME - -DTK_D1_TRACE=1, tools/d1_trace.py):
// per-block start / end wall clock (100 MHz) and HW_ID / XCC_ID of one step's k_arn_d1
// launch, factor 0
#define TRACE_MAX 8192
__device__ int g_trace_j = -1;
__device__ uint64_t g_trace[3 * TRACE_MAX];
__device__ uint64_t g_trace_ph[4 * TRACE_MAX];   // phase clocks (loads done, SpMV 1, SpMV 2, dots)
#define D1_PHASE(k)                                                                   \
    do {                                                                              \
        __builtin_amdgcn_s_waitcnt(0);                                                \
        if (t == 0 && d.gidx == 0 && j == g_trace_j && slot < TRACE_MAX)          \
            g_trace_ph[4 * slot + (k)] = __builtin_amdgcn_s_memrealtime();            \
    } while (0)
#else
#define D1_PHASE(k) do { } while (0)
#endif
__device__ void bk_arn_d(const DFac& d, const KArgs& a, double* rec, double* lds);
template <bool MM, bool FUSED>
__device__ __forceinline__ void red256_block(const DFac& d, int fidx, int c, int which, int nv, int np, int coefJ,
                                             const KArgs& ax, unsigned long long wseq);
__device__ void post_signal(const KArgs& a, const DFac& d, int fidx, bool mirrored, bool coherent = false);
// narrow rows leave registers for more waves: the tiers rs64's register count allows (one
// more wave per SIMD spills: -30..-45 %)
#define D1_OCC (MAXC <= 8 ? 8 : (MAXC <= 16 ? 6 : (MAXC <= 24 ? 5 : (MAXC <= TK_D1_L4 ? 4 : (MAXC <= TK_D1_L3 ? 3 : 2)))))
template <int MAXC, int FMT, int MODE>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(D1_OCC, D1_OCC))) void k_arn_d1(const DFac* __restrict__ F, KArgs a,
                                                                                                  KArgs b) {
    constexpr int NUZ = MAXC / 8, NG = (MAXC + 15) / 16;
    // MODE bit 0 (VC): the basis rows through the caches (the launcher's choice while the rank's
    // per-step working set fits the Infinity Cache), else nt.  Bit 1 (FUSE): the previous step's
    // reduce runs in this launch's leading blocks (a.red) -- the window blocks issue their row
    // loads, wait for the factor's step word, and read the coefficients the reducers produced in
    // this launch through sc1 vector loads; partials alternate between P1 / P1b by step parity
    constexpr bool VC = MODE & 1, FUSE = (MODE & 2) != 0;
    // Bit 2 (WSC, one stream only): the previous step's reduce was a plain reduction -- wave 0
    // evaluates the step's scalars (d1_scalars) and hands them to the block through LDS
    constexpr bool WSC = (MODE & 4) != 0 && !FUSE;
    __shared__ double xs[2][TPB];                      // u_j, u_{j+1}
    __shared__ double d1s[2];                          // the step's ib, gamma (wave 0 -> the block; WSC)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const DFac& d = F[blockIdx.y];
    // XCD-aware slot: workgroups are dispatched round-robin over the 8 XCDs, so block x runs
    // on XCD x % 8 (gridDim.x is a multiple of 8); each XCD takes a contiguous range of
    // windows -- neighbouring windows share halo rows in its L2 and its partial stores
    // fill whole lines there
    // With the previous step's bookkeeping (b.j >= 0) the grid has 8 leading blocks (one per
    // XCD, so the windows keep their XCD mapping); those of the first factor row run it for
    // factors x, x+8, .. -- dispatched first, they finish while the windows stream (as
    // trailing blocks they lengthened short launches by their own duration) -- and the window
    // blocks do not wait for them.
    // fused: XR leading reducer blocks (row 0; value c of factor f at x = f * NVR + c), then the
    // bookkeeping blocks, then the windows -- every block a window waits for is dispatched first
    const int NVR = (FUSE && a.red) ? 3 * a.j + 3 : 0;
    const int XR = (FUSE && a.red) ? (((int)gridDim.y * NVR + 7) & ~7) : 0;
    if (FUSE && (int)blockIdx.x < XR) {
        const int f = (int)blockIdx.x / NVR, c = (int)blockIdx.x - f * NVR;
        if (blockIdx.y == 0 && f < (int)gridDim.y) {
            // step j-1's reduce (k_reduce256's block; its last block evaluates this step's scalars)
            const int jp = a.j - 1;
            // (a.red implies j >= 1: red256_block's one-sweep Lanczos branch, coefJ == RED_LAN, is
            // then dead code -- without this the compiler kept it, and its 20 B/lane of scratch
            // memory made every fused instantiation a scratch-using kernel)
            __builtin_assume(jp >= 0);
            if (a.redmm) red256_block<true, true>(F[f], f, c, (jp & 1) ? 5 : 1, 3 * jp + 6, 0, jp + 1, a, a.wseq);
            else red256_block<false, true>(F[f], f, c, (jp & 1) ? 5 : 1, 3 * jp + 6, 0, jp + 1, a, a.wseq);
        }
        return;
    }
    const int x0 = XR + (b.j >= 0 ? 8 : 0);
    if ((int)blockIdx.x < x0) {
        if (blockIdx.y == 0)
            for (int f = (int)blockIdx.x - XR; f < (int)gridDim.y; f += 8) {
                const DFac& df = F[f];
                if (FUSE && a.red) fuse_wait(df.rword, a.wseq, a.werr, a.wspin, a.redmm);
                bk_arn_d(df, b, b.rec + (int64_t)df.gidx * b.m, lds);
                post_signal(b, df, f, true, true);
                __syncthreads();
            }
        return;
    }
    const int bx = (int)blockIdx.x - x0;
    const int slot = (bx & 7) * (((int)gridDim.x - x0) >> 3) + (bx >> 3);
    if (slot >= d.nwin) return;
#if TK_D1_TRACE
    const uint64_t trace_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int64_t TS = (int64_t)TPB * kcp(a.kmax);
    // dynamic LDS: the column-dot slots
    double* acc = lds;
    const int j = a.j, t = threadIdx.x;
    const int hl = d.hl, hu = d.hu, WS = TPB - 2 * (hl + hu);
    const double* Uin = a.ubuf ? d.W : d.U;
    double* Uout = a.ubuf ? d.U : d.W;
    // coefficients from the previous step's reduced dots (no post kernel in between):
    // c = RED1[0, j), q = RED1[j, 2j), scalars after them (k_reduce256)
    const double* c = d.RED1;
    const double* qv = d.RED1 + j;
    const rsrc_t tv = mkrsrc(d.V, (uint32_t)(a.ntiles * TS * 8));
    const bool gram = d.track_gram != 0;
    const int nch = NUZ + 1 + (gram ? NG : 0);
    for (int e = t; e < nch * D1_CHW; e += TPB) acc[e] = 0.0;   // private slots
    // KArgs::pgrp: the window's reduced values by value index, stored as whole groups at the end
    __shared__ double pv[D1G * ((3 * 64 + 6 + D1G - 1) / D1G)];
    const bool pg = !FUSE && a.pgrp;
    const int nvp = pg ? d1_groups(d1_nv(j + 1, gram)) * D1G : 0;
    for (int e = t; e < nvp; e += TPB) pv[e] = 0.0;
    // one window per block (no window loop: nothing loop-invariant to hoist)
    {
        const int w = slot;
        const int64_t S = (int64_t)w * WS - 2 * hl;
        const int64_t r = S + t;
        const bool inb = r >= 0 && r < a.ld;
        const bool ok = r >= 0 && r < a.n;
        const uint32_t toff = inb ? (uint32_t)((r >> 8) * TS * 8 + (r & 255) * 16) : 0x80000000u;
        Row<MAXC> R;
        // odd j: column j-1 was written to E by the previous step (the pair (j-1, j) is stored
        // once, below), so the row loads the complete pairs of columns 0..j-2 and takes
        // column j-1 from E
        int jl = j & ~1;   // the per-pair conditions are re-derived each window (hoisted: SGPR spills)
        asm volatile("" : "+s"(jl));
        // VC: the basis row through the caches (default policy) -- the launcher's choice when
        // this rank's per-step working set fits the 256 MiB Infinity Cache, so the next step
        // re-reads it from there; nt otherwise (streamed once, never re-read in time)
        // the step's scalars come from the previous step's reduced dots (RED1 = [c (j) | q (j) |
        // |u|^2, <u,z>, ..]): lane l loads c[l], q[l] ahead of the row (vmcnt lets these land
        // first) and every wave evaluates them (d1_scalars); step 0 reads the init's
        const int l = t & 63;
        double cl0 = 0.0, ql0 = 0.0;
        double* xv = xs[0];
        double* xu = xs[1];
        // u_j (and column j-1 from E) first, then the basis row: A u_j needs only u_j, so the
        // first SpMV (its barrier and LDS reads) runs while the row's loads are in flight, and
        // the row is waited for at the projections row . c, row . q that follow (round 6, same
        // box: C2 +1..3 %, C4 N = 8 rank 0 +8 %, rank 7 +3..8 %; profiles/r06/early_spmv_ab.txt)
        const double up = inb ? ld(Uin, r) : 0.0;
        const double e = (inb && (j & 1)) ? ld(d.E, r) : 0.0;
        if constexpr (!FUSE) {
            // (wave 0 evaluates them for the block and hands them on through LDS at the barrier
            // before the SpMV, the first place that needs them: one 1 KB load per block)
            if (WSC && j > 0 && t < 64 && l < j) {
                cl0 = ld(d.RED1, l);
                ql0 = ld(d.RED1, j + l);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        R.template loadm_even<0, VC ? 0 : 2>(tv, toff, jl);
        __builtin_amdgcn_sched_barrier(0);
        // (step 0: ib, gamma of the init, k_post; with factor groups the reduce's last block
        // stored them after the values)
        const double* s1 = d.RED1 + (j > 0 ? 3 * j + 3 : 2);
        double inv_beta, gamma;
        double sc, sq;
        if constexpr (!FUSE) {
            if (WSC && j > 0 && t < 64) {
                double beta, ib, t1;
                d1_scalars(cl0, ql0, CP4(d.RED1)[2 * j], CP4(d.RED1)[2 * j + 1], beta, ib, t1);
                if (t == 0) {
                    d1s[0] = ib;
                    d1s[1] = t1 * ib;
                }
            }
        }
        xv[t] = up;
        __syncthreads();
        const double au = ok ? spmv<FMT>(d.A, r, [&](int64_t cc) { return xv[clamp_row(cc - S)]; }) : 0.0;
        if (j & 1) R.set_col(j - 1, e);
        if constexpr (FUSE) {
            // (the row loads above are in flight while the reducers of this launch finish)
            if (a.red) fuse_wait(d.rword, a.wseq, a.werr, a.wspin, a.redmm);
            // lane l holds c[l] and q[l]; row_dot2_rl broadcasts them column by column (the same
            // values and FMA order as the scalar-cache form: bitwise the same sums)
            const double hl = ld_ag(d.RED1 + l), gl = ld_ag(d.RED1 + j + l);
            if (j > 0) {
                double beta, t1;
                d1_scalars(l < j ? hl : 0.0, l < j ? gl : 0.0, ld_ag(d.RED1 + 2 * j), ld_ag(d.RED1 + 2 * j + 1), beta,
                           inv_beta, t1);
                gamma = t1 * inv_beta;
            } else {
                inv_beta = ld_ag(s1 + D1S_IB);
                gamma = ld_ag(s1 + D1S_GAMMA);
            }
            row_dot2_rl<MAXC>(R, hl, gl, sc, sq);
        } else {
            if (WSC && j > 0) {
                inv_beta = d1s[0];
                gamma = d1s[1];
            } else {
                inv_beta = CP4(s1)[D1S_IB];
                gamma = CP4(s1)[D1S_GAMMA];
            }
            row_dot2<MAXC>(R, c, qv, sc, sq);
        }
        D1_PHASE(0);
        // v_j = (u_j - V c) ib.  With h1 = V'A v_j = (q - Hbar c) ib (CGS's first projection;
        // q = V'A u_j from the previous sweep) and A v_j = (A u_j - A V c) ib, the Arnoldi
        // relation A V c = V Hbar c turns CGS's
        //   u_{j+1} = A v_j - V h1[0..j) - h1[j] v_j   into   ib (A u_j - V q) - gamma v_j
        // (the Hbar c terms cancel): the SpMV is applied to u_j itself, no Hbar is needed
        const double vj = ok ? (up - sc) * inv_beta : 0.0;
        const double u = ok ? inv_beta * (au - sq) - gamma * vj : 0.0;
        D1_PHASE(1);
        xu[t] = u;
        __syncthreads();
        const double z = ok ? spmv<FMT>(d.A, r, [&](int64_t cc) { return xu[clamp_row(cc - S)]; }) : 0.0;
        D1_PHASE(2);
        const bool own = ok && t >= 2 * hl && t < TPB - 2 * hu;
        if (own) {
            if (j & 1) st_pair_wt(tv, toff, j, vj, R.last);   // (v_{j-1}, v_j)
            else st_wt(d.E, r, vj);
            st_wt(Uout, r, u);
        }
        const double uo = own ? u : 0.0, zo = own ? z : 0.0, vo = own ? vj : 0.0;
        // update_rhs!'s <v_j, b> as norm(b) * <v_j, v_0> (b = norm(b) v_0, src/decompositions.jl:
        // 112-118): v_0 is column 0 of the register row, so b is not read (-8 B per row)
#define D1_V0R (j > 0 ? R.v[0] : vj)   // (read where used)
        // rs64's first step on the inputs: the basis entries of columns c and c+4 are
        // half-exchanged once for the u, the z and the Gram products, and each lane forms its
        // half's two-lane sums as one product and one FMA (the partner's u, z, v come from one
        // exchange per window).  Gram chunk g takes the pairs of column chunks 2g and 2g+1.
        double mu1, mu2, mz1, mz2, mv1 = 0.0, mv2 = 0.0;
        swap32(uo, uo, mu1, mu2);
        swap32(zo, zo, mz1, mz2);
        if (gram) swap32(vo, vo, mv1, mv2);
#pragma unroll
        for (int g = 0; g < (NUZ + 1) / 2; ++g) {
            double yg[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = 2 * g + h;
                if (k < NUZ && 8 * k < j) {
                    double y[8], c8[8];
#pragma unroll
                    for (int i = 0; i < 8; i += 2) {
                        c8[i] = R.v[8 * k + i < MAXC ? 8 * k + i : 0];
                        c8[i + 1] = R.v[8 * k + i + 1 < MAXC ? 8 * k + i + 1 : 0];
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        double vd, vs;
                        swap32(c8[q], c8[4 + q], vd, vs);
                        y[2 * q] = fma(vs, mu2, vd * mu1);
                        y[2 * q + 1] = fma(vs, mz2, vd * mz1);
                        yg[4 * h + q] = fma(vs, mv2, vd * mv1);   // 0 unless gram (mv = 0)
                    }
                    D1_ACC_Y(k, y);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) yg[4 * h + q] = 0.0;
                }
            }
            if (gram && 16 * g < j) D1_ACC_Y(NUZ + 1 + g, yg);
        }
        {
            // the six scalars in value slots 0..2 (lower half-wave) and 8..10 (upper): three
            // cross-half exchanges, the rest of the first step is zeros
            const double v0r = D1_V0R;
            double y[8] = {swap_add32(vo * u, uo * z), swap_add32(vo * z, vo * v0r), swap_add32(uo * u, vo * vj)};
            D1_ACC_Y(NUZ, y);
        }
    }
    // combine the row-group partials of every value (fixed order) -> P1, in the layout the
    // next step reads its coefficients from (k_reduce256's last block, bk_arn_d)
    //   [ c = p (c<=j) | q (c<=j) | |u|^2, <u,z>, <v_j,v_0>, gram_jj | gram (c<j) ]
    D1_PHASE(3);
    __syncthreads();
    for (int e = t; e < nch * 16; e += TPB) {
        const int k = e >> 4, sl = e & 15;
        double sum = 0.0;
#pragma unroll
        for (int p = 0; p < D1_NP; ++p) sum += D1_PART(k, p, sl);
        int vi = -1;
        if (k < NUZ) {
            const int col = 8 * k + (sl >> 1);
            if (col < j) vi = (sl & 1) ? j + 1 + col : col;
        } else if (k == NUZ) {
            if ((sl & 7) < 3) vi = sl == 0 ? j : 2 * j + (sl < 8 ? sl : sl - 5);   // slots 0,1,2 | 8,9,10
        } else {
            // slot sl of Gram chunk g: pair q = sl & 3 of column chunk 2g + bit 2, upper
            // column (+4) for bit 3
            const int col = 16 * (k - NUZ - 1) + (sl & 3) + 8 * ((sl >> 2) & 1) + 4 * ((sl >> 3) & 1);
            if (col < j) vi = 2 * j + 6 + col;
        }
        if (vi >= 0) {
            if (pg) pv[vi] = sum;
            else st_wt((FUSE && (j & 1)) ? d.P1b : d.P1, (int64_t)vi * d.npd + slot, sum);
        }
    }
    if (pg) {
        // window-major groups of D1G values (tk_internal.h): each group one whole 128-byte line
        // from 16 lanes of one store instruction.  Value-major partials (one 8-byte write per value
        // and window, each its own transaction) cost ~10 % of the step's memory time in the traffic
        // probe (profiles/r06/d1probe_store_variants.txt); whole lines recover most of it, for a
        // heavier reduce (red_d1_block) -- where it is hidden: factor groups over long grids
        __syncthreads();
        for (int e = t; e < nvp; e += TPB) st_wt(d.P1, ((int64_t)(e / D1G) * d.npd + slot) * D1G + (e % D1G), pv[e]);
    }
#if TK_D1_TRACE
    __syncthreads();
    if (t == 0 && d.gidx == 0 && j == g_trace_j && slot < TRACE_MAX) {
        g_trace[3 * slot] = trace_t0;
        g_trace[3 * slot + 1] = __builtin_amdgcn_s_memrealtime();
        g_trace[3 * slot + 2] = ((uint64_t)__builtin_amdgcn_s_getreg(63508) << 32) | __builtin_amdgcn_s_getreg(63492);
    }
#endif
}

// ------------------------------------------------------------------ Lanczos, one sweep per step
// TTR (src/orthogonal_bases.jl:39-67) with the orthogonalization against v_j delayed into the
// next step: step j enters with u_{j-1} = A v_{j-1} - beta_{j-2} v_{j-2} (U or W) and the
// previous reduce's alpha_{j-1}, inv(beta_{j-1}), beta_{j-1} (DFac::sc), and per row
//   w   = u_{j-1} - alpha_{j-1} v_{j-1}              (:53)
//   v_j = inv(beta_{j-1}) .* w                        (:59; zero when beta == 0)   -> E / V
//   u_j = A v_j - beta_{j-1} v_{j-1}                  (:45-47)                     -> other buffer
//   P1  = [ <u_j,v_j>, |u_j|^2, |v_j|^2, <v_j,b> | gram <V[:,c],v_j> (c<j, tracked factor) ]
// The reduce's last block then takes alpha_j = <u_j,v_j> (:50) and
// beta_j = ||u_j - alpha_j v_j|| = sqrt(|u|^2 - 2 alpha^2 + alpha^2 |v|^2) (:56) and writes the
// step's record.  One banded SpMV from LDS (window halo as k_arn_d1); the basis row is loaded
// only for the factor that tracks the Gram row.  Products and sums separately rounded like the
// reference's broadcasts.  Columns written once (even j -> E, odd j -> the pair).
// (launched when some factor of the launch keeps a Gram row; otherwise k_lan_1w below)
template <int MAXC, int FMT>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(D1_OCC, D1_OCC))) void k_lan_1s(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    constexpr int NG = (MAXC + 15) / 16;
    __shared__ double xv[TPB];
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const DFac& d = F[blockIdx.y];
    const int slot = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
    if (slot >= d.nwin) return;
    const int64_t TS = (int64_t)TPB * kcp(a.kmax);
    double* acc = lds;   // [1 + NG chunks][64]: 4 wave slots per value
    const int j = a.j, t = threadIdx.x;
    const int hl = d.hl, hu = d.hu, WS = TPB - 2 * (hl + hu);
    const double* Uin = a.ubuf ? d.W : d.U;
    double* Uout = a.ubuf ? d.U : d.W;
    const double alpha = ld(d.sc, SC_ALPHA), ib = ld(d.sc, SC_INVBETA), betap = ld(d.sc, SC_BETAPREV);
    const rsrc_t tv = mkrsrc(d.V, (uint32_t)(a.ntiles * TS * 8));
    const bool gram = d.track_gram != 0;
    const int nch = 1 + (gram ? NG : 0);
    for (int k = t; k < nch * 64; k += TPB) acc[k] = 0.0;
    const int64_t S = (int64_t)slot * WS - 2 * hl;
    const int64_t r = S + t;
    const bool inb = r >= 0 && r < a.ld;
    const bool ok = r >= 0 && r < a.n;
    const uint32_t toff = inb ? (uint32_t)((r >> 8) * TS * 8 + (r & 255) * 16) : 0x80000000u;
    Row<MAXC> R;
    int jl = j & ~1;
    asm volatile("" : "+s"(jl));
    if (gram) R.loadm_even(tv, toff, jl);
    const double up = inb ? ld(Uin, r) : 0.0;
    // v_{j-1}: E after an even step, the odd half of its pair otherwise
    const double vp = j == 0 ? 0.0 : ((j & 1) ? (inb ? ld(d.E, r) : 0.0) : bld(tv, toff + cofs(j - 1)));
    const double bv = ok ? ld(d.b, r) : 0.0;
    if (gram && (j & 1)) R.set_col(j - 1, vp);
    const double w = sub_rn_(up, mul_rn(alpha, vp));
    const double vj = ok ? mul_rn(ib, w) : 0.0;
    xv[t] = vj;
    __syncthreads();
    const double av = ok ? spmv<FMT>(d.A, r, [&](int64_t cc) { return xv[clamp_row(cc - S)]; }) : 0.0;
    const double u = ok ? sub_rn_(av, mul_rn(betap, vp)) : 0.0;
    const bool own = ok && t >= 2 * hl && t < TPB - 2 * hu;
    if (own) {
        if (j & 1) st_pair(d.V, (r >> 8) * TS, j, (int)(r & 255), vj, vp);
        else st(d.E, r, vj);
        st(Uout, r, u);
    }
    const double uo = own ? u : 0.0, vo = own ? vj : 0.0;
    {
        // beta_j = ||u - alpha_j v_j|| is taken from dots of wt = u - alpha_{j-1} v_j (alpha_{j-1}
        // estimates alpha_j): ||wt + (alpha_{j-1} - alpha_j) v_j||^2 expands without the
        // |u|^2 - alpha^2 cancellation that loses eps (alpha/beta)^2 relative when |alpha| >> beta
        const double wt = own ? u - alpha * vj : 0.0;
        double x[16] = {uo * vj, uo * u, vo * vj, vo * bv, wt * wt, wt * vj};
        D1_ACC(0, x);
    }
    if (gram) {
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            if (16 * k < j) {
                double x[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) x[i] = R.v[16 * k + i < MAXC ? 16 * k + i : 0] * (16 * k + i < MAXC ? vo : 0.0);
                D1_ACC(1 + k, x);
            }
        }
    }
    __syncthreads();
    // combine the 4 wave slots of every value -> P1 [ 4 scalars | gram (c<j) ]
    for (int e = t; e < nch * 16; e += TPB) {
        const int k = e >> 4, sl = e & 15;
        double sum = 0.0;
#pragma unroll
        for (int p = 0; p < D1_NP; ++p) sum += D1_PART(k, p, sl);
        int vi = -1;
        if (k == 0) {
            if (sl < 6) vi = sl;
        } else {
            const int col = 16 * (k - 1) + sl;
            if (col < j) vi = 6 + col;
        }
        if (vi >= 0) st(d.P1, (int64_t)vi * d.npd + slot, sum);
    }
}

// The same step when no factor of the launch keeps a Gram row (the deferred Gram): the
// kernel moves 40-48 bytes per row and nothing else, so a 256-row block would be all
// latency (load, barrier, SpMV, store, reduce for 11 KB).  Each thread takes LAN_RPT rows
// of a window of LAN_RPT * 256 (loads of all its rows in flight together), the window owns
// all but its hl + hu edge rows (one SpMV: v_j is computed pointwise on every row of the
// window, u = A v_j - beta v_{j-1} is valid on the owned rows), and the block's dots are
// summed per thread over its rows in row order, then reduce-scattered like k_lan_1s.
// P1 = [ <u,v_j>, |u|^2, |v_j|^2, <v_j,b>, |wt|^2, <wt,v_j> ] at stride DFac::nwl.  (The
// reduce stays a launch of its own: ending the step in the factor's last block to arrive
// took ~1000 same-address agent atomics per factor and measured 10 us slower per step.)
// SL: single-column tiles -- v_{j-1} is read from its own column and v_j written to its own
// (40 bytes per row: u, v_{j-1}, b in; v_j, u out); otherwise an even v_j goes to E and the
// odd step after it stores the pair.
template <int FMT, bool SL>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_lan_1w(const DFac* __restrict__ F, KArgs a,
                                                                                          KArgs b) {
#pragma clang fp contract(off)
    constexpr int RW = LAN_RPT * TPB;
    __shared__ double xv[RW];
    extern __shared__ __attribute__((aligned(16))) double lds[];
    // b.j >= 0: 8 leading blocks (one per XCD; dispatched first, done while the windows
    // stream) mirror the previous step's record rows to the host and signal them
    const int x0 = b.j >= 0 ? 8 : 0;
    if ((int)blockIdx.x < x0) {
        if (blockIdx.y == 0)
            for (int f = blockIdx.x; f < (int)gridDim.y; f += 8) post_signal(b, F[f], f, false);
        return;
    }
    const DFac& d = F[blockIdx.y];
    const int bx = (int)blockIdx.x - x0;   // (x0 is a multiple of 8: the XCD of bx is kept)
    const int slot = (bx & 7) * (((int)gridDim.x - x0) >> 3) + (bx >> 3);
    if (slot >= d.nwl) return;
    const int64_t TS = (int64_t)TPB * kcp(a.kmax);
    double* acc = lds;   // [64]: 4 wave slots per value
    const int j = a.j, t = threadIdx.x;
    const int hl = d.hl, hu = d.hu;
    const double* Uin = a.ubuf ? d.W : d.U;
    double* Uout = a.ubuf ? d.U : d.W;
    const double alpha = ld(d.sc, SC_ALPHA), ib = ld(d.sc, SC_INVBETA), betap = ld(d.sc, SC_BETAPREV);
    const rsrc_t tv = mkrsrc(d.V, (uint32_t)(a.ntiles * TS * 8));
    if (t < 64) acc[t] = 0.0;
    const int64_t S = (int64_t)slot * (RW - hl - hu) - hl;
    double up[LAN_RPT], vp[LAN_RPT], bv[LAN_RPT];
#pragma unroll
    for (int i = 0; i < LAN_RPT; ++i) {
        const int64_t r = S + i * TPB + t;
        const bool inb = r >= 0 && r < a.ld;
        const bool ok = r >= 0 && r < a.n;
        const uint32_t toff = inb ? (uint32_t)((r >> 8) * TS * 8 + (r & 255) * (SL ? 8 : 16)) : 0x80000000u;
        up[i] = inb ? ld(Uin, r) : 0.0;
        // v_{j-1}: its own column (SL); E after an even step, the odd half of its pair otherwise
        if (SL) vp[i] = j == 0 ? 0.0 : bld(tv, toff + sofs(j - 1));
        else vp[i] = j == 0 ? 0.0 : ((j & 1) ? (inb ? ld(d.E, r) : 0.0) : bld(tv, toff + cofs(j - 1)));
        bv[i] = ok ? ld(d.b, r) : 0.0;
    }
    double vj[LAN_RPT];
#pragma unroll
    for (int i = 0; i < LAN_RPT; ++i) {
        const int64_t r = S + i * TPB + t;
        const bool ok = r >= 0 && r < a.n;
        const double w = sub_rn_(up[i], mul_rn(alpha, vp[i]));
        vj[i] = ok ? mul_rn(ib, w) : 0.0;
        xv[i * TPB + t] = vj[i];
    }
    __syncthreads();
    double x[16] = {0.0};
#pragma unroll
    for (int i = 0; i < LAN_RPT; ++i) {
        const int w = i * TPB + t;
        const int64_t r = S + w;
        const bool ok = r >= 0 && r < a.n;
        const bool own = ok && w >= hl && w < RW - hu;
        const double av = own ? spmv<FMT>(d.A, r, [&](int64_t cc) {
            const int64_t q = cc - S;
            return xv[q < 0 ? 0 : (q >= RW ? RW - 1 : (int)q)];
        }) : 0.0;
        const double u = own ? sub_rn_(av, mul_rn(betap, vp[i])) : 0.0;
        if (own) {
            if (SL) st(d.V, (r >> 8) * TS + svofs(j, (int)(r & 255)), vj[i]);
            else if (j & 1) st_pair(d.V, (r >> 8) * TS, j, (int)(r & 255), vj[i], vp[i]);
            else st(d.E, r, vj[i]);
            st(Uout, r, u);
        }
        const double vo = own ? vj[i] : 0.0;
        // beta_j from dots of wt = u - alpha_{j-1} v_j (see k_lan_1s)
        const double wt = own ? u - alpha * vo : 0.0;
        x[0] += u * vo;
        x[1] += u * u;
        x[2] += vo * vo;
        x[3] += vo * bv[i];
        x[4] += wt * wt;
        x[5] += wt * vo;
    }
    D1_ACC(0, x);   // (acc was zeroed before the barrier above)
    __syncthreads();
    if (t < 6) {
        double sum = 0.0;
#pragma unroll
        for (int p = 0; p < D1_NP; ++p) sum += D1_PART(0, p, t);
        st(d.P1, (int64_t)t * d.nwl + slot, sum);
    }
}

// Initialization for the one-sweep Arnoldi: V[:,0] = U = inv(norm(b)) .* b
// (src/decompositions.jl:112-118) and the first projection of A v_0 (v_0 is known at
// every row from b, so the SpMV needs no halo):
//   P1 = [ <v0,b>, <v0,v0>, <v0, A v0> ]
template <int FMT>
__global__ __launch_bounds__(TPB) void k_init_bd(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    if ((int)blockIdx.x >= d.npd) return;
    double* acc = lds;
    const double inv = ld(d.sc, SC_INVB);
    if (threadIdx.x < 3) acc[threadIdx.x] = 0.0;   // npd may exceed the tile count
    __syncthreads();
    bool first = false;
    const int nt = (int)(a.ld / TPB);
    for (int tile = blockIdx.x; tile < nt; tile += d.npd, first = false) {
        const int64_t r = (int64_t)tile * TPB + threadIdx.x;
        const bool ok = r < a.n;
        const double bv = ld(d.b, r);
        const double v0 = inv * bv;
        const double* bg = d.b;
        const double av = ok ? spmv<FMT>(d.A, r, [=](int64_t cc) { return mul_rn(inv, ld(bg, cc)); }) : 0.0;
        if (a.sl) st(d.V, (int64_t)tile * TS + threadIdx.x, v0);
        else st_pair(d.V, (int64_t)tile * TS, 0, threadIdx.x, v0, 0.0);
        st(d.U, r, v0);
        const double e[3] = {v0 * bv, v0 * v0, v0 * av};
        reduce_scalars<3>(e, tr, acc, 0, first);
    }
    store_partials(acc, d.P1, d.npd, 3);
}

// Write the pending column j+1 (the flush of every method, and LanczosReorth's per-step
// write of v_{j+1}) with the one-sweep kernel's reductions: one 256-row tile per block,
// XCD-aware tile slots, column dots reduce-scattered by DPP into private LDS slots, one
// partial per tile.  MODE 0 (Arnoldi): v = (u - V[:,0..j] h2) * inv(beta) from U or W;
//   P1 = [ gram <V[:,c],v> (c<=j, tracked factors) | <v,v> | <v,b> ]      (POST_ARN_FIN)
// MODE 1 (Lanczos TTR): v = (beta == 0 ? 0 : inv(beta) .* W) (src/orthogonal_bases.jl:59);
//   P1 = [ <v,b> | gram <V[:,c],v> (c<=j) | <v,v> ]  (gram and <v,v>: tracked)  (POST_LAN_FIN)
// For j + 1 <= 64 columns (the register row); beyond, and for gated launches, the
// tile-loop kernels above.  Single-column tiles (a.sl, MODE 2 only): the Gram-free branch
// checks a.sl itself; the register-row path (V * Y) takes SL as a template argument.
template <int MAXC, int MODE, bool VY = false, bool SL = false>
__device__ __forceinline__ void fin_d_tile(const DFac& d, const KArgs& a, int slot, double* lds,
                                           const double* __restrict__ Yf = nullptr, double* __restrict__ Xf = nullptr,
                                           int ldy = 0, int tq = 0) {
    constexpr int NG = (MAXC + 15) / 16;
    const int j = a.j, nc = j + 1, t = threadIdx.x;
    const int64_t TS = (int64_t)TPB * kcp(a.kmax);
    const int64_t r = (int64_t)slot * TPB + t;
    const bool ok = r < a.n;
    const double* Vt = d.V + (int64_t)slot * TS;
    const uint32_t toff = t * 16u;
    // one-sweep Arnoldi after an even step: column j is in E, its pair in V is not written yet
    const bool em = (MODE == 0 || MODE == 2) && a.ecol == j;
    const rsrc_t tv = mkrsrc(Vt, vrange(em ? j : nc));
    const bool gram = d.track_gram != 0;
    double* acc = lds;
    const double inv_beta = ld(d.sc, SC_INVBETA);
    // MODE 2 (one-sweep Lanczos): v = inv(beta) .* (u - alpha v_j), u = the last step's raw vector
    const double alpha2 = MODE == 2 ? ld(d.sc, SC_ALPHA) : 0.0;
    const double up2 = MODE == 2 ? ld(a.ubuf ? d.W : d.U, r) : 0.0;
    if (MODE >= 1 && !gram && !VY) {
        // Lanczos without a Gram row: v, the pair store (other half = column j), <v,b>
        const double vjc = em ? (ok ? ld(d.E, r) : 0.0) : (a.sl ? bld(tv, t * 8u + sofs(j)) : bld(tv, toff + cofs(j)));
        double v;
        if (MODE == 2) {
            v = ok ? mul_rn(inv_beta, sub_rn_(up2, mul_rn(alpha2, vjc))) : 0.0;
        } else {
            const bool zero = ld(d.sc, SC_BETA) == 0.0;
            v = (zero || !ok) ? 0.0 : mul_rn(ld(d.W, r), inv_beta);
        }
        const double other = ((j + 1) & 1) ? vjc : 0.0;
        if (a.sl) st(d.V, (int64_t)slot * TS + svofs(j + 1, t), v);
        else st_pair(d.V, (int64_t)slot * TS, j + 1, t, v, other);
        double x[16] = {v * ld(d.b, r)};
        acc[t] = rs16(x);
        __syncthreads();
        if (t == 0) {
            double sum = 0.0;
#pragma unroll
            for (int p = 0; p < 16; ++p) sum += acc[p * 16];
            st(d.P1, slot, sum);   // vi = 0
        }
        return;
    }
    double* Ys = lds + (NG + 1) * TPB;   // VY: Y_s staged in LDS (tq x ldy)
    if constexpr (VY)
        for (int i = t; i < tq * ldy; i += TPB) Ys[i] = ld(Yf, i);
    Row<MAXC> R;
    if (SL) {
        R.load_sl(tv, t * 8u, nc);
    } else {
        R.load(tv, toff, em ? j : nc);
        if (em) R.set_col(j, ok ? ld(d.E, r) : 0.0);
    }
    double v;
    if (MODE == 0) {
        const double up = ld(a.ubuf ? d.W : d.U, r);
        v = ok ? (up - row_dot<MAXC, true>(R, tv, toff, nc, d.h2)) * inv_beta : 0.0;
    } else if (MODE == 2) {
        v = ok ? mul_rn(inv_beta, sub_rn_(up2, mul_rn(alpha2, R.last))) : 0.0;   // R.last = column j
    } else {
        const bool zero = ld(d.sc, SC_BETA) == 0.0;
        v = (zero || !ok) ? 0.0 : mul_rn(ld(d.W, r), inv_beta);
    }
    if (SL) st(d.V, (int64_t)slot * TS + svofs(j + 1, t), v);
    else st_pair(d.V, (int64_t)slot * TS, j + 1, t, v, ((j + 1) & 1) ? R.last : 0.0);
    if constexpr (VY) {
        // X_s[r, q] = sum_{c < k} V[r, c] Y_s[c, q] from the register row the flush just
        // loaded (the tile is streamed once for both); Y_s columns zero-padded to ldy >= MAXC
        // (so columns k..j of the row meet zeros), two columns at a time from LDS (broadcast
        // reads; through the scalar cache each group of coefficients was a dependent round trip)
        __syncthreads();
        for (int q = 0; q < tq; q += 2) {
            double x0, x1;
            row_dot2_lds<MAXC, TK_VY_GRP>(R, Ys + q * ldy, Ys + (q + 1 < tq ? q + 1 : q) * ldy, x0, x1);
            // X tile-major like V: the tile's tq columns of 256 rows are one contiguous block,
            // so the stores stream (column-major n x t stores cost a third of the kernel)
            if (ok) {
                double* Xt = Xf + (int64_t)slot * TPB * tq + t;
                st_x(Xt, (int64_t)q * TPB, x0);
                if (q + 1 < tq) st_x(Xt, (int64_t)(q + 1) * TPB, x1);
            }
        }
    }
    if (gram) {
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            double x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = 16 * k + i < MAXC ? R.v[16 * k + i < MAXC ? 16 * k + i : 0] * v : 0.0;
            acc[k * TPB + t] = rs16(x);
        }
    }
    {
        double x[16] = {v * v, v * ld(d.b, r)};
        acc[NG * TPB + t] = rs16(x);
    }
    __syncthreads();
    // combine the 16 row-group partials of every value in fixed order
    for (int e = t; e < (NG + 1) * 16; e += TPB) {
        const int k = e >> 4, sl = e & 15;
        if (k < NG && !gram) continue;
        double sum = 0.0;
#pragma unroll
        for (int p = 0; p < 16; ++p) sum += acc[k * TPB + p * 16 + sl];
        int vi = -1;
        if (k < NG) {
            const int c = 16 * k + sl;
            if (c < nc) vi = MODE == 0 ? c : 1 + c;
        } else if (sl == 0) {            // <v,v>
            if (MODE == 0) vi = nc;
            else if (gram) vi = 1 + nc;
        } else if (sl == 1) {            // <v,b>
            vi = MODE == 0 ? nc + 1 : 0;
        }
        if (vi >= 0) st(d.P1, (int64_t)vi * a.ntiles + slot, sum);
    }
}

template <int MAXC, int MODE>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(MAXC <= 32 ? 4 : 3, MAXC <= 32 ? 4 : 3)))
void k_fin_d(const DFac* __restrict__ F, KArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];   // acc[NG + 1][256]
    const DFac& d = F[blockIdx.y];
    const int slot = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
    if (slot >= a.ntiles) return;
    fin_d_tile<MAXC, MODE>(d, a, slot, lds);
}

// ------------------------------------------------------------------ Lanczos (TTR)

// Plain, v_j stored (src/orthogonal_bases.jl:45-50):
//   U = A v_j - beta_{j-1} v_{j-1};  P1 = [ <U, v_j> ]
template <int FMT>
__global__ __launch_bounds__(TPB) void k_lan_l1_plain(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    double* acc = lds;
    const int j = a.j;
    const double bp = j > 0 ? ld(d.sc, SC_BETAPREV) : 0.0;
    TILE_LOOP
        const double* Vg = d.V;
        const double av = ok ? spmv<FMT>(d.A, r, [=](int64_t c) { return ld(Vg, (c >> 8) * TS + vofs(j, (int)(c & 255))); }) : 0.0;
        const double prev = j > 0 ? ld(Vt, vofs(j - 1, threadIdx.x)) : 0.0;
        const double u = av - bp * prev;
        const double v = ld(Vt, vofs(j, threadIdx.x));
        st(d.U, r, u);
        const double e[1] = {u * v};
        reduce_scalars<1>(e, tr, acc, 0, first);
    }
    store_partials(acc, d.P1, a.npart, 1);
}

// Fused: pending v_j = (beta == 0 ? 0 : inv(beta) .* W) (src/orthogonal_bases.jl:59) is
// written while  U = A v_j - beta v_{j-1};
//   P1 = [ <U,v_j>, <v_j,b> | gram <V[:,c],v_j> (c<j), <v_j,v_j> ]
template <int FMT>
__global__ __launch_bounds__(TPB) void k_lan_l1_fused(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    double* acc = lds;
    const int j = a.j;
    const double beta = ld(d.sc, SC_BETA);
    const double inv_beta = ld(d.sc, SC_INVBETA);
    const bool zero = (beta == 0.0);
    const bool gram = d.track_gram != 0;
    TILE_LOOP
        const double vj = (zero || !ok) ? 0.0 : mul_rn(ld(d.W, r), inv_beta);
        const double* Wg = d.W;
        const double av = ok ? spmv<FMT>(d.A, r, [=](int64_t c) { return zero ? 0.0 : mul_rn(ld(Wg, c), inv_beta); }) : 0.0;
        const double vprev = ld(Vt, vofs(j - 1, threadIdx.x));
        const double u = av - beta * vprev;
        st_pair(d.V, (int64_t)tile * TS, j, threadIdx.x, vj, (j & 1) ? vprev : 0.0);
        st(d.U, r, u);
        const rsrc_t tv = mkrsrc(Vt, vrange(j));
        const double e1[2] = {u * vj, vj * ld(d.b, r)};
        reduce_scalars<2>(e1, tr, acc, 0, first);
        if (gram) {
            reduce_stream(tv, toff, j, vj, tr, acc, 2, first);
            const double e2[1] = {vj * vj};
            reduce_scalars<1>(e2, tr, acc, 2 + j, first);
        }
    }
    store_partials(acc, d.P1, a.npart, gram ? j + 3 : 2);
}

// The same step as k_lan_l1_fused for j <= 64, laid out like k_fin_d: one tile per block
// (XCD-aware slots), the tracked factor's Gram row from a register row of V[:, 0..j) with DPP
// reduce-scatters, one partial per tile.  The Gram row was the long pole of the tile-loop
// kernel: factor 1's 1024 blocks streamed it through LDS transposes while the other factors'
// blocks had long finished.
//   P1 = [ <U,v_j>, <v_j,b> | gram <V[:,c],v_j> (c<j), <v_j,v_j> ]   (as k_lan_l1_fused)
template <int MAXC, int FMT>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(MAXC <= 32 ? 4 : 3, MAXC <= 32 ? 4 : 3)))
void k_lan_d1(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    constexpr int NG = (MAXC + 15) / 16;
    extern __shared__ __attribute__((aligned(16))) double lds[];   // acc[NG + 1][256]
    const DFac& d = F[blockIdx.y];
    const int slot = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
    if (slot >= a.ntiles) return;
    const int j = a.j, t = threadIdx.x;
    const int64_t TS = (int64_t)TPB * kcp(a.kmax);
    const int64_t r = (int64_t)slot * TPB + t;
    const bool ok = r < a.n;
    const double* Vt = d.V + (int64_t)slot * TS;
    const uint32_t toff = t * 16u;
    const rsrc_t tv = mkrsrc(Vt, vrange(j));
    const bool gram = d.track_gram != 0;
    double* acc = lds;
    const double beta = ld(d.sc, SC_BETA);
    const double inv_beta = ld(d.sc, SC_INVBETA);
    const bool zero = (beta == 0.0);
    const double vj = (zero || !ok) ? 0.0 : mul_rn(ld(d.W, r), inv_beta);
    const double* Wg = d.W;
    const double av = ok ? spmv<FMT>(d.A, r, [=](int64_t c) { return zero ? 0.0 : mul_rn(ld(Wg, c), inv_beta); }) : 0.0;
    if (!gram) {
        const double vprev = bld(tv, toff + cofs(j - 1));
        const double u = av - beta * vprev;
        st_pair(d.V, (int64_t)slot * TS, j, t, vj, (j & 1) ? vprev : 0.0);
        st(d.U, r, u);
        double x[16] = {u * vj, vj * ld(d.b, r)};
        acc[t] = rs16(x);
        __syncthreads();
        if (t < 2) {
            double sum = 0.0;
#pragma unroll
            for (int p = 0; p < 16; ++p) sum += acc[p * 16 + t];
            st(d.P1, (int64_t)t * a.ntiles + slot, sum);
        }
        return;
    }
    Row<MAXC> R;
    R.load(tv, toff, j);
    const double vprev = R.last;   // column j - 1
    const double u = av - beta * vprev;
    st_pair(d.V, (int64_t)slot * TS, j, t, vj, (j & 1) ? vprev : 0.0);
    st(d.U, r, u);
#pragma unroll
    for (int k = 0; k < NG; ++k) {
        double x[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = 16 * k + i < MAXC ? R.v[16 * k + i < MAXC ? 16 * k + i : 0] * vj : 0.0;
        acc[k * TPB + t] = rs16(x);
    }
    {
        double x[16] = {u * vj, vj * ld(d.b, r), vj * vj};
        acc[NG * TPB + t] = rs16(x);
    }
    __syncthreads();
    for (int e = t; e < (NG + 1) * 16; e += TPB) {
        const int k = e >> 4, sl = e & 15;
        double sum = 0.0;
#pragma unroll
        for (int p = 0; p < 16; ++p) sum += acc[k * TPB + p * 16 + sl];
        int vi = -1;
        if (k < NG) {
            const int c = 16 * k + sl;
            if (c < j) vi = 2 + c;
        } else if (sl < 2) {
            vi = sl;             // <U,v_j>, <v_j,b>
        } else if (sl == 2) {
            vi = 2 + j;          // <v_j,v_j>
        }
        if (vi >= 0) st(d.P1, (int64_t)vi * a.ntiles + slot, sum);
    }
}

// W = U - alpha v_j (src/orthogonal_bases.jl:53);  P2 = [ <W,W> ]
__global__ __launch_bounds__(TPB) void k_lan_l2(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    double* acc = lds;
    const int j = a.j;
    const double alpha = ld(d.RED1, 0);
    TILE_LOOP
        const double w = ok ? ld(d.U, r) - alpha * ld(Vt, vofs(j, threadIdx.x)) : 0.0;
        st(d.W, r, w);
        const double e[1] = {w * w};
        reduce_scalars<1>(e, tr, acc, 0, first);
    }
    store_partials(acc, d.P2, a.npart, 1);
}

// Write pending column j+1 = (beta == 0 ? 0 : inv(beta) .* W);
//   P1 = [ <v,b> | gram <V[:,c],v> (c<=j), <v,v> ]
__global__ __launch_bounds__(TPB) void k_lan_finalize(const DFac* __restrict__ F, KArgs a) {
#pragma clang fp contract(off)
    KERNEL_PROLOGUE
    double* acc = lds;
    const int j = a.j, nc = j + 1;
    const double beta = ld(d.sc, SC_BETA);
    const double inv_beta = ld(d.sc, SC_INVBETA);
    const bool zero = (beta == 0.0);
    const bool gram = d.track_gram != 0;
    TILE_LOOP
        const double v = (zero || !ok) ? 0.0 : mul_rn(ld(d.W, r), inv_beta);
        st_pair(d.V, (int64_t)tile * TS, j + 1, threadIdx.x, v, ((j + 1) & 1) ? ld(Vt, vofs(j, threadIdx.x)) : 0.0);
        const rsrc_t tv = mkrsrc(Vt, vrange(nc));
        const double e1[1] = {v * ld(d.b, r)};
        reduce_scalars<1>(e1, tr, acc, 0, first);
        if (gram) {
            reduce_stream(tv, toff, nc, v, tr, acc, 1, first);
            const double e2[1] = {v * v};
            reduce_scalars<1>(e2, tr, acc, 1 + nc, first);
        }
    }
    store_partials(acc, d.P1, a.npart, gram ? nc + 2 : 1);
}

// ------------------------------------------------------------------ reductions

// RED[c] = sum_b P[c*npart + b]: one wave per value, fixed order (16 independent
// strided loads per lane, then a fixed-order combine).
__global__ __launch_bounds__(64) void k_reduce(const DFac* __restrict__ F, int which, int nv, int npart, int gate) {
    const DFac& d = F[blockIdx.y];
    const int c = blockIdx.x;
    if (c >= nv) return;
    if (gate && ld(d.sc, SC_REDO) == 0.0) return;
    if (npart <= 0) npart = d.npd;
    const double* P = (which == 2 ? d.P2 : d.P1) + (int64_t)c * npart;   // which 3: P1 -> RED2
    const int l = threadIdx.x;
    double s = 0.0;
    for (int b0 = 0; b0 < npart; b0 += 1024) {   // rounds of 16 independent loads per lane
        double part[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int b = b0 + l + 64 * i;
            part[i] = b < npart ? ld(P, b) : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) s += part[i];
    }
    s = row16_sum(s);
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (l == 0) st(which == 1 ? d.RED1 : d.RED2, c, s);
}

// Same for the one-sweep kernel's per-window partials (npart = DFac::npd, ~4k at n = 2^20):
// four waves per value, each lane a strided subset in rounds of 16 independent loads, DPP
// row sums, the 16 row totals summed in fixed order.
__device__ void post_signal(const KArgs& a, const DFac& d, int fidx, bool mirrored, bool coherent);
// The one-sweep Lanczos step's end, in the block that has its reduced dots (every thread
// alike): alpha_j = <u,v_j> (src/orthogonal_bases.jl:50), beta_j = ||u - alpha v_j|| (:56),
// v_{j+1}'s scalars for the next step / the flush, and the step's record row (as POST_LAN:
// H[j,j], H[j+1,j], btilde_j = <v_j,b>, the Gram row of v_j via gram(c)) written through,
// with its host mirror, then the exchange / host signal.  al_est = alpha_{j-1}, the estimate
// the sweep took wt = u - al_est v_j around.
template <class G>
__device__ void lan_step_record(const DFac& d, const KArgs& ax, int fidx, double al, double vv, double bt, double ww,
                                double wv, double al_est, G gram) {
#pragma clang fp contract(off)
    const int t = threadIdx.x;
    const int j = ax.j, kmax = ax.kmax;
    // ||u - al v||^2 = ||wt + dl v||^2, dl = al_est - al: no cancellation of the size of
    // alpha^2 (k_lan_1s)
    const double dl = al_est - al;
    const double bsq = add_rn(add_rn(ww, mul_rn(2.0 * dl, wv)), mul_rn(mul_rn(dl, dl), vv));
    const double beta = sqrt(bsq > 0.0 ? bsq : 0.0);
    const double ib = beta == 0.0 ? 0.0 : 1.0 / beta;
    if (t == 0) {
        st(d.sc, SC_ALPHA, al);
        st(d.sc, SC_INVBETA, ib);
        st(d.sc, SC_BETA, beta);
        st(d.sc, SC_BETAPREV, beta);
        __hip_atomic_store(d.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    double* rec = ax.rec + (int64_t)d.gidx * ax.m;
    double* hr = ax.hdone ? ax.hrec + (int64_t)d.gidx * ax.m : nullptr;
    const int g0 = rec_gram(kmax);
    for (int i = t; i < ax.m; i += blockDim.x) {
        double v = 0.0;
        if (i == j) v = al;
        else if (i == j + 1) v = beta;
        else if (i >= g0 && i <= g0 + j) v = d.track_gram ? (i - g0 < j ? gram(i - g0) : vv) : 0.0;
        else if (i == rec_beta(kmax)) v = beta;
        else if (i == rec_bt(kmax)) v = bt;
        else if (i == rec_col(kmax)) v = (double)j;
        else if (i == rec_tracked(kmax)) v = d.track_gram ? 1.0 : 0.0;
        __hip_atomic_store(rec + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (hr) __hip_atomic_store(hr + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    post_signal(ax, d, fidx, true, true);
}

// The gram-free one-sweep Lanczos step's reduce (k_lan_1w's 6 values over DFac::nwl
// partials) in ONE block of 1024 threads per factor: every partial of the step loaded in one
// round (<= 3 per value per thread up to nwl = 3072), summed per thread in order, DPP row sums,
// the 64 row totals in fixed order -- then alpha, beta and the record in the same block: no
// arrival counting between blocks (k_reduce256's six blocks and their hand-off measured
// ~6 us per step, most of it the chain load -> coherent store -> atomic -> load).
__global__ __launch_bounds__(1024) void k_red_lan(const DFac* __restrict__ F, KArgs ax) {
    __shared__ double rs[6][64];
    __shared__ double red[6];
    const DFac& d = F[blockIdx.x];
    const int t = threadIdx.x, np = d.nwl;
    // (read before the barrier below: thread 0 overwrites it in lan_step_record)
    const double al_est = ld(d.sc, SC_ALPHA);
    double sv[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int p0 = 0; p0 < np; p0 += 3 * 1024) {
        double q[3][6];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                const int p = p0 + k * 1024 + t;
                q[k][c] = p < np ? ld(d.P1, (int64_t)c * np + p) : 0.0;
            }
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c = 0; c < 6; ++c) sv[c] += q[k][c];
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const double r = row16_sum(sv[c]);
        if ((t & 15) == 0) rs[c][t >> 4] = r;
    }
    __syncthreads();
    if (t < 6) {
        double r = 0.0;
        for (int q = 0; q < 64; ++q) r += rs[t][q];
        red[t] = r;
    }
    __syncthreads();
    lan_step_record(d, ax, (int)blockIdx.x, red[0], red[2], red[3], red[4], red[5], al_est, [](int) { return 0.0; });
}

// coefJ >= 0: one-sweep Arnoldi step -- a plain reduction into RED1 (its readers evaluate the
// next step's scalars from it themselves, d1_scalars; round 4's last block that evaluated and
// handed them on cost C4's one-factor step ~2 us);
// RED_LAN: one-sweep Lanczos step (nv = 6 + j; 6 for factors without a Gram row; the last
// block evaluates alpha, beta and writes the step's record, ax = the step's KArgs).
// MM: the hand-off in the HIP memory model's own form (release/acquire add + acquire fence);
// otherwise the measured relaxed form -- chosen per process by red_mm() (tk_abi.cpp's startup
// self-check compares the two and keeps MM if they ever differ)
// FUSED (a fused one-sweep launch's leading blocks, k_arn_d1 with a pending reduce): every
// value is stored with an agent-scope atomic and drained before the block counts its arrival;
// the last block publishes `wseq` in the factor's step word -- the in-launch hand-off row of
// /opt/skills/guides/MI355X_MICROARCH.md (every store of the handed-off bytes sc1 and drained
// before the flag, every load of them sc1).
// which: 1 P1 -> RED1, 2 P2 -> RED2, 3 P1 -> RED2, 5 P1b -> RED1 (the odd steps' partials of a
// fused handle).
template <bool MM, bool FUSED>
__device__ __forceinline__ void red256_block(const DFac& d, int fidx, int c, int which, int nv, int np, int coefJ,
                                             const KArgs& ax, unsigned long long wseq) {
    __shared__ double rs[16];
    __shared__ int last;
    const int nv0 = nv;   // (the stored scalars' place after the values)
    if (coefJ == RED_LAN && !d.track_gram) nv = 6;
    if (coefJ >= 0 && !d.track_gram) nv = 2 * coefJ + 4;   // one-sweep Arnoldi: no Gram row
    if (c >= nv) return;
    const int npart = np > 0 ? np : d.npd;
    const double* P = (which == 2 ? d.P2 : (which == 5 ? d.P1b : d.P1)) + (int64_t)c * npart;   // which 3: P1 -> RED2
    const int t = threadIdx.x;
    double s = 0.0;
    for (int b0 = 0; b0 < npart; b0 += 6144) {   // one round up to 6144 partials (n ~ 1.5M)
        double part[24];
#pragma unroll
        for (int i = 0; i < 24; ++i) {
            const int b = b0 + t + 256 * i;
            part[i] = b < npart ? ld(P, b) : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 24; ++i) s += part[i];
    }
    s = row16_sum(s);
    if ((t & 15) == 0) rs[t >> 4] = s;
    __syncthreads();
    if (t == 0) {
        double r = 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) r += rs[q];
        if ((coefJ < 0 && coefJ != RED_LAN) || (coefJ >= 0 && !FUSED && ax.wsc)) {
            st(which == 1 || which == 5 ? d.RED1 : d.RED2, c, r);
        } else {
            // one-sweep step: publish the value coherently (agent-scope store, through to the
            // device-coherent level; its completion awaited), then count the arrival -- no
            // L2 writeback.  The last of the nv blocks of this factor evaluates the scalars.
            // This is the hand-off row "ONE lane of each storing workgroup ... an agent-scope
            // atomic add | ... the workgroup whose add came last, told by the value its add
            // returned | ... the other waves load after a workgroup barrier" of the measured
            // table in /opt/skills/guides/MI355X_MICROARCH.md (stores and loads sc1 = the
            // agent-scope relaxed atomics here, vmcnt(0) before the add): measured correct on
            // gfx950, not an architectural guarantee.  The memory-model form -- a
            // release on the add, an acquire in the last block (TK_RED_MM=1) -- writes back /
            // invalidates L2 on this 8-XCD part: C2 -5 %, C1 -12 %
            // (profiles/r04/reduce_handoff_mm_ab.txt).  ctr's reset below is ordered before the
            // next launch by the kernel boundary.
            __hip_atomic_store(d.RED1 + c, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if constexpr (MM) {
                // memory-model form: the add releases this block's value and acquires the others'
                last = __hip_atomic_fetch_add(d.ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nv - 1);
            } else {
                __builtin_amdgcn_s_waitcnt(0);
                last = __hip_atomic_fetch_add(d.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nv - 1);
            }
        }
    }
    if ((coefJ < 0 && coefJ != RED_LAN) || (coefJ >= 0 && !FUSED && ax.wsc)) return;
    // (the one-sweep Lanczos' alpha estimate, read before the barrier: thread 0 of the last
    // block overwrites it below)
    const double al_est = coefJ == RED_LAN ? ld(d.sc, SC_ALPHA) : 0.0;
    __syncthreads();
    if (!last) return;
    // (every wave of the last block: its loads ordered after thread 0's acquire)
    if constexpr (MM) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    auto cld = [&](int i) { return __hip_atomic_load(d.RED1 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    if (coefJ == RED_LAN) {
        lan_step_record(d, ax, fidx, cld(0), cld(2), cld(3), cld(4), cld(5), al_est,
                        [&](int c) { return cld(6 + c); });
        return;
    }
    if constexpr (!FUSED) {
        // one-sweep Arnoldi with factor groups: the last block evaluates the next step's scalars
        // (d1_scalars, J = coefJ <= 64) and stores them after the values for the windows and
        // the bookkeeping (the same bits as evaluating them there)
        if (t >= 64) return;
        const int J = coefJ;
        double beta, ib, t1;
        d1_scalars(t < J ? cld(t) : 0.0, t < J ? cld(J + t) : 0.0, cld(2 * J), cld(2 * J + 1), beta, ib, t1);
        if (t == 0) {
            double* o = d.RED1 + nv0;
            st(o, D1S_IB, ib);
            st(o, D1S_GAMMA, t1 * ib);
            st(o, D1S_BETA, beta);
            st(o, D1S_T1, t1);
            __hip_atomic_store(d.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // FUSED one-sweep Arnoldi: every value is through to the device (each block drained its
    // store before counting): publish the step (ctr's reset is ordered before the next launch
    // by the kernel boundary)
    if (t == 0) {
        __hip_atomic_store(d.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (MM) {
            // memory-model form: a release store (the windows' fuse_wait takes the acquire);
            // this thread acquired every block's value at its add above, so the release covers them
            __hip_atomic_store(d.rword, wseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __builtin_amdgcn_s_waitcnt(0);
            __hip_atomic_store(d.rword, wseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
// The one-sweep Arnoldi step's reduce over window-major partials (KArgs::pgrp: factor groups
// over long grids; groups of D1G values, tk_internal.h), in EXACTLY the arithmetic order of the
// value-major reduce (red256_block), so that the layout a launch uses never changes a bit.  There,
// lane t of a value's block sums windows t, t + 256, t + 512, ... in order, the 16 lanes of each
// DPP row combine through row16_sum (rotations by 8, 4, 2, 1; lane 0's result is kept) and the 16
// row results are summed in order.  Here block `bid` = (group g, row q) takes lanes 16q .. 16q+15
// of all D1G values of the group (a wave loads four windows' whole 128-byte lines per
// instruction), evaluates row16_sum's tree for lane 0 of the row, stores the D1G row results to Q
// and counts its arrival on the group's counter; the group's last row block sums the 16 rows in
// order into RED1.  The factor's last group (a second counter) evaluates the next step's scalars
// (d1_scalars) and stores them after the values, as k_reduce256's last block does.
// Hand-offs: the relaxed form of the measured table in /opt/skills/guides/MI355X_MICROARCH.md
// (every handed-off value stored sc1 by the adding lane's own wave, drained with vmcnt(0) before
// the add; every reader loads sc1 after its add returned), or with MM the memory-model form
// (acq_rel adds, an acquire fence in the last block).
template <bool MM>
__device__ __forceinline__ void red_d1_block(const DFac& d, int bid, int which, int J) {
    __shared__ double sv[TPB];
    __shared__ int last;
    const int nvr = d1_nv(J, d.track_gram), ng = d1_groups(nvr);
    if (bid >= ng * 16) return;
    const int g = bid >> 4, row = bid & 15;
    const double* P = (which == 5 ? d.P1b : d.P1) + (int64_t)g * d.npd * D1G;
    const int t = threadIdx.x, v = t % D1G, tl = t / D1G, lane = 16 * row + tl;
    const int npart = d.npd;
    double s = 0.0;
    for (int b0 = 0; b0 < npart; b0 += 6144) {   // (red256_block's rounds, zeros past the end included)
        double part[24];
#pragma unroll
        for (int i = 0; i < 24; ++i) {
            const int b = b0 + lane + 256 * i;
            part[i] = b < npart ? ld(P, (int64_t)b * D1G + v) : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 24; ++i) s += part[i];
    }
    sv[tl * D1G + v] = s;
    __syncthreads();
    auto cld = [&](const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    if (t < D1G) {
        // row16_sum's lane 0: x_i = s_i + s_{i+8}, y_i = x_i + x_{i+4}, z_i = y_i + y_{i+2},
        // w_0 = z_0 + z_1 (each rotation adds the lane's own value first; IEEE addition commutes)
        double x[8], y[4], z[2];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = sv[i * D1G + t] + sv[(i + 8) * D1G + t];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = x[i] + x[i + 4];
        z[0] = y[0] + y[2];
        z[1] = y[1] + y[3];
        __hip_atomic_store(d.Q + ((int64_t)g * 16 + row) * D1G + t, z[0] + z[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0) {   // (lanes 0..15 of this wave stored the rows)
        if constexpr (MM) {
            last = __hip_atomic_fetch_add(d.ctrg + g, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 15u;
        } else {
            __builtin_amdgcn_s_waitcnt(0);
            last = __hip_atomic_fetch_add(d.ctrg + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 15u;
        }
    }
    __syncthreads();
    if (!last) return;
    if constexpr (MM) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (t < D1G) {
        double r = 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) r += cld(d.Q + ((int64_t)g * 16 + q) * D1G + t);
        if (g * D1G + t < nvr) __hip_atomic_store(d.RED1 + g * D1G + t, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // (the counter's reset is ordered before the next reduce by the kernel boundary)
    if (t == 0) __hip_atomic_store(d.ctrg + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the factor's groups: the last one to finish evaluates the scalars
    if (t == 0) {   // (lanes 0..15 of this wave stored the values)
        if constexpr (MM) {
            last = __hip_atomic_fetch_add(d.ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(ng - 1);
        } else {
            __builtin_amdgcn_s_waitcnt(0);
            last = __hip_atomic_fetch_add(d.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(ng - 1);
        }
    }
    __syncthreads();
    if (!last || t >= 64) return;
    if constexpr (MM) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    double beta, ib, t1;
    d1_scalars(t < J ? cld(d.RED1 + t) : 0.0, t < J ? cld(d.RED1 + J + t) : 0.0, cld(d.RED1 + 2 * J),
               cld(d.RED1 + 2 * J + 1), beta, ib, t1);
    if (t == 0) {
        double* o = d.RED1 + 3 * J + 3;
        st(o, D1S_IB, ib);
        st(o, D1S_GAMMA, t1 * ib);
        st(o, D1S_BETA, beta);
        st(o, D1S_T1, t1);
        __hip_atomic_store(d.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
template <bool MM>
__global__ __launch_bounds__(256) void k_red_d1(const DFac* __restrict__ F, int which, int J) {
    red_d1_block<MM>(F[blockIdx.y], (int)blockIdx.x, which, J);
}
template <bool MM>
__global__ __launch_bounds__(256) void k_reduce256(const DFac* __restrict__ F, int which, int nv, int np,
                                                   int coefJ, KArgs ax) {
    red256_block<MM, false>(F[blockIdx.y], (int)blockIdx.y, (int)blockIdx.x, which, nv, np, coefJ, ax, 0ull);
}

// ------------------------------------------------------------------ post-processing
// One 256-thread block per local factor: reduced values -> H / beta / records.
// `clear` zeroes the factor's record row first (the first post of a record slot).

__device__ __forceinline__ void put_gram(double* rec, int kmax, int c, const double* row, double bt,
                                         int tracked) {
    if (tracked)
        for (int i = threadIdx.x; i <= c; i += TPB) st(rec, rec_gram(kmax) + i, row[i]);   // row: LDS or global
    if (threadIdx.x == 0) {
        st(rec, rec_bt(kmax), bt);
        st(rec, rec_col(kmax), (double)c);
        st(rec, rec_tracked(kmax), tracked ? 1.0 : 0.0);
    }
}

// Column c's share of ||V'V - I||_F^2 from its Gram row g[0..c] (g[i] = <V[:,i], V[:,c]>):
// off-diagonal entries count twice (the Gram matrix is symmetric).
__device__ __forceinline__ double loss_row(const double* g, int c) {
    double s = 0.0;
    for (int i = 0; i < c; ++i) {
        const double v = ld(g, i);
        s += 2.0 * v * v;
    }
    const double dv = ld(g, c) - 1.0;
    return s + dv * dv;
}

#define POST_LDS_MAX 8192   // doubles of dynamic LDS for Hbar in k_post (kmax <= 88)
// Arnoldi post-processing of step j (one 256-thread block per factor): from
// red1 = [h1 (j+1)] (global) and red2 = [h2 (j+1) | |w'|^2 | bt_j | gram_j (j+1)] (LDS or
// global) write H[:, j] = h1 + h2 and beta = sqrt(|w'|^2 - |h2|^2) (the CGS2 form of
// src/orthogonal_bases.jl:22-36), g = Hbar h2 for the next step's lazy column, the
// step's record and scalars.  Hs: LDS for Hbar ((j+1)*(j+2) doubles) or null (global reads).
__device__ void post_arn(const DFac& d, const KArgs& a, double* rec, const double* red1, const double* red2,
                         double* Hs, double* h2s, double* sh) {
    const int j = a.j, kmax = a.kmax, KP = kmax + 2;
    const int t = threadIdx.x;
    double* Hc = d.H + (int64_t)j * KP;
    const int J2 = j + 2;
    double hh = 0.0;
    for (int i = t; i <= j; i += TPB) {
        const double h2 = red2[i];
        const double hv = ld(red1, i) + h2;
        st(Hc, i, hv);
        st(d.h2, i, h2);
        st(rec, i, hv);
        h2s[i] = h2;
        if (Hs) Hs[j * J2 + i] = hv;
        hh += h2 * h2;
    }
    if (Hs)   // stage Hbar[:, 0..j): eight independent loads in flight per thread
        for (int i0 = 0; i0 < j * J2; i0 += 8 * TPB) {
            double hv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int idx = i0 + q * TPB + t;
                const int i = idx / J2, l = idx - i * J2;
                hv[q] = (idx < j * J2 && l <= i + 1) ? ld(d.H, (int64_t)i * KP + l) : 0.0;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (i0 + q * TPB + t < j * J2) Hs[i0 + q * TPB + t] = hv[q];
        }
    hh = row16_sum(hh);
    hh += __shfl_xor(hh, 16);
    hh += __shfl_xor(hh, 32);
    if ((t & 63) == 0) sh[t >> 6] = hh;
    __syncthreads();
    if (t == 0) {
        const double s2 = (sh[0] + sh[1]) + (sh[2] + sh[3]);
        const double bsq = red2[j + 1] - s2;
        const double beta = sqrt(bsq > 0.0 ? bsq : 0.0);
        st(Hc, j + 1, beta);
        if (Hs) Hs[j * J2 + j + 1] = beta;
        st(rec, j + 1, beta);
        st(rec, rec_beta(kmax), beta);
        st(d.sc, SC_BETA, beta);
        st(d.sc, SC_INVBETA, 1.0 / beta);
        st(d.sc, SC_BETAPREV, beta);
        sh[8] = beta;
    }
    __syncthreads();
    // g = Hbar[0..j+1, 0..j] * h2 (column i of Hbar has rows 0..i+1)
    for (int l = t; l <= j + 1; l += TPB) {
        double s = 0.0;
        for (int i = (l > 0 ? l - 1 : 0); i <= j; ++i) {
            const double hv = Hs ? Hs[i * J2 + l]
                                 : (i == j ? (l == j + 1 ? sh[8] : ld(Hc, l)) : ld(d.H, (int64_t)i * KP + l));
            s += hv * h2s[i];
        }
        st(d.g, l, s);
    }
    put_gram(rec, kmax, j, red2 + j + 3, red2[j + 2], d.track_gram);
}

// Bookkeeping of one-sweep Arnoldi step j (a.j): everything the host and the later kernels
// read, none of which the next step's blocks wait for (they derive their coefficients from
// RED1 and the scalars k_reduce256 appends).  RED1 holds step j's reduced dots (k_arn_d1's layout)
//   c = <V[:,i],u> (i<=j) | q = <V[:,i],z> (i<=j) | |u|^2, <u,z>, <v_j,v_0>, gram_jj | gram (i<j)
// with u = u_{j+1}, z = A u.  c are the reorthogonalization coefficients of u, so
//   H[0..j, j] = h1 + c,  beta = H[j+1, j] = sqrt(|u|^2 - |c|^2)   (CGS2 of
//   src/orthogonal_bases.jl:22-36 in exact arithmetic),  v_{j+1} = (u - V c) * inv(beta),
// with h1 = d.g the first projection of A v_j (from the previous bookkeeping).  The first
// projection of A v_{j+1} = (z - A V c) * inv(beta) = (z - V Hbar c) * inv(beta) follows from
// the sweep's dots with V'V = I, V'v_{j+1} = 0:
//   h1'[l] = (q_l - (Hbar c)_l) * inv(beta)   (l <= j)
//   h1'[j+1] = ((<u,z> - c.q) * inv(beta) - (Hbar c)_{j+1}) * inv(beta)
// c -> h2, inv(beta) -> scalars (the flush of the pending column reads them), h1' -> d.g,
// and the step's record row (H column j, beta, bt_j = norm(b) <v_j,v_0>, the Gram row of
// column j) with its host mirror -- every entry written once.  lds: Hbar ((j+1)(j+2)
// doubles, j <= 64) then the reduced dots (3j+6).
__device__ void bk_arn_d(const DFac& d, const KArgs& a, double* rec, double* lds) {
    const int j = a.j, kmax = a.kmax;
    const int t = threadIdx.x;
    double* Hc = d.H + (int64_t)j * (kmax + 2);
    const int J2 = j + 2, nv = 3 * j + 6;
    double* Hs = lds;
    double* red = lds + (((j + 1) * J2 + 1) & ~1);
    // Hbar[:, 0..j) eight loads in flight per thread (few registers: this also runs in a
    // spare block of k_arn_d1, whose register budget is the window blocks'), the reduced
    // dots and h1 (column j of Hs until + c)
    const int HN = j * J2;
    for (int e0 = 0; e0 < HN; e0 += 8 * TPB) {
        double hv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = e0 + q * TPB + t;
            const int i = e / J2, l = e - i * J2;
            hv[q] = (e < HN && l <= i + 1) ? ld(d.H + (int64_t)i * (kmax + 2), l) : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (e0 + q * TPB + t < HN) Hs[e0 + q * TPB + t] = hv[q];
    }
    // (RED1 through sc1 loads: in a fused launch the reducers of the same launch wrote it)
    for (int i = t; i < nv; i += TPB) red[i] = ld_ag(d.RED1 + i);
    for (int i = t; i <= j; i += TPB) Hs[j * J2 + i] = ld(d.g, i);
    const double bnorm = ld(d.sc, SC_BNORM);
    __syncthreads();
    // the step's scalars, evaluated here as the next step's windows evaluate them (d1_scalars:
    // the same bits); RED1 = c [0,J) | q [J,2J) | |u|^2 | <u,z>, J = j + 1
    double beta, ib, t1;
    {
        const int l = t & 63, J = j + 1;
        d1_scalars(l < J ? red[l] : 0.0, l < J ? red[J + l] : 0.0, red[2 * J], red[2 * J + 1], beta, ib, t1);
    }
    for (int i = t; i <= j; i += TPB) {
        const double ci = red[i];
        const double hv = Hs[j * J2 + i] + ci;
        st(Hc, i, hv);
        st(d.h2, i, ci);
        Hs[j * J2 + i] = hv;
    }
    if (t == 0) {
        st(Hc, j + 1, beta);
        Hs[j * J2 + j + 1] = beta;
        st(d.sc, SC_BETA, beta);
        st(d.sc, SC_INVBETA, ib);
        st(d.sc, SC_BETAPREV, beta);
    }
    __syncthreads();
    // h1'[l] from (Hbar c)_l: four lanes per l over interleaved i, combined in fixed order
    for (int l0 = 0; l0 <= j + 1; l0 += TPB / 4) {
        const int l = l0 + (t >> 2), r = t & 3;
        double sum = 0.0;
        if (l <= j + 1)
            for (int i = (l > 0 ? l - 1 : 0) + r; i <= j; i += 4) sum += Hs[i * J2 + l] * red[i];
        sum += __shfl_xor(sum, 1);
        sum += __shfl_xor(sum, 2);
        if (r == 0 && l <= j + 1) st(d.g, l, l <= j ? (red[j + 1 + l] - sum) * ib : (t1 - sum) * ib);
    }
    // the record row (zeros included) and its host mirror
    double* hr = a.hdone ? a.hrec + (int64_t)d.gidx * a.m : nullptr;
    const int g0 = rec_gram(kmax);
    for (int i = t; i < a.m; i += TPB) {
        double v = 0.0;
        if (i <= j + 1) v = Hs[j * J2 + i];
        else if (i >= g0 && i <= g0 + j) v = d.track_gram ? (i - g0 < j ? red[2 * j + 6 + i - g0] : red[2 * j + 5]) : 0.0;
        else if (i == rec_beta(kmax)) v = beta;
        else if (i == rec_bt(kmax)) v = bnorm * red[2 * j + 4];   // norm(b) <v_j, v_0>
        else if (i == rec_col(kmax)) v = (double)j;
        else if (i == rec_tracked(kmax)) v = d.track_gram ? 1.0 : 0.0;
        // (post_signal: stores through to the coherence level the readers use -- the device's
        // for the exchange's all-reduce, the system's for the host mirror)
        __hip_atomic_store(rec + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (hr) __hip_atomic_store(hr + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
__host__ __device__ inline size_t bk_lds_doubles(int j) {
    return (size_t)((((j + 1) * (j + 2) + 1) & ~1) + 3 * j + 10);
}

// Tell the exchange stream that this block's record row is complete: all threads' stores
// are ordered before thread 0's device-scope release, then one system-scope add to the
// signal word (the stream waits for the count of all of the step's blocks; no event marker
// in the compute queue).
// coherent: the block wrote its record row with agent-scope stores (through to the device-
// coherent level, what the exchange stream's all-reduce reads) and its host mirror with
// system-scope stores (through to host memory), so each thread's completed stores
// (s_waitcnt) are all the signal must follow -- no system-scope fence, whose L2 writeback
// stalls the kernels running beside this block.
__device__ void post_signal(const KArgs& a, const DFac& d, int fidx, bool mirrored, bool coherent) {
    if (!a.xflag && !a.hdone) return;
    if (coherent) {
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (threadIdx.x == 0) {
            if (a.xflag) {
                if (d.xsig) __hip_atomic_store(d.xsig, a.xval, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                else __hip_atomic_fetch_add(a.xflag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (a.hdone) __hip_atomic_store(a.hdone + fidx, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    __syncthreads();
    if (a.hdone && !mirrored) {
        // host mirror of the record row (host-mapped, coherent), then its sequence number:
        // the host reads the record as soon as the word shows this step, without touching
        // the queues (later steps may already be running)
        const double* src = a.rec + (int64_t)d.gidx * a.m;
        double* dst = a.hrec + (int64_t)d.gidx * a.m;
        for (int i = threadIdx.x; i < a.m; i += TPB) dst[i] = ld(src, i);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        __threadfence_system();
        if (a.xflag) {
            if (d.xsig) __hip_atomic_store(d.xsig, a.xval, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            else atomicAdd_system(a.xflag, 1ull);
        }
        if (a.hdone)
            __hip_atomic_store(a.hdone + fidx, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(TPB) void k_post(const DFac* __restrict__ F, KArgs a, int kind, int flag,
                                              int clear) {
    __shared__ double sh[16];
    __shared__ double h2s[1024 + 8];
    extern __shared__ __attribute__((aligned(16))) double post_lds[];
    const DFac& d = F[blockIdx.x];
    if (a.gate && ld(d.sc, SC_REDO) == 0.0) return;
    if (kind == POST_SIGNAL) {
        post_signal(a, d, (int)blockIdx.x, false);
        return;
    }
    const int j = a.j, kmax = a.kmax;
    double* rec = a.rec + (int64_t)d.gidx * a.m;
    const int t = threadIdx.x;
    if (clear && kind != POST_ARN_D) {   // (POST_ARN_D writes the whole row)
        for (int i = t; i < a.m; i += TPB) st(rec, i, 0.0);
        __syncthreads();
    }
    if (kind == POST_INIT_A) {
        // coefficient arrays start clean (register-row dot products read them past the
        // current column count, against zero basis entries)
        for (int i = t; i < kmax + 2 + COEF_TAIL; i += TPB) {
            st(d.h2, i, 0.0);
            st(d.g, i, 0.0);
        }
        for (int i = t + 1; i < 2 * kmax + 8; i += TPB) st(d.RED2, i, 0.0);
        // (one-sweep register rows read RED1 past the live coefficients, against zero basis
        // entries: nothing stale from an earlier solve may be non-finite there)
        for (int i = t + 1; i < RED1_LEN(kmax); i += TPB) st(d.RED1, i, 0.0);
        if (t == 0) {
            const double nrm = sqrt(ld(d.RED1, 0));
            st(d.sc, SC_BNORM, nrm);
            st(d.sc, SC_INVB, 1.0 / nrm);
        }
        return;
    }
    if (kind == POST_INIT_B) {
        put_gram(rec, kmax, 0, d.RED1 + 1, ld(d.RED1, 0), d.track_gram);
        if (t == 0 && d.track_gram) st(d.lossrow, 0, loss_row(d.RED1 + 1, 0));
        if (flag) {
            // one-sweep Arnoldi: step 0 re-derives v_0 = U * 1.0 with no coefficients: its
            // scalars are beta = ib = 1 and gamma = <v0, A v0> (after the 3 init values), and
            // the bookkeeping's h1 = [<v0, A v0>]
            __syncthreads();   // (the record reads of RED1 above are done)
            if (t == 0) {
                const double vav = ld(d.RED1, 2);
                st(d.g, 0, vav);
                st(d.sc, SC_INVBETA, 1.0);
                // one-sweep Lanczos step 0: v_0 = 1 .* (U - alpha * 0), u_0 = A v_0 - 0 * 0; alpha
                // is only the estimate of alpha_0 = <v0, A v0> its beta is taken around (k_lan_1s)
                st(d.sc, SC_ALPHA, vav);
                st(d.sc, SC_BETAPREV, 0.0);
                double* o = d.RED1 + 2;   // (k_arn_d1 step 0 reads its scalars here)
                st(o, D1S_IB, 1.0);
                st(o, D1S_GAMMA, vav);
                st(o, D1S_BETA, 1.0);
                st(o, D1S_T1, vav);
            }
        }
        return;
    }
    if (kind == POST_ARN) {
        double* Hs = (a.kmax + 1) * (a.kmax + 2) <= POST_LDS_MAX ? post_lds : nullptr;   // = launcher's size
        post_arn(d, a, rec, d.RED1, d.RED2, Hs, h2s, sh);
        post_signal(a, d, (int)blockIdx.x, false);
        return;
    }
    if (kind == POST_ARN_D) {
        // dynamic LDS: Hbar ((j+1)(j+2) doubles, j <= 64), then the reduced dots
        bk_arn_d(d, a, rec, post_lds);
        post_signal(a, d, (int)blockIdx.x, true, true);
        return;
    }
    if (kind == POST_ARN_FIN) {
        // RED2 = [gram_{j+1} (j+2) | bt] (reduced from P1 into RED2: RED1 keeps the one-sweep
        // step's dots, which the next step still reads)
        put_gram(rec, kmax, j + 1, d.RED2, ld(d.RED2, j + 2), d.track_gram);
        if (t == 0 && d.track_gram) st(d.lossrow, j + 1, loss_row(d.RED2, j + 1));   // (redone column)
        return;
    }
    if (kind == POST_LAN) {
        // RED1 = [alpha | bt_j | gram_j (j+1)] (bt/gram only when fused), RED2 = [|w|^2]
        if (t == 0) {
            const double alpha = ld(d.RED1, 0);
            const double beta = sqrt(ld(d.RED2, 0));
            st(rec, j, alpha);
            st(rec, j + 1, beta);
            st(rec, rec_beta(kmax), beta);
            st(d.sc, SC_BETA, beta);
            st(d.sc, SC_INVBETA, 1.0 / beta);
            st(d.sc, SC_BETAPREV, beta);
        }
        if (flag) put_gram(rec, kmax, j, d.RED1 + 2, ld(d.RED1, 1), d.track_gram);
        else if (t == 0) st(rec, rec_col(kmax), -1.0);
        post_signal(a, d, (int)blockIdx.x, false);
        return;
    }
    if (kind == POST_LAN_FIN) {
        // RED1 = [bt | gram_{j+1} (j+2)]
        put_gram(rec, kmax, j + 1, d.RED1 + 1, ld(d.RED1, 0), d.track_gram);
        if (t == 0 && d.track_gram) {
            st(d.lossrow, j + 1, loss_row(d.RED1 + 1, j + 1));
            if (flag) {
                // LanczosReorth loss check (src/orthogonal_bases.jl:119-123):
                // loss = ||V[:,1:k+1]'V[:,1:k+1] - I||_F, MGS redo when loss > sqrt(eps)
                double s2 = 0.0;
                for (int c = 0; c <= j + 1; ++c) s2 += ld(d.lossrow, c);
                const double loss = sqrt(s2);
                const bool redo = loss > 1.4901161193847656e-8;   // sqrt(eps(Float64))
                st(rec, rec_loss(kmax), loss);
                st(rec, rec_flag(kmax), redo ? 1.0 : 0.0);
                st(d.sc, SC_REDO, redo ? 1.0 : 0.0);
            }
        }
        return;
    }
}

// ------------------------------------------------------------------ V * Y on MFMA

typedef double f64x4 __attribute__((ext_vector_type(4)));

// X[:, t0..t0+16*NG) = V[:, 0..k) * Y[:, t0..) (Y column-major k x t) for factor
// blockIdx.y; X column-major with leading dimension ld.  Block = one 256-row tile;
// wave w owns rows 64w..64w+63 as 4 strips of 16; NG 16-column groups per launch
// (blockIdx.z walks further groups).  v_mfma_f64_16x16x4_f64 with
//   A = V[16 rows x 4 k]  lane l: row l&15, k-slot l>>4
//   B = Y[4 k x 16]       lane l: k-slot l>>4, col l&15 (LDS)
//   D                     lane l: row (l>>4) + 4i, col l&15
// The sum over k is order-free, so the k-slots are permuted to match the paired-column
// layout: one dwordx4 per lane fetches V[row, 2m..2m+1] (m = kk/2 + slot) and feeds two
// MFMAs, the first over columns kk + 2*slot, the second over kk + 2*slot + 1.
// Each D register store covers 4 consecutive rows of 16 columns; the four registers
// of a strip complete 16-row runs that the L2 merges before write-back.
#define YS_STRIDE 72   // LDS row stride of Ys: rows 2*slot apart land 32 banks apart
#define XS_STRIDE 260  // LDS column stride of the staged X tile: a 64-lane b64 write is 2-way (optimal)
#define BM_LDS_DOUBLES (64 * YS_STRIDE)   // Ys; the X staging (16 x XS_STRIDE) reuses it
// One 256-row tile of X_s[:, t0 .. t0+16NG+TL) = V_s[:, 0..k) Y_s: NG 16-column groups on
// v_mfma_f64_16x16x4f64 (wave w owns rows 64w .. 64w+63, four 16-row groups) and TL <= 4 tail
// columns on the VALU -- a 16-column MFMA group holding t mod 16 <= 4 live columns would be
// three-quarters padding (t = 17 at C2: 2.1x the useful MFMAs when padded to 32); Y staged in
// LDS per 64-deep k chunk.  The k dimension runs in chunks of 8 columns (two MFMAs over one
// dwordx4 per lane); a last partial chunk of <= 4 columns takes ONE MFMA whose k-slot l>>4 is
// column kk + (l>>4) (the half of its pair), not two MFMAs over a padded 8 (k = 50: 13 MFMAs
// per 16 x 16 block instead of 14).  Each tail column: every lane accumulates its k-slots'
// products, the 4 k-slot lanes of a row are summed at the end (xor 16, xor 32; fixed order).
// The accumulators go through LDS (16 columns at a time) so each X column is written as 256
// contiguous rows (full lines) instead of 32-B pieces.  SL: single-column tiles, the two
// columns of a lane's k-slot pair as two 8-byte loads (16 consecutive rows per k-slot: 128 B).
template <int NG, int TL, bool SL>
__device__ __forceinline__ void basis_mul_tile(const DFac& d, const KArgs& a, const double* __restrict__ Y,
                                               double* __restrict__ X, int k, int t, int tile, int t0,
                                               double* Ys) {
    constexpr int NC = 16 * NG + TL;   // columns of this block
    const int64_t TS = (int64_t)TPB * kcp(a.kmax);
    const double* Vt = d.V + (int64_t)tile * TS;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    const int tn = min(NC, t - t0);
    f64x4 acc[4][NG > 0 ? NG : 1];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < NG; ++q) acc[s][q] = (f64x4){0.0, 0.0, 0.0, 0.0};
    double tac[4][TL > 0 ? TL : 1];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int c = 0; c < TL; ++c) tac[s][c] = 0.0;
    for (int k0 = 0; k0 < k; k0 += 64) {
        const int kn = min(64, k - k0);
        __syncthreads();
        for (int i = threadIdx.x; i < 64 * NC; i += 256) {
            const int kk = i & 63, tt = i >> 6;
            Ys[kk * YS_STRIDE + tt] = (kk < kn && tt < tn) ? ld(Y, (int64_t)(t0 + tt) * k + k0 + kk) : 0.0;
        }
        __syncthreads();
        const rsrc_t tv = mkrsrc(Vt + (int64_t)k0 * TPB, vrange(kn));   // k0 is even: pair aligned
        const int kf = kn & ~7;          // full 8-column chunks
        const int kr = kn - kf;          // the rest: one 4-slot MFMA if <= 4, else a padded chunk
        const int kp = kr > 4 ? kn : kf;
        for (int kk = 0; kk < kp; kk += 8) {
            const int ka = kk + 2 * lk;   // this lane's first column of the pair
            double bq0[NG > 0 ? NG : 1], bq1[NG > 0 ? NG : 1], tq0[TL > 0 ? TL : 1], tq1[TL > 0 ? TL : 1];
#pragma unroll
            for (int q = 0; q < NG; ++q) {
                bq0[q] = Ys[ka * YS_STRIDE + 16 * q + lr];
                bq1[q] = Ys[(ka + 1) * YS_STRIDE + 16 * q + lr];
            }
#pragma unroll
            for (int c = 0; c < TL; ++c) {
                tq0[c] = Ys[ka * YS_STRIDE + 16 * NG + c];
                tq1[c] = Ys[(ka + 1) * YS_STRIDE + 16 * NG + c];
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int row = wave * 64 + s * 16 + lr;
                d2_t av;
                if (SL) {
                    av.x = bld(tv, ((uint32_t)ka * TPB + row) * 8u);
                    av.y = bld(tv, ((uint32_t)(ka + 1) * TPB + row) * 8u);
                } else {
                    av = bld2(tv, ((uint32_t)(ka >> 1) * TPB + row) * 16u);
                }
                const double a1 = ka + 1 < kn ? av.y : 0.0;   // odd column past k: stale data
#pragma unroll
                for (int q = 0; q < NG; ++q)
                    acc[s][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bq0[q], acc[s][q], 0, 0, 0);
#pragma unroll
                for (int q = 0; q < NG; ++q)
                    acc[s][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bq1[q], acc[s][q], 0, 0, 0);
#pragma unroll
                for (int c = 0; c < TL; ++c) tac[s][c] = fma(a1, tq1[c], fma(av.x, tq0[c], tac[s][c]));
            }
        }
        if (kr > 0 && kr <= 4) {
            // k-slot lk = column kf + lk (the even or odd half of its pair), masked past kn
            const int kc = kf + lk;
            double bq[NG > 0 ? NG : 1], tq[TL > 0 ? TL : 1];
#pragma unroll
            for (int q = 0; q < NG; ++q) bq[q] = Ys[kc * YS_STRIDE + 16 * q + lr];
#pragma unroll
            for (int c = 0; c < TL; ++c) tq[c] = Ys[kc * YS_STRIDE + 16 * NG + c];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int row = wave * 64 + s * 16 + lr;
                double x;
                if (SL) {
                    x = kc < kn ? bld(tv, ((uint32_t)kc * TPB + row) * 8u) : 0.0;
                } else {
                    const d2_t av = bld2(tv, ((uint32_t)(kc >> 1) * TPB + row) * 16u);
                    x = kc < kn ? ((lk & 1) ? av.y : av.x) : 0.0;
                }
#pragma unroll
                for (int q = 0; q < NG; ++q)
                    acc[s][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, bq[q], acc[s][q], 0, 0, 0);
#pragma unroll
                for (int c = 0; c < TL; ++c) tac[s][c] = fma(x, tq[c], tac[s][c]);
            }
        }
    }
    // the tail columns' k-slot partials of each row, summed over the 4 k-slot lanes
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int c = 0; c < TL; ++c) {
            tac[s][c] += __shfl_xor(tac[s][c], 16);
            tac[s][c] += __shfl_xor(tac[s][c], 32);
        }
    // epilogue: 16 columns at a time through LDS (Xs[c][row], reusing Ys), then every thread
    // writes its row of each column -- a wave covers 512 contiguous bytes per column
    double* Xs = Ys;
    const int64_t r = (int64_t)tile * TPB + threadIdx.x;
#pragma unroll
    for (int q = 0; q < NG + (TL > 0 ? 1 : 0); ++q) {
        if (16 * q >= tn) break;
        __syncthreads();
        if (q < NG) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < 4; ++i) Xs[lr * XS_STRIDE + wave * 64 + s * 16 + lk + 4 * i] = acc[s][q < NG ? q : 0][i];
        } else if (lk == 0) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int c = 0; c < TL; ++c) Xs[c * XS_STRIDE + wave * 64 + s * 16 + lr] = tac[s][c];
        }
        __syncthreads();
        if (r < a.n) {
            const int cn = min(16, tn - 16 * q);
            for (int c = 0; c < cn; ++c)   // X tile-major (as k_fin_vy)
                st_x(X, (int64_t)tile * TPB * t + (int64_t)(t0 + 16 * q + c) * TPB + threadIdx.x, Xs[c * XS_STRIDE + threadIdx.x]);
        }
    }
}

// blockIdx.z = column slice: NG MFMA groups per slice, the last slice of the launch also
// takes the TL tail columns (slices before it are launched with TL = 0, see launch_basis_mul)
template <int NG, int TL, bool SL>
__global__ __launch_bounds__(256) void k_basis_mul(const DFac* __restrict__ F, KArgs a,
                                                   const double* __restrict__ Yall,
                                                   double* __restrict__ Xall, int k, int t, int z0) {
    __shared__ __attribute__((aligned(16))) double Ys[BM_LDS_DOUBLES];
    const int f = blockIdx.y;
    basis_mul_tile<NG, TL, SL>(F[f], a, Yall + (int64_t)f * k * t, Xall + (int64_t)f * a.ld * t, k, t, blockIdx.x,
                           (z0 + (int)blockIdx.z) * 16 * 2, Ys);
}

// The pending column's flush (fin_d_tile, MODE 0: Arnoldi) and V * Y of the same tile in one
// block: the register row the flush loads also feeds the product, so each basis tile is
// streamed from HBM once for both.  Y: [nf][t][ldy] with zero rows k..ldy-1, k <= j + 1.
template <int MAXC, int MODE, bool SL>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(MAXC <= TK_VY_OCC4 ? 4 : 3, MAXC <= TK_VY_OCC4 ? 4 : 3)))
void k_fin_vy(const DFac* __restrict__ F, KArgs a, const double* __restrict__ Yall, double* __restrict__ Xall,
              int ldy, int t) {
    extern __shared__ __attribute__((aligned(16))) double lds[];   // acc[NG + 1][256]
    const int f = blockIdx.y;
    const DFac& d = F[f];
    const int slot = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
    if (slot >= a.ntiles) return;
    fin_d_tile<MAXC, MODE, true, SL>(d, a, slot, lds, Yall + (int64_t)f * t * ldy, Xall + (int64_t)f * a.ld * t, ldy, t);
}

// ------------------------------------------------------------------ orthogonality Gram on MFMA
// G = V_s[:, 0..k)' V_s[:, 0..k) of one factor (orthogonality_loss, src/orthogonal_bases.jl:
// 231-257; the driver's orthogonality_data of factor 1, src/tensor_krylov_method.jl:103) as a
// SYRK on v_mfma_f64_16x16x4f64 (k <= 64): the MFMA's k-dimension runs over 4 basis rows, so
// the sum over n -- what per-step Gram rows spend DPP reduce-scatters on -- happens in the
// matrix core, and the basis is read once for all k columns instead of once per step.
// Column groups of 16 (lane l: row slot l>>4 of a 4-row quad, column (l&15) of the group):
//   group 0 / 1 = even / odd columns of 0..31 (one dwordx4 per lane: pair l&15),
//   group 2+g   = columns 32+16g .. 32+16g+15 (one dwordx2 per lane), g < NC16,
// and TAIL (<= 4) columns K0 = 32+16 NC16 .. k-1 that would fill a group of 16 by a quarter
// or less are formed on the VALU instead (all lanes load the tail pairs of their row: each
// lane multiplies the tail entries by its own group entries, and lane l&15 < TAIL by tail
// column l&15) -- at k = 50, 6 MFMA tiles per quad instead of 10 (the padded 16-column
// group had 2 live columns), which left the launch MFMA-bound at 58 % pipe use.
//   A = V[4 rows, group ga]'   lane l: column (l&15) of ga, row slot l>>4
//   B = V[4 rows, group gb]    lane l: row slot l>>4, column (l&15) of gb
//   D[m][n] = G[col(ga, m)][col(gb, n)],  lane l, reg i: m = (l>>4) + 4i, n = l&15.
// Blocks walk tiles (tile += gridDim.x, the grid a function of n only); the 4 waves'
// accumulators (and the tail's 4 row slots) are summed in fixed order through LDS and each
// block writes its partial Pg[block][value]; k_gram_reduce sums partials in block order.
// Values: NT tiles of 256 (group pairs ga <= gb), then with a tail 256 more: [a*64 + c] =
// G[K0 + a][c], c < K0 + TAIL (gram_unpack decodes both).
#ifndef TK_GRAM_GQ
#define TK_GRAM_GQ 8   // row quads whose loads are in flight before their MFMAs
#endif
// SL: single-column tiles -- two consecutive rows of a column per lane and dwordx4, two MFMA
// rounds per load (a different row-to-slot assignment: the same sums in another order).
template <int NC16, int TAIL, bool SL>
__global__ __launch_bounds__(256) void k_gram(const DFac* __restrict__ F, KArgs a, int f, int k,
                                              double* __restrict__ Pg) {
    constexpr int NGR = 2 + NC16;
    constexpr int NT = NGR * (NGR + 1) / 2;
    constexpr int K0 = 32 + 16 * NC16;
    constexpr int NS = NGR + 1;              // tail products per lane and tail column
    constexpr int NTP = (TAIL + 1) / 2;      // tail pairs
    constexpr int TA = TAIL > 0 ? TAIL : 1;
    __shared__ double red[NT * 4 * 64 + TAIL * NS * 256];
    const DFac& d = F[f];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, kr = lane >> 4, ci = lane & 15;
    const int64_t TS = (int64_t)TPB * kcp(a.kmax);
    f64x4 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i] = (f64x4){0.0, 0.0, 0.0, 0.0};
    double tac[TA][NS];
#pragma unroll
    for (int x = 0; x < TA; ++x)
#pragma unroll
        for (int s = 0; s < NS; ++s) tac[x][s] = 0.0;
    const bool ev = 2 * ci < k, od = 2 * ci + 1 < k;
    bool cm[NC16 > 0 ? NC16 : 1];
#pragma unroll
    for (int g = 0; g < NC16; ++g) cm[g] = 32 + 16 * g + ci < k;
    const int gq = w * 64 + kr;   // row of quad 0 of this lane
    // the products of one row slot: v[NGR] = this lane's entries of the column groups, tt[TA]
    // = the tail columns of its row
#define TK_GRAM_ACC(v, tt)                                                                               \
    {                                                                                                   \
        int i_ = 0;                                                                                     \
        _Pragma("unroll") for (int ga = 0; ga < NGR; ++ga)                                              \
            _Pragma("unroll") for (int gb = ga; gb < NGR; ++gb, ++i_)                                   \
                acc[i_] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[ga], v[gb], acc[i_], 0, 0, 0);        \
        if (TAIL > 0) {                                                                                 \
            double own = 0.0; /* tail column ci of this row (lanes ci < TAIL) */                        \
            _Pragma("unroll") for (int x2 = 0; x2 < TA; ++x2) own = ci == x2 ? tt[x2] : own;            \
            _Pragma("unroll") for (int x2 = 0; x2 < TA; ++x2) {                                         \
                _Pragma("unroll") for (int s = 0; s < NGR; ++s) tac[x2][s] = fma(tt[x2], v[s], tac[x2][s]); \
                tac[x2][NGR] = fma(tt[x2], own, tac[x2][NGR]);                                          \
            }                                                                                           \
        }                                                                                               \
    }
    // (loads of the next batch issued before this batch's MFMAs -- ping-pong buffers -- measured
    // 8-20 % slower: the register budget drops the launch to fewer waves)
    for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
        const rsrc_t tv = mkrsrc(d.V + (int64_t)tile * TS, vrange(k));
        constexpr int GQ = TK_GRAM_GQ;
        if constexpr (SL) {
            // single-column tiles: each lane loads TWO consecutive rows of a column per dwordx4
            // (the 4 row slots of a load then cover 8 rows: 64-byte runs per column, as the
            // pairs), feeding two MFMA rounds (.x rows, then .y rows) -- the sum over rows is
            // order-free.  GQ/2 such octets in flight.
            constexpr int GO = GQ >= 2 ? GQ / 2 : 1;
#pragma unroll 1
            for (int o0 = 0; o0 < 8; o0 += GO) {
                d2_t xe[GO], xo[GO];
                d2_t y2[GO][NC16 > 0 ? NC16 : 1];
                d2_t tc[GO][TA];
#pragma unroll
                for (int o = 0; o < GO; ++o) {
                    const uint32_t row = (uint32_t)(w * 64 + 8 * (o0 + o) + 2 * kr);
                    xe[o] = bld2(tv, ((uint32_t)(2 * ci) * TPB + row) * 8u);
                    xo[o] = bld2(tv, ((uint32_t)(2 * ci + 1) * TPB + row) * 8u);
#pragma unroll
                    for (int g = 0; g < NC16; ++g) y2[o][g] = bld2(tv, sofs(32 + 16 * g + ci) + row * 8u);
#pragma unroll
                    for (int x2 = 0; x2 < TAIL; ++x2) tc[o][x2] = bld2(tv, ((uint32_t)(K0 + x2) * TPB + row) * 8u);
                }
#pragma unroll
                for (int o = 0; o < GO; ++o)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        double v[NGR], tt[TA];
                        v[0] = ev ? (h ? xe[o].y : xe[o].x) : 0.0;
                        v[1] = od ? (h ? xo[o].y : xo[o].x) : 0.0;
#pragma unroll
                        for (int g = 0; g < NC16; ++g) v[2 + g] = cm[g] ? (h ? y2[o][g].y : y2[o][g].x) : 0.0;
#pragma unroll
                        for (int x2 = 0; x2 < TA; ++x2) tt[x2] = TAIL > 0 ? (h ? tc[o][x2].y : tc[o][x2].x) : 0.0;
                        TK_GRAM_ACC(v, tt)
                    }
            }
            continue;
        }
        // GQ row quads' loads in flight before their MFMAs (pairs past k read 0; the odd
        // column k of the last pair is stale and masked)
#pragma unroll 1
        for (int q0 = 0; q0 < 16; q0 += GQ) {
            d2_t x[GQ];
            double y[GQ][NC16 > 0 ? NC16 : 1];
            d2_t tl[GQ][NTP > 0 ? NTP : 1];
#pragma unroll
            for (int q = 0; q < GQ; ++q) {
                const uint32_t row = (uint32_t)(gq + (q0 + q) * 4);
                x[q] = bld2(tv, ((uint32_t)ci * TPB + row) * 16u);
#pragma unroll
                for (int g = 0; g < NC16; ++g) y[q][g] = bld(tv, cofs(32 + 16 * g + ci) + row * 16u);
#pragma unroll
                for (int p = 0; p < NTP; ++p) tl[q][p] = bld2(tv, ((uint32_t)(K0 / 2 + p) * TPB + row) * 16u);
            }
#pragma unroll
            for (int q = 0; q < GQ; ++q) {
                double v[NGR], tt[TA];
                v[0] = ev ? x[q].x : 0.0;
                v[1] = od ? x[q].y : 0.0;
#pragma unroll
                for (int g = 0; g < NC16; ++g) v[2 + g] = cm[g] ? y[q][g] : 0.0;
#pragma unroll
                for (int x2 = 0; x2 < TA; ++x2) tt[x2] = TAIL > 0 ? ((x2 & 1) ? tl[q][x2 >> 1].y : tl[q][x2 >> 1].x) : 0.0;
                TK_GRAM_ACC(v, tt)
            }
        }
    }
#undef TK_GRAM_ACC
    // waves 0, 1, 2, 3 summed in this order
    for (int ww = 0; ww < 4; ++ww) {
        if (w == ww) {
#pragma unroll
            for (int i = 0; i < NT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int e = (i * 4 + r) * 64 + lane;
                    red[e] = ww == 0 ? acc[i][r] : red[e] + acc[i][r];
                }
        }
        __syncthreads();
    }
    double* trd = red + NT * 256;
    if (TAIL > 0) {
#pragma unroll
        for (int x2 = 0; x2 < TA; ++x2)
#pragma unroll
            for (int s = 0; s < NS; ++s) trd[((x2 * NS + s) * 4 + w) * 64 + lane] = tac[x2][s];
        __syncthreads();
    }
    auto out = GP(double, Pg) + (int64_t)blockIdx.x * (NT * 256 + (TAIL > 0 ? 256 : 0));
    for (int e = threadIdx.x; e < NT * 256; e += 256) out[e] = red[e];
    if (TAIL > 0) {
        // entry (x2, c): slot s and lane column of the products that formed it, summed over
        // waves and row slots in fixed order
        const int x2 = threadIdx.x >> 6, c = threadIdx.x & 63;
        double sum = 0.0;
        if (x2 < TAIL && c < K0 + TAIL) {
            int s, cc;
            if (c < 32) { s = c & 1; cc = c >> 1; }
            else if (c < K0) { s = 2 + ((c - 32) >> 4); cc = (c - 32) & 15; }
            else { s = NGR; cc = c - K0; }
            for (int ww = 0; ww < 4; ++ww)
                for (int r = 0; r < 4; ++r) sum += trd[((x2 * NS + s) * 4 + ww) * 64 + r * 16 + cc];
        }
        out[NT * 256 + threadIdx.x] = sum;
    }
}

// out[v] = sum over the nb block partials P[b][v] in one launch: 32 threads per value, thread s
// summing partials [s*seg, (s+1)*seg) in order, then the 32 segment sums in order (fixed order
// for a given nb, so bitwise reproducible); 8 values per block, lanes of a value group read
// 8 consecutive values of one partial row
__global__ __launch_bounds__(256) void k_gram_reduce(const double* __restrict__ P, int nb, int nv,
                                                     double* __restrict__ out) {
    __shared__ double ss[32][8];
    const int vv = threadIdx.x & 7, sg = threadIdx.x >> 3;
    const int v = blockIdx.x * 8 + vv;
    const int seg = (nb + 31) / 32, b0 = sg * seg, b1 = min(nb, b0 + seg);
    double s = 0.0;
    if (v < nv)
        for (int b = b0; b < b1; ++b) s += ld(P, (int64_t)b * nv + v);
    ss[sg][vv] = s;
    __syncthreads();
    if (sg == 0 && v < nv) {
        double r = 0.0;
        for (int q = 0; q < 32; ++q) r += ss[q][vv];
        st(out, v, r);
    }
}

// ------------------------------------------------------------------ plain SpMV (test hook)
template <int FMT>
__global__ __launch_bounds__(TPB) void k_spmv(SpM A, const double* __restrict__ x, double* __restrict__ y) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r < A.n) st(y, r, spmv<FMT>(A, r, [=](int64_t c) { return ld(x, c); }));
}

// ------------------------------------------------------------------ tile-major gather/scatter
// out[c*n + r] = V[r, c0 + c] for one factor (column extraction for the ABI)
__global__ __launch_bounds__(TPB) void k_get_cols(const double* __restrict__ V, int64_t n, int kmax,
                                                  int c0, int nc, double* __restrict__ out, int sl) {
    const int64_t TS = (int64_t)TPB * kcp(kmax);
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    const int c = blockIdx.y;
    const int64_t o = sl ? svofs(c0 + c, (int)(r & 255)) : vofs(c0 + c, (int)(r & 255));
    if (r < n && c < nc) st(out, (int64_t)c * n + r, ld(V, (r >> 8) * TS + o));
}

// ------------------------------------------------------------------ launchers

static size_t lds_bytes(int nv, int kmax, int ncoef) {
    return (size_t)(ncoef * COEF_PAD(kmax) + ((nv + 32 + 15) & ~15)) * sizeof(double);
}

// The register row is sized to the step's column count in steps of 8: out-of-range
// columns cost a load issue each even though the range check fetches nothing, and the
// unused registers lower occupancy (tools/bwprobe.hip: 12 columns with a 48-register row
// streamed at 3.5 TB/s, with a 16-register row at 5.6 TB/s).
template <int V>
using IC = std::integral_constant<int, V>;
template <class F>
static void with_maxc(int nc, F f) {
    if (nc <= 8) f(IC<8>{});
    else if (nc <= 16) f(IC<16>{});
    else if (nc <= 24) f(IC<24>{});
    else if (nc <= 32) f(IC<32>{});
    else if (nc <= 40) f(IC<40>{});
    else if (nc <= 48) f(IC<48>{});
    else if (nc <= 56) f(IC<56>{});
    else f(IC<64>{});
}
template <class F>
static void with_fmt(int fmt, F f) {
    switch (fmt) {
        case SPM_DIA: f(IC<SPM_DIA>{}); break;
        case SPM_SELL: f(IC<SPM_SELL>{}); break;
        case SPM_CSR: f(IC<SPM_CSR>{}); break;
        case SPM_DIAN: f(IC<SPM_DIAN>{}); break;
        case SPM_DIAT: f(IC<SPM_DIAT>{}); break;
        default: f(IC<SPM_ANY>{}); break;
    }
}

void launch_init_a(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    hipLaunchKernelGGL(k_init_a, dim3(a.npart, nf), dim3(TPB), lds_bytes(1, a.kmax, 0), s, F, a);
}
void launch_init_b(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    hipLaunchKernelGGL(k_init_b, dim3(a.npart, nf), dim3(TPB), lds_bytes(2, a.kmax, 0), s, F, a);
}
void launch_arn_a1_plain(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const size_t lds = lds_bytes(a.j + 1, a.kmax, 0);
    auto go = [&](auto FM) {
        with_maxc(a.j + 1, [&](auto M) {
            hipLaunchKernelGGL((k_arn_a1_plain<decltype(M)::value, decltype(FM)::value>), dim3(a.npart, nf),
                               dim3(TPB), lds, s, F, a);
        });
    };
    if (a.mfs) go(IC<SPM_PRE>{});   // A v_j from k_spmv_mf
    else with_fmt(a.fmt, go);
}
void launch_spmv_mf(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    hipLaunchKernelGGL(k_ilv, dim3((int)(a.ld / TPB)), dim3(TPB), 0, s, F, nf, a.ld);
    const int nb = (int)((a.ld + TPB / 4 - 1) / (TPB / 4));
    auto go = [&](auto FM) {
        constexpr int FMv = decltype(FM)::value;
        switch (nf) {   // the group size is a template parameter (2..8 factors)
            case 2: hipLaunchKernelGGL((k_spmv_mf<FMv, 2>), dim3(nb), dim3(TPB), 0, s, F, nf, a); break;
            case 3: hipLaunchKernelGGL((k_spmv_mf<FMv, 3>), dim3(nb), dim3(TPB), 0, s, F, nf, a); break;
            case 4: hipLaunchKernelGGL((k_spmv_mf<FMv, 4>), dim3(nb), dim3(TPB), 0, s, F, nf, a); break;
            case 5: hipLaunchKernelGGL((k_spmv_mf<FMv, 5>), dim3(nb), dim3(TPB), 0, s, F, nf, a); break;
            case 6: hipLaunchKernelGGL((k_spmv_mf<FMv, 6>), dim3(nb), dim3(TPB), 0, s, F, nf, a); break;
            case 7: hipLaunchKernelGGL((k_spmv_mf<FMv, 7>), dim3(nb), dim3(TPB), 0, s, F, nf, a); break;
            default: hipLaunchKernelGGL((k_spmv_mf<FMv, 8>), dim3(nb), dim3(TPB), 0, s, F, nf, a); break;
        }
    };
    if (a.fmt == SPM_SELL) go(IC<SPM_SELL>{});
    else go(IC<SPM_CSR>{});
}
void launch_arn_a1_fused(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const size_t lds = lds_bytes(a.j + 1, a.kmax, TK_A1_SCALAR ? 0 : 2);
    auto go = [&](auto FM) {
        with_maxc(a.j, [&](auto M) {
            hipLaunchKernelGGL((k_arn_a1_fused<decltype(M)::value, decltype(FM)::value>), dim3(a.npart, nf),
                               dim3(TPB), lds, s, F, a);
        });
    };
    if (a.mfs) go(IC<SPM_PRE>{});   // A U from k_spmv_mf
    else with_fmt(a.fmt, go);
}
void launch_arn_a2(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const size_t lds = lds_bytes(2 * a.j + 4, a.kmax, TK_A2_SCALAR ? 0 : 1);
    with_maxc(a.j + 1, [&](auto M) {
        hipLaunchKernelGGL((k_arn_a2<decltype(M)::value>), dim3(a.npart, nf), dim3(TPB), lds, s, F, a);
    });
}
void launch_arn_finalize(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const size_t lds = lds_bytes(a.j + 3, a.kmax, TK_A2_SCALAR ? 0 : 1);
    with_maxc(a.j + 1, [&](auto M) {
        hipLaunchKernelGGL((k_arn_finalize<decltype(M)::value>), dim3(a.npart, nf), dim3(TPB), lds, s, F, a);
    });
}
// the one-sweep kernels exist for banded storage only (the host routes other formats to CGS2)
template <class F>
static void with_band_fmt(int fmt, F f) {
    if (fmt == SPM_DIAT) f(IC<SPM_DIAT>{});
    else f(IC<SPM_DIA>{});
}
void launch_init_bd(const DFac* F, int nf, const KArgs& a, int npd, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    with_band_fmt(a.fmt, [&](auto FM) {
        hipLaunchKernelGGL((k_init_bd<decltype(FM)::value>), dim3(npd, nf), dim3(TPB), lds_bytes(3, a.kmax, 0), s, F, a);
    });
}
void launch_lan_1s(const DFac* F, int nf, const KArgs& a, int npd, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const int M = a.j <= 8 ? 8 : (a.j + 7) / 8 * 8;
    const size_t lds = (size_t)(1 + (M + 15) / 16) * 64 * sizeof(double);
    with_band_fmt(a.fmt, [&](auto FM) {
        with_maxc(a.j, [&](auto M) {
            hipLaunchKernelGGL((k_lan_1s<decltype(M)::value, decltype(FM)::value>), dim3((npd + 7) / 8 * 8, nf),
                               dim3(TPB), lds, s, F, a);
        });
    });
}
void launch_red_lan(const DFac* F, int nf, const KArgs& ax, hipStream_t s) {
    if (nf <= 0) return;
    hipLaunchKernelGGL(k_red_lan, dim3(nf), dim3(1024), 0, s, F, ax);
}
void launch_lan_1w(const DFac* F, int nf, const KArgs& a, const KArgs& b, int npd, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const dim3 grid((npd + 7) / 8 * 8 + (b.j >= 0 ? 8 : 0), nf);
    with_band_fmt(a.fmt, [&](auto FM) {
        if (a.sl) hipLaunchKernelGGL((k_lan_1w<decltype(FM)::value, true>), grid, dim3(TPB), 64 * sizeof(double), s, F, a, b);
        else hipLaunchKernelGGL((k_lan_1w<decltype(FM)::value, false>), grid, dim3(TPB), 64 * sizeof(double), s, F, a, b);
    });
}
void launch_arn_d1(const DFac* F, int nf, const KArgs& a0, const KArgs& b, int npd, bool gram, bool vcache,
                   bool fuse, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const KArgs& a = a0;
    // per-lane accumulators: register-row chunks (u,z) + scalars + Gram chunks; with the
    // previous step's bookkeeping (b.j >= 0) at least its Hbar + reduced dots
    const int M = a.j <= 8 ? 8 : (a.j + 7) / 8 * 8;
    // column-dot slots: (u,z) chunks + scalars (+ Gram chunks)
    size_t lds = ((size_t)(M / 8 + 1 + (gram ? (M + 15) / 16 : 0)) * D1_CHW) * sizeof(double);
    if (b.j >= 0) lds = std::max(lds, bk_lds_doubles(b.j) * sizeof(double));
    // (fused with a pending reduce: nf * (3j + 3) leading reducer blocks, rounded to whole XCD rounds)
    const int xr = (fuse && a.red) ? (nf * (3 * a.j + 3) + 7) & ~7 : 0;
    const int gx = xr + (npd + 7) / 8 * 8 + (b.j >= 0 ? 8 : 0);
    with_band_fmt(a.fmt, [&](auto FM) {
        with_maxc(a.j, [&](auto M) {
            constexpr int MV = decltype(M)::value, FV = decltype(FM)::value;
            if (fuse) {
                if (vcache) hipLaunchKernelGGL((k_arn_d1<MV, FV, 3>), dim3(gx, nf), dim3(TPB), lds, s, F, a, b);
                else hipLaunchKernelGGL((k_arn_d1<MV, FV, 2>), dim3(gx, nf), dim3(TPB), lds, s, F, a, b);
            } else if (a.wsc) {
                if (vcache) hipLaunchKernelGGL((k_arn_d1<MV, FV, 5>), dim3(gx, nf), dim3(TPB), lds, s, F, a, b);
                else hipLaunchKernelGGL((k_arn_d1<MV, FV, 4>), dim3(gx, nf), dim3(TPB), lds, s, F, a, b);
            } else {
                if (vcache) hipLaunchKernelGGL((k_arn_d1<MV, FV, 1>), dim3(gx, nf), dim3(TPB), lds, s, F, a, b);
                else hipLaunchKernelGGL((k_arn_d1<MV, FV, 0>), dim3(gx, nf), dim3(TPB), lds, s, F, a, b);
            }
        });
    });
}
void launch_lan_l1_plain(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const size_t lds = lds_bytes(1, a.kmax, 0);
    with_fmt(a.fmt, [&](auto FM) {
        hipLaunchKernelGGL((k_lan_l1_plain<decltype(FM)::value>), dim3(a.npart, nf), dim3(TPB), lds, s, F, a);
    });
}
void launch_lan_d1(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const int M = a.j <= 8 ? 8 : (a.j + 7) / 8 * 8;
    const size_t lds = (size_t)((M + 15) / 16 + 1) * TPB * sizeof(double);
    const dim3 grid((a.ntiles + 7) / 8 * 8, nf);
    with_fmt(a.fmt, [&](auto FM) {
        with_maxc(a.j, [&](auto Mc) {
            hipLaunchKernelGGL((k_lan_d1<decltype(Mc)::value, decltype(FM)::value>), grid, dim3(TPB), lds, s, F, a);
        });
    });
}
void launch_lan_l1_fused(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const size_t lds = lds_bytes(a.j + 3, a.kmax, 0);
    with_fmt(a.fmt, [&](auto FM) {
        hipLaunchKernelGGL((k_lan_l1_fused<decltype(FM)::value>), dim3(a.npart, nf), dim3(TPB), lds, s, F, a);
    });
}
void launch_lan_l2(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    hipLaunchKernelGGL(k_lan_l2, dim3(a.npart, nf), dim3(TPB), lds_bytes(1, a.kmax, 0), s, F, a);
}
void launch_fin_d(const DFac* F, int nf, const KArgs& a, int mode, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const int nc = a.j + 1;
    const int M = nc <= 8 ? 8 : (nc + 7) / 8 * 8;
    const size_t lds = (size_t)((M + 15) / 16 + 1) * TPB * sizeof(double);
    const dim3 grid((a.ntiles + 7) / 8 * 8, nf);
    with_maxc(nc, [&](auto Mc) {
        if (mode == 0) hipLaunchKernelGGL((k_fin_d<decltype(Mc)::value, 0>), grid, dim3(TPB), lds, s, F, a);
        else if (mode == 1) hipLaunchKernelGGL((k_fin_d<decltype(Mc)::value, 1>), grid, dim3(TPB), lds, s, F, a);
        else hipLaunchKernelGGL((k_fin_d<decltype(Mc)::value, 2>), grid, dim3(TPB), lds, s, F, a);
    });
}
void launch_fin_vy(const DFac* F, int nf, const KArgs& a, const double* Y, double* X, int ldy, int t, int mode,
                   hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const int nc = a.j + 1;
    const int M = nc <= 8 ? 8 : (nc + 7) / 8 * 8;
    const size_t lds = ((size_t)((M + 15) / 16 + 1) * TPB + (size_t)t * ldy) * sizeof(double);   // acc + Y_s
    const dim3 grid((a.ntiles + 7) / 8 * 8, nf);
    with_maxc(nc, [&](auto Mc) {
        if (mode == 2 && a.sl) hipLaunchKernelGGL((k_fin_vy<decltype(Mc)::value, 2, true>), grid, dim3(TPB), lds, s, F, a, Y, X, ldy, t);
        else if (mode == 2) hipLaunchKernelGGL((k_fin_vy<decltype(Mc)::value, 2, false>), grid, dim3(TPB), lds, s, F, a, Y, X, ldy, t);
        else hipLaunchKernelGGL((k_fin_vy<decltype(Mc)::value, 0, false>), grid, dim3(TPB), lds, s, F, a, Y, X, ldy, t);
    });
}
void launch_lan_finalize(const DFac* F, int nf, const KArgs& a, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    hipLaunchKernelGGL(k_lan_finalize, dim3(a.npart, nf), dim3(TPB), lds_bytes(a.j + 3, a.kmax, 0), s, F, a);
}
// the reduce hand-off form of this process: TK_RED_MM at build time, then tk_abi.cpp's
// startup self-check (or TKHIP_RED_MM) may switch it to the memory-model form
static std::atomic<int> g_red_mm{TK_RED_MM};
int red_mm() { return g_red_mm.load(std::memory_order_relaxed); }
void set_red_mm(int on) { g_red_mm.store(on ? 1 : 0, std::memory_order_relaxed); }

void launch_red_d1(const DFac* F, int nf, int which, int J, int npd, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    (void)npd;
    const dim3 grid(d1_groups(d1_nv(J, 1)) * 16, nf);
    if (red_mm()) hipLaunchKernelGGL(k_red_d1<true>, grid, dim3(256), 0, s, F, which, J);
    else hipLaunchKernelGGL(k_red_d1<false>, grid, dim3(256), 0, s, F, which, J);
}
void launch_reduce(const DFac* F, int nf, int which, int nv, int npart, hipStream_t s, int gate, int coefJ,
                   const KArgs* ax) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    KArgs none;
    memset(&none, 0, sizeof(none));
    if (npart <= 0 && !gate) {
        if (red_mm())
            hipLaunchKernelGGL(k_reduce256<true>, dim3(nv, nf), dim3(256), 0, s, F, which, nv, 0, coefJ, ax ? *ax : none);
        else
            hipLaunchKernelGGL(k_reduce256<false>, dim3(nv, nf), dim3(256), 0, s, F, which, nv, 0, coefJ, ax ? *ax : none);
    } else if (npart > 1024 && !gate) {   // one partial per tile (k_fin_d)
        hipLaunchKernelGGL(k_reduce256<false>, dim3(nv, nf), dim3(256), 0, s, F, which, nv, npart, -1, none);
    }
    else
        hipLaunchKernelGGL(k_reduce, dim3(nv, nf), dim3(64), 0, s, F, which, nv, npart, gate);
}
// Multi-rank host mirror of one all-reduced group of record slots (runs on the exchange
// stream after the all-reduce): copy the slots to host-mapped coherent memory, then publish
// their sequence number, so the host reads the records without any queue call.
__global__ __launch_bounds__(TPB) void k_mirror_records(const double* __restrict__ src, double* dst, int cnt,
                                                        unsigned long long* done, int nslots, unsigned long long seq) {
    // (system-scope stores go through to host memory: each thread's completed stores are all
    // the sequence words must follow; no system-scope fence and its L2 writeback beside the
    // compute kernels)
    for (int i = threadIdx.x; i < cnt; i += TPB)
        __hip_atomic_store(dst + i, ld(src, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0)
        for (int q = 0; q < nslots; ++q) __hip_atomic_store(done + q, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Test-only latency stand-in (TKHIP_TEST_XCH_DELAY_US, tk_abi.cpp exchange_range): one wave
// that waits `ticks` of the 100 MHz wall clock on the exchange stream ahead of an all-reduce,
// so a 1-rank communicator's exchange takes as long as an 8-peer one would.
// Nothing is read or written.
__global__ __launch_bounds__(64) void k_delay(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}
void launch_delay_us(double us, hipStream_t s) {
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, (uint64_t)(us * 100.0 + 0.5));
}
void launch_mirror_records(const double* src, double* dst, int cnt, unsigned long long* done, int nslots,
                           unsigned long long seq, hipStream_t s) {
    hipLaunchKernelGGL(k_mirror_records, dim3(1), dim3(TPB), 0, s, src, dst, cnt, done, nslots, seq);
}

void launch_post(const DFac* F, int nf, const KArgs& a, int kind, int flag, int clear, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    const size_t hb = (size_t)(a.kmax + 1) * (a.kmax + 2);
    size_t lds = (kind == POST_ARN && hb <= POST_LDS_MAX) ? hb * sizeof(double) : 0;
    if (kind == POST_ARN_D) lds = bk_lds_doubles(a.j) * sizeof(double);
    hipLaunchKernelGGL(k_post, dim3(nf), dim3(TPB), lds, s, F, a, kind, flag, clear);
}
void launch_basis_mul(const DFac* F, int nf, const KArgs& a, const double* Y, double* X, int k,
                      int t, hipStream_t s) {
    if (nf <= 0) return;   // (a rank that owns no factors launches nothing)
    // 16-column MFMA groups; t mod 16 <= 4 leftover columns go to the VALU tail instead of a
    // padded group.  Slices of 32 columns (blockIdx.z); the last slice holds the rest.
    int ng = t / 16, tl = t % 16;
    if (tl > 4) {
        ++ng;
        tl = 0;
    }
    const int nz = ng > 2 ? (ng - 1) / 2 : 0;   // full slices of two groups before the last
    const int ngl = ng - 2 * nz;                // groups of the last slice (0, 1 or 2)
    if (nz > 0 && a.sl)
        hipLaunchKernelGGL((k_basis_mul<2, 0, true>), dim3(a.ntiles, nf, nz), dim3(256), 0, s, F, a, Y, X, k, t, 0);
    else if (nz > 0)
        hipLaunchKernelGGL((k_basis_mul<2, 0, false>), dim3(a.ntiles, nf, nz), dim3(256), 0, s, F, a, Y, X, k, t, 0);
#define TK_BM_CASE(G_, L_)                                                                             \
    if (ngl == G_ && tl == L_ && a.sl)                                                                \
        hipLaunchKernelGGL((k_basis_mul<G_, L_, true>), dim3(a.ntiles, nf, 1), dim3(256), 0, s, F, a, Y, X, k, t, nz); \
    else if (ngl == G_ && tl == L_)                                                                   \
        hipLaunchKernelGGL((k_basis_mul<G_, L_, false>), dim3(a.ntiles, nf, 1), dim3(256), 0, s, F, a, Y, X, k, t, nz);
    TK_BM_CASE(0, 1) TK_BM_CASE(0, 2) TK_BM_CASE(0, 3) TK_BM_CASE(0, 4)
    TK_BM_CASE(1, 0) TK_BM_CASE(1, 1) TK_BM_CASE(1, 2) TK_BM_CASE(1, 3) TK_BM_CASE(1, 4)
    TK_BM_CASE(2, 0) TK_BM_CASE(2, 1) TK_BM_CASE(2, 2) TK_BM_CASE(2, 3) TK_BM_CASE(2, 4)
#undef TK_BM_CASE
}
#ifndef TK_GRAM_BLOCKS
#define TK_GRAM_BLOCKS 512    // k_gram blocks (2 per CU; A/B in profiles/r03/gram_ab.txt): a function of n only
#endif
// column groups of k_gram for k columns: NC16 runs of 16 beyond column 32, TAIL (<= 4) on the VALU
static void gram_config(int k, int& nc16, int& tail) {
    nc16 = 0;
    tail = 0;
    if (k <= 32) return;
    nc16 = (k - 32) / 16;
    tail = (k - 32) % 16;
    if (tail > 4) {   // a group of 16 with more than 4 live columns: padded MFMA group
        ++nc16;
        tail = 0;
    }
}
int gram_values(int k) {
    int nc16, tail;
    gram_config(k, nc16, tail);
    const int ngr = 2 + nc16;
    return ngr * (ngr + 1) / 2 * 256 + (tail ? 256 : 0);
}
int gram_blocks(int ntiles) { return ntiles < TK_GRAM_BLOCKS ? ntiles : TK_GRAM_BLOCKS; }
size_t gram_scratch_doubles(int ntiles) { return (size_t)(gram_blocks(ntiles) + 64 + 1) * 10 * 256; }
void gram_unpack(int k, const double* v, double* G) {
    int nc16, tail;
    gram_config(k, nc16, tail);
    const int ngr = 2 + nc16, k0 = 32 + 16 * nc16;
    auto col = [](int g, int x) { return g < 2 ? 2 * x + g : 32 + 16 * (g - 2) + x; };
    int i = 0;
    for (int ga = 0; ga < ngr; ++ga)
        for (int gb = ga; gb < ngr; ++gb, ++i)
            for (int r = 0; r < 4; ++r)
                for (int l = 0; l < 64; ++l) {
                    const int p = col(ga, (l >> 4) + 4 * r), q = col(gb, l & 15);
                    if (p >= k || q >= k) continue;
                    const double x = v[(size_t)(i * 4 + r) * 64 + l];
                    G[(size_t)q * k + p] = x;
                    G[(size_t)p * k + q] = x;
                }
    const double* tv = v + (size_t)i * 256;
    for (int x = 0; x < tail; ++x)
        for (int c = 0; c <= k0 + x; ++c) {
            G[(size_t)(k0 + x) * k + c] = tv[x * 64 + c];
            G[(size_t)c * k + (k0 + x)] = tv[x * 64 + c];
        }
}
void launch_gram(const DFac* F, int f, const KArgs& a, int k, double* scratch, hipStream_t s) {
    const int nb = gram_blocks(a.ntiles), nv = gram_values(k);
    double* P = scratch;
    double* Q = P + (size_t)nb * nv;
    double* out = Q + (size_t)64 * nv;
    int nc16, tail;
    gram_config(k, nc16, tail);
#define TK_GRAM_CASE(A_, B_)                                                                       \
    if (nc16 == A_ && tail == B_ && a.sl) hipLaunchKernelGGL((k_gram<A_, B_, true>), dim3(nb), dim3(256), 0, s, F, a, f, k, P); \
    else if (nc16 == A_ && tail == B_) hipLaunchKernelGGL((k_gram<A_, B_, false>), dim3(nb), dim3(256), 0, s, F, a, f, k, P);
    TK_GRAM_CASE(0, 0) TK_GRAM_CASE(0, 1) TK_GRAM_CASE(0, 2) TK_GRAM_CASE(0, 3) TK_GRAM_CASE(0, 4)
    TK_GRAM_CASE(1, 0) TK_GRAM_CASE(1, 1) TK_GRAM_CASE(1, 2) TK_GRAM_CASE(1, 3) TK_GRAM_CASE(1, 4)
    TK_GRAM_CASE(2, 0)
#undef TK_GRAM_CASE
    (void)Q;
    hipLaunchKernelGGL(k_gram_reduce, dim3((nv + 7) / 8), dim3(256), 0, s, P, nb, nv, out);
}

void launch_spmv(const SpM& A, const double* x, double* y, hipStream_t s) {
    const int nb = (int)((A.n + TPB - 1) / TPB);
    const int fmt = A.ndiag > 0 ? (A.ndiag <= 4 ? (A.toep ? SPM_DIAT : SPM_DIA) : SPM_DIAN) : (A.sell ? SPM_SELL : SPM_CSR);
    with_fmt(fmt, [&](auto FM) {
        hipLaunchKernelGGL((k_spmv<decltype(FM)::value>), dim3(nb), dim3(TPB), 0, s, A, x, y);
    });
}
void launch_get_cols(const double* V, int64_t n, int kmax, int c0, int nc, double* out, int sl, hipStream_t s) {
    const int nb = (int)((n + TPB - 1) / TPB);
    hipLaunchKernelGGL(k_get_cols, dim3(nb, nc), dim3(TPB), 0, s, V, n, kmax, c0, nc, out, sl);
}

}  // namespace tk

#if TK_D1_TRACE
extern "C" int tk_debug_d1_trace(int j, uint64_t* out, int n) {
    if (!out) return (int)hipMemcpyToSymbol(HIP_SYMBOL(tk::g_trace_j), &j, sizeof(int));
    hipDeviceSynchronize();
    const int m = n < TRACE_MAX ? n : TRACE_MAX;
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(tk::g_trace), sizeof(uint64_t) * 3 * m);
    if (e == hipSuccess) e = hipMemcpyFromSymbol(out + 3 * m, HIP_SYMBOL(tk::g_trace_ph), sizeof(uint64_t) * 4 * m);
    return (int)e;
}
#endif
