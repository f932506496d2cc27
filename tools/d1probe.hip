// Ceiling of k_arn_d1's exact memory traffic: the one-sweep Arnoldi step's
// loads and stores with its launch geometry, and no arithmetic beyond what keeps the loads
// alive.  Per block one window of WS = 256 - 2(hl + hu) rows at S = w*WS - 2hl (tridiagonal:
// 252 rows), XCD-aware slots, the row's j basis columns as 16-byte pairs from the paired-column
// tiles (non-temporal, as k_arn_d1 at C2 N = 1), u_j read, u_{j+1} and the v_j pair (odd j; E
// for even j) stored write-through on the owned rows, 3j+6 partials per window stored.
// Algorithmic bytes per factor-step: 8n(j + 3).
// Modes: 1 = one launch over all nf factors; 2 = two launches of nf/2 factors each on two
// streams (k_arn_d1's two factor groups); "rd" = loads only.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/d1probe.hip -o tools/_build/d1probe
// Run:   tools/_build/d1probe [n=2^20] [nf=8] [kmax=50] [variant ...]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define TPB 256
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef double d2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ rsrc_t mkrsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void st_wt(double* p, int64_t i, double v) {
    __hip_atomic_store(p + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Fac {
    const double* V;
    const double* Uin;
    double* Uout;
    double* E;
    double* P;
};

// the k_arn_d1 occupancy tiers (waves / SIMD by register-row width)
#define OCC(M) ((M) <= 8 ? 8 : ((M) <= 16 ? 6 : ((M) <= 24 ? 5 : ((M) <= 40 ? 4 : ((M) <= 56 ? 3 : 2)))))

// variant bits (the store side): 1 no partial stores, 2 partials with plain stores (not sc1),
// 4 u / E stored as 16-byte row pairs by the even lanes (the odd lane's value over DPP),
// 8 u / v / E with plain stores
template <int MAXC, bool STORE, int BS>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(OCC(MAXC), OCC(MAXC)))) void k_probe(
    const Fac* __restrict__ F, int64_t n, int64_t ld, int ntiles, int kmax, int j, int nwin, int npd, int var,
    int xx = 0, int xoff = 0, int xnv = 0) {
    const Fac& d = F[blockIdx.y];
    // (xx > 0: leading blocks sum the npd partials of value x of factor F[xoff + y] first -- the
    // other group's reduce inside this launch)
    if ((int)blockIdx.x < xx) {
        if ((int)blockIdx.x < xnv) {
            const Fac& xd = F[xoff + (int)blockIdx.y];   // (xoff < 0 for the second group: int arithmetic)
            const double* P = xd.P + (int64_t)blockIdx.x * npd;
            double s = 0.0;
            for (int b = threadIdx.x; b < npd; b += BS) s += __builtin_nontemporal_load(P + b);
            if (s == 12345.678) st_wt(xd.P, 0, s);
        }
        return;
    }
    const int bx = (int)blockIdx.x - xx;
    const int slot = (bx & 7) * (((int)gridDim.x - xx) >> 3) + (bx >> 3);
    if (slot >= nwin) return;
    const int t = threadIdx.x, hl = 1, hu = 1, WS = BS - 2 * (hl + hu);
    const int64_t TS = (int64_t)TPB * ((kmax + 2) & ~1);
    const rsrc_t tv = mkrsrc(d.V, (uint32_t)(ntiles * TS * 8));
    const int64_t S = (int64_t)slot * WS - 2 * hl, r = S + t;
    const bool inb = r >= 0 && r < ld, ok = r >= 0 && r < n;
    const uint32_t toff = inb ? (uint32_t)((r >> 8) * TS * 8 + (r & 255) * 16) : 0x80000000u;
    const int jl = j & ~1;
    d2_t v[MAXC / 2];
#pragma unroll
    for (int p = 0; p < MAXC / 2; ++p) {
        const uint32_t off = (p < MAXC / 2 - 4 || 2 * p < jl) ? toff + (uint32_t)p * (TPB * 16) : 0x80000000u;
        v[p] = __builtin_bit_cast(d2_t, __builtin_amdgcn_raw_buffer_load_b128(tv, off, 0, 2));
    }
    const double up = inb ? d.Uin[r] : 0.0;
    const double e = (inb && (j & 1)) ? d.E[r] : 0.0;
    double s = up + e;
#pragma unroll
    for (int p = 0; p < MAXC / 2; ++p) s += v[p].x + v[p].y;
    if (!STORE) {
        if (s == 12345.678) st_wt(d.P, slot, s);
        return;
    }
    const bool own = ok && t >= 2 * hl && t < BS - 2 * hu;
    const bool wt = !(var & 8);
    if (var & 4) {
        // rows r, r+1 as one 16-byte store by the even lane (S is even: r even <=> t even); a
        // pair's rows are owned together except at the window edges, where the owner stores 8 B
        const double su = s * 0.5;
        const double nu = __shfl_down(su, 1), ns = __shfl_down(s, 1);
        const bool own1 = (r + 1) < n && (t + 1) >= 2 * hl && (t + 1) < BS - 2 * hu;
        if (!(t & 1)) {
            if (own && own1) {
                const d2_t xu = {su, nu}, xe = {s, ns};
                const rsrc_t ru = mkrsrc(d.Uout, (uint32_t)(ld * 8)), re = mkrsrc(d.E, (uint32_t)(ld * 8));
                const uint32_t bo = (uint32_t)(r * 8);
                if (wt) {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, xu), ru, bo, 0, 16);
                    if (!(j & 1)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, xe), re, bo, 0, 16);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, xu), ru, bo, 0, 0);
                    if (!(j & 1)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, xe), re, bo, 0, 0);
                }
            } else if (own) {
                st_wt(d.Uout, r, su);
                if (!(j & 1)) st_wt(d.E, r, s);
            }
        } else if (own && !(r - 1 >= 0 && (t - 1) >= 2 * hl)) {
            st_wt(d.Uout, r, su);
            if (!(j & 1)) st_wt(d.E, r, s);
        }
        if (own && (j & 1)) {
            const d2_t x = {s, up};
            if (wt) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, x), tv,
                                                           toff + (uint32_t)(j >> 1) * (TPB * 16), 0, 16);
            else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, x), tv,
                                                        toff + (uint32_t)(j >> 1) * (TPB * 16), 0, 0);
        }
    } else if (own) {
        if (j & 1) {
            const d2_t x = {s, up};
            if (wt) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, x), tv,
                                                           toff + (uint32_t)(j >> 1) * (TPB * 16), 0, 16);
            else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, x), tv,
                                                        toff + (uint32_t)(j >> 1) * (TPB * 16), 0, 0);
        } else {
            if (wt) st_wt(d.E, r, s);
            else d.E[r] = s;
        }
        if (wt) st_wt(d.Uout, r, s * 0.5);
        else d.Uout[r] = s * 0.5;
    }
    // the window's 3j + 6 partials (one store per value, spread over the block's threads)
    if (var & 64) {
        // slot-major groups of 16 values: each group of a window one whole 128-byte line
        for (int vi = t; vi < 3 * j + 6; vi += BS) st_wt(d.P, ((int64_t)(vi >> 4) * npd + slot) * 16 + (vi & 15), s);
    } else if (!(var & 1))
        for (int vi = t; vi < 3 * j + 6; vi += BS) {
            if (var & 2) d.P[(int64_t)vi * npd + slot] = s;
            else st_wt(d.P, (int64_t)vi * npd + slot, s);
        }
}

// a stand-in for the step's reduce: block (c, f) sums value c's npd window partials
__global__ __launch_bounds__(256) void k_red_probe(const Fac* __restrict__ F, int npd, double* out) {
    const double* P = F[blockIdx.y].P + (int64_t)blockIdx.x * npd;
    double s = 0.0;
    for (int b = threadIdx.x; b < npd; b += 256) s += __builtin_nontemporal_load(P + b);
    if (s == 12345.678) out[blockIdx.x] = s;   // (never: keeps the loads)
}
static void launch_red(const Fac* F, int nf, int nv, int npd, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_red_probe, dim3(nv, nf), dim3(256), 0, s, F, npd, out);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static int g_var = 0, g_bs = 256;
static int g_xoff = 0, g_xnv = 0;   // (mode 8: the other group's reduce in the leading blocks)
template <bool STORE, int BS>
static void launch_bs(int M, const Fac* F, int nf, int64_t n, int64_t ld, int ntiles, int kmax, int j, int npd,
                      hipStream_t s) {
    const int nwin = (int)((n + (BS - 4) - 1) / (BS - 4));
    const int xx = (g_xnv + 7) & ~7;
    dim3 g(xx + ((nwin + 7) & ~7), nf);
#define L_(MM) case MM: hipLaunchKernelGGL((k_probe<MM, STORE, BS>), g, dim3(BS), 0, s, F, n, ld, ntiles, kmax, j, nwin, npd, g_var, xx, g_xoff, g_xnv); break;
    switch (M) { L_(8) L_(16) L_(24) L_(32) L_(40) L_(48) L_(56) L_(64) }
#undef L_
}
// (variant bit 16: 512-row windows, bit 32: 1024-row windows -- fewer partials per row)
template <bool STORE>
static void launch(int M, const Fac* F, int nf, int64_t n, int64_t ld, int ntiles, int kmax, int j, int nwin, int npd,
                   hipStream_t s) {
    (void)nwin;
    if (g_var & 32) launch_bs<STORE, 1024>(M, F, nf, n, ld, ntiles, kmax, j, npd, s);
    else if (g_var & 16) launch_bs<STORE, 512>(M, F, nf, n, ld, ntiles, kmax, j, npd, s);
    else launch_bs<STORE, 256>(M, F, nf, n, ld, ntiles, kmax, j, npd, s);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atol(argv[1]) : (1 << 20);
    const int nf = argc > 2 ? atoi(argv[2]) : 8;
    const int kmax = argc > 3 ? atoi(argv[3]) : 50;
    const int64_t ld = (n + 255) & ~255;
    const int ntiles = (int)(ld / 256);
    const int WS = 252, nwin = (int)((n + WS - 1) / WS), npd = nwin;
    const int64_t TS = 256LL * ((kmax + 2) & ~1);
    std::vector<Fac> hf(nf);
    for (int f = 0; f < nf; ++f) {
        double *V, *U, *W, *E, *P;
        CK(hipMalloc(&V, (size_t)ntiles * TS * 8));
        CK(hipMalloc(&U, (size_t)ld * 8));
        CK(hipMalloc(&W, (size_t)ld * 8));
        CK(hipMalloc(&E, (size_t)ld * 8));
        CK(hipMalloc(&P, (size_t)npd * (3 * kmax + 8 + 16) * 8));
        CK(hipMemset(V, 0, (size_t)ntiles * TS * 8));
        CK(hipMemset(U, 0, (size_t)ld * 8));
        CK(hipMemset(W, 0, (size_t)ld * 8));
        CK(hipMemset(E, 0, (size_t)ld * 8));
        hf[f] = {V, U, W, E, P};
    }
    Fac* F;
    CK(hipMalloc(&F, nf * sizeof(Fac)));
    CK(hipMemcpy(F, hf.data(), nf * sizeof(Fac), hipMemcpyHostToDevice));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t a, b, jn;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreateWithFlags(&jn, hipEventDisableTiming));
    hipEvent_t ea, eb;
    CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
    CK(hipEventRecord(eb, s1));
    hipEvent_t ra, rb;
    CK(hipEventCreateWithFlags(&ra, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&rb, hipEventDisableTiming));
    CK(hipEventRecord(ra, s1));
    CK(hipEventRecord(rb, s1));
    double* dout;
    CK(hipMalloc(&dout, 4096 * sizeof(double)));
    const int nvar = argc > 4 ? argc - 4 : 1;
    printf("n=%ld nf=%d kmax=%d windows=%d (per-step algorithmic bytes 8n(j+3) per factor; TB/s)\n", (long)n, nf,
           kmax, nwin);
    for (int vi = 0; vi < nvar; ++vi) {
        g_var = argc > 4 ? atoi(argv[4 + vi]) : 0;
        printf("variant %d: %4s %4s %16s %16s %16s %16s %16s %16s %16s %16s %16s\n", g_var, "j", "MAXC", "1 launch", "2 groups+join",
               "2 groups", "loads only", "2 in sequence", "2 turns (events)", "seq + side reduces", "groups + reduces",
               "seq + in-launch reduces");
        for (int j = 4; j < kmax && j <= 63; j += 4) {
            const int M = j < 8 ? 8 : ((j + 7) / 8) * 8;
            const double bytes = 8.0 * n * (j + 3) * nf;
            float ms[9];
            for (int mode = 0; mode < 9; ++mode) {
                auto run = [&] {
                    if (mode == 1 || mode == 2) {
                        if (mode == 1) {
                            CK(hipEventRecord(jn, s0));
                            CK(hipStreamWaitEvent(s1, jn, 0));
                        }
                        launch<true>(M, F, nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                        launch<true>(M, F + nf / 2, nf - nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s1);
                        if (mode == 1) {
                            CK(hipEventRecord(jn, s1));
                            CK(hipStreamWaitEvent(s0, jn, 0));
                        }
                    } else if (mode == 0) {
                        launch<true>(M, F, nf, n, ld, ntiles, kmax, j, nwin, npd, s0);
                    } else if (mode == 4) {
                        // (the two groups' launches one after the other: groups taking turns)
                        launch<true>(M, F, nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                        launch<true>(M, F + nf / 2, nf - nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                    } else if (mode == 5) {
                        // (the same order from two streams: each launch waits for the other
                        // stream's last launch through an event, as factor groups taking turns)
                        CK(hipStreamWaitEvent(s0, eb, 0));
                        launch<true>(M, F, nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                        CK(hipEventRecord(ea, s0));
                        CK(hipStreamWaitEvent(s1, ea, 0));
                        launch<true>(M, F + nf / 2, nf - nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s1);
                        CK(hipEventRecord(eb, s1));
                    } else if (mode == 6) {
                        // sweeps back to back on one stream; each group's reduce on the side
                        // stream behind its sweep, and the group's next sweep behind that reduce
                        const int nv = 3 * j + 6;
                        CK(hipStreamWaitEvent(s0, ra, 0));
                        launch<true>(M, F, nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                        CK(hipEventRecord(ea, s0));
                        CK(hipStreamWaitEvent(s1, ea, 0));
                        launch_red(F, nf / 2, nv, npd, dout, s1);
                        CK(hipEventRecord(ra, s1));
                        CK(hipStreamWaitEvent(s0, rb, 0));
                        launch<true>(M, F + nf / 2, nf - nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                        CK(hipEventRecord(eb, s0));
                        CK(hipStreamWaitEvent(s1, eb, 0));
                        launch_red(F + nf / 2, nf - nf / 2, nv, npd, dout, s1);
                        CK(hipEventRecord(rb, s1));
                    } else if (mode == 8) {
                        // groups taking turns on one stream, each launch reducing the other group's
                        // last sweep in its leading blocks
                        g_xnv = 3 * j + 6;
                        g_xoff = nf / 2;
                        launch<true>(M, F, nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                        g_xoff = -(nf / 2);
                        launch<true>(M, F + nf / 2, nf - nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                        g_xnv = 0;
                        g_xoff = 0;
                    } else if (mode == 7) {
                        // today's factor groups: each group's sweep and reduce on its own stream
                        const int nv = 3 * j + 6;
                        launch<true>(M, F, nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s0);
                        launch_red(F, nf / 2, nv, npd, dout, s0);
                        launch<true>(M, F + nf / 2, nf - nf / 2, n, ld, ntiles, kmax, j, nwin, npd, s1);
                        launch_red(F + nf / 2, nf - nf / 2, nv, npd, dout, s1);
                    } else {
                        launch<false>(M, F, nf, n, ld, ntiles, kmax, j, nwin, npd, s0);
                    }
                };
                run();
                CK(hipDeviceSynchronize());
                const int reps = 20;
                CK(hipEventRecord(a, s0));
                CK(hipStreamWaitEvent(s1, a, 0));
                for (int i = 0; i < reps; ++i) run();
                CK(hipEventRecord(jn, s1));
                CK(hipStreamWaitEvent(s0, jn, 0));
                CK(hipEventRecord(b, s0));
                CK(hipEventSynchronize(b));
                float t;
                CK(hipEventElapsedTime(&t, a, b));
                ms[mode] = t / reps;
            }
            printf("           %4d %4d", j, M);
            for (int mode = 0; mode < 9; ++mode)
                printf(" %8.1f us %5.2f", ms[mode] * 1e3, bytes / (ms[mode] * 1e-3) / 1e12);
            printf("\n");
        }
    }
    return 0;
}
