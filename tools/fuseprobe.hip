// Price of moving the one-sweep step's reduce INTO the next step's launch (VERDICT r3 #1's
// target: the per-step kernel boundary + reduce launch at one factor per GPU), against the
// launch-based step the product runs (k_arn_d1, then k_reduce256, per step).
//
// Per step the product does: window blocks (nwin = 4161 at n = 2^20) stream their basis rows,
// read the previous step's reduced values, compute, and publish nv partials each; a reduce
// launch (one block per value) sums them in a fixed order and its last block publishes the
// scalars.  Modelled here with the same sizes:
//   launch  k_win (nwin blocks: stream SLAB bytes, read the nv values, publish nv partials)
//           + k_red (nv blocks: fixed-order sum over the partials, arrival count, the last
//           block bumps the step word) -- two launches per step, as the product
//   fused   ONE launch per step: blocks 0..nv-1 reduce the PREVIOUS step's partials (as
//           k_red); the window blocks issue their slab loads first, then wait for the step
//           word (bounded poll), then read the values and publish this step's partials
//           (ping-pong partial buffers).  The reduce blocks are the lowest block indices, so
//           they are dispatched before any window block: nothing they wait for is behind them.
// Every poll is bounded (2^22 tries): a wait that never ends sets an error word and the block
// goes on (the numbers are then void and say so) -- no hang.
// Build: hipcc -O3 --offload-arch=gfx950 tools/fuseprobe.hip -o tools/_build/fuseprobe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

#ifndef NWIN
#define NWIN 4161   // C2 at one factor (n = 2^20); -DNWIN=525 for C4 (n = 2^17, bandwidth 3)
#endif
#define SPIN_MAX (1 << 22)
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void st_ag(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ double ld_ag(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ double row16(double s) {
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    s += __shfl_xor(s, 8);
    return s;
}

// the window work: stream this block's slab (nld 16-byte loads per thread in flight), read the
// nv values, publish nv partials (one per value, thread v)
template <bool WAIT>
__device__ void window(const d2* __restrict__ X, int nld, const double* vals, double* P, int nv, int step,
                       const unsigned* word, unsigned* err) {
    const int w = blockIdx.x;
    const d2* slab = X + (size_t)w * nld * 256;
    d2 a[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) a[i] = i < nld ? __builtin_nontemporal_load(slab + i * 256 + threadIdx.x) : (d2){0.0, 0.0};
    if (WAIT) {
        __shared__ int ok;
        if (threadIdx.x == 0) {
            int spins = 0;
            while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)step && ++spins < SPIN_MAX)
                __builtin_amdgcn_s_sleep(1);
            ok = spins < SPIN_MAX;
            if (!ok) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 24; ++i) s += a[i].x * a[i].y;
    double v = 0.0;
    for (int c = threadIdx.x & 63; c < nv; c += 64) v += ld_ag(vals + c);
    s += 1e-30 * v;
    if (threadIdx.x < nv) st_ag(P + (size_t)threadIdx.x * NWIN + w, s + threadIdx.x);
}

// value c over the NWIN partials (24 loads per thread in flight, row sums, 16 in order), the
// arrival count; the last block bumps the step word to `step`
__device__ void reduce_value(const double* P, double* vals, int nv, unsigned* ctr, unsigned* word, unsigned step) {
    __shared__ double rs[16];
    __shared__ int last;
    const int c = blockIdx.x, t = threadIdx.x;
    double part[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) {
        const int b = t + 256 * i;
        part[i] = b < NWIN ? ld_ag(P + (size_t)c * NWIN + b) : 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 24; ++i) s += part[i];
    s = row16(s);
    if ((t & 15) == 0) rs[t >> 4] = s;
    __syncthreads();
    if (t == 0) {
        double r = 0.0;
        for (int q = 0; q < 16; ++q) r += rs[q];
        st_ag(vals + c, r);
        __builtin_amdgcn_s_waitcnt(0);
        last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nv - 1);
        if (last) {
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_s_waitcnt(0);
            __hip_atomic_store(word, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ __launch_bounds__(256) void k_win(const d2* X, int nld, const double* vals, double* P, int nv) {
    window<false>(X, nld, vals, P, nv, 0, nullptr, nullptr);
}
__global__ __launch_bounds__(256) void k_red(const double* P, double* vals, int nv, unsigned* ctr, unsigned* word, unsigned step) {
    reduce_value(P, vals, nv, ctr, word, step);
}
// blocks [0, nv): reduce the previous step's partials Pprev; blocks [nv, nv + NWIN): windows
__global__ __launch_bounds__(256) void k_fused(const d2* X, int nld, double* vals, const double* Pprev, double* P,
                                               int nv, unsigned* ctr, unsigned* word, unsigned step, unsigned* err) {
    if ((int)blockIdx.x < nv) {
        reduce_value(Pprev, vals, nv, ctr, word, step);
        return;
    }
    // (window index = blockIdx.x - nv)
    const int w = blockIdx.x - nv;
    const d2* slab = X + (size_t)w * nld * 256;
    d2 a[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) a[i] = i < nld ? __builtin_nontemporal_load(slab + i * 256 + threadIdx.x) : (d2){0.0, 0.0};
    __shared__ int ok;
    if (threadIdx.x == 0) {
        int spins = 0;
        while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < step && ++spins < SPIN_MAX)
            __builtin_amdgcn_s_sleep(1);
        ok = spins < SPIN_MAX;
        if (!ok) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 24; ++i) s += a[i].x * a[i].y;
    double v = 0.0;
    for (int c = threadIdx.x & 63; c < nv; c += 64) v += ld_ag(vals + c);
    s += 1e-30 * v;
    if (threadIdx.x < nv) st_ag(P + (size_t)threadIdx.x * NWIN + w, s + threadIdx.x);
}

int main() {
    CK(hipSetDevice(0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    printf("%s, %d CUs; nwin %d\n", prop.gcnArchName, prop.multiProcessorCount, NWIN);
    const int maxld = 24;
    d2* X;
    double *vals, *P0, *P1;
    unsigned *ctr, *word, *err;
    CK(hipMalloc(&X, (size_t)NWIN * maxld * 256 * sizeof(d2)));
    CK(hipMemset(X, 0, (size_t)NWIN * maxld * 256 * sizeof(d2)));
    CK(hipMalloc(&vals, 256 * 8));
    CK(hipMalloc(&P0, (size_t)128 * NWIN * 8));
    CK(hipMalloc(&P1, (size_t)128 * NWIN * 8));
    CK(hipMemset(P0, 0, (size_t)128 * NWIN * 8));
    CK(hipMemset(P1, 0, (size_t)128 * NWIN * 8));
    CK(hipMalloc(&ctr, 64));
    CK(hipMalloc(&word, 64));
    CK(hipMalloc(&err, 64));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int steps = 50;
    // slab per window: nld x 4 KiB (the basis row block of j columns: 252 rows x j x 8 B ~ j x 2 KiB)
    for (int nv : {52, 100}) {
        for (int nld : {6, 12, 24}) {
            float best_l = 1e9, best_f = 1e9;
            unsigned e = 0;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipMemsetAsync(ctr, 0, 64, s));
                CK(hipMemsetAsync(word, 0, 64, s));
                CK(hipEventRecord(a, s));
                for (int st = 1; st <= steps; ++st) {
                    hipLaunchKernelGGL(k_win, dim3(NWIN), dim3(256), 0, s, X, nld, vals, P0, nv);
                    hipLaunchKernelGGL(k_red, dim3(nv), dim3(256), 0, s, P0, vals, nv, ctr, word, (unsigned)st);
                }
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep) best_l = ms < best_l ? ms : best_l;
            }
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipMemsetAsync(ctr, 0, 64, s));
                CK(hipMemsetAsync(word, 0, 64, s));
                CK(hipMemsetAsync(err, 0, 64, s));
                CK(hipEventRecord(a, s));
                for (int st = 1; st <= steps; ++st) {
                    double* Pp = (st & 1) ? P0 : P1;
                    double* Pn = (st & 1) ? P1 : P0;
                    hipLaunchKernelGGL(k_fused, dim3(nv + NWIN), dim3(256), 0, s, X, nld, vals, Pp, Pn, nv, ctr, word,
                                       (unsigned)st, err);
                }
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
                if (e) break;
                if (rep) best_f = ms < best_f ? ms : best_f;
            }
            printf("nv=%3d slab=%3d KiB  launch-based %6.2f us/step   fused %6.2f us/step%s\n", nv, nld * 4,
                   best_l * 1e3f / steps, best_f * 1e3f / steps, e ? "  (a wait expired: void)" : "");
        }
    }
    return 0;
}
