// Price of the step synchronisation a persistent one-sweep Arnoldi kernel would need at one
// factor per GPU (VERDICT r3 "next round" 1), against what the launch-based step pays now.
//
// One step of k_arn_d1 ends in (a) every window block publishing its partials of nv = 2j+4
// column dots (one partial per window, nwin = 4161 windows at n = 2^20), (b) a fixed-order
// reduction of each value over the nwin partials, (c) every block of the next step reading the
// nv reduced values.  The launch-based form does (b) in k_reduce256 (one block per value) with a
// kernel boundary on each side.  A persistent kernel does (a)-(c) inside one launch: grid
// barrier, values reduced by blocks 0..nv-1, grid barrier, reads.  No basis is streamed here:
// what is timed is exactly the synchronisation work a step adds on top of its window work.
//
//   launch   per step: k_pub (G blocks write the nwin partials) + k_red (nv blocks, as
//            k_reduce256: 24 loads per thread in flight, row sums, 16 in order) + k_use (G blocks
//            read the nv values) -- two kernel boundaries per step like the product
//   persist  one cooperative launch of G blocks for all steps: publish (sc1 stores + vmcnt(0)),
//            XCD-sharded barrier (8 counters, one top counter, a generation word; sc1 polls
//            with s_sleep), reduce by blocks < nv (same order), barrier, read
// Every spin is bounded (2^24 polls): a barrier that never completes sets an error word and
// the kernel exits -- no hang.  Prints microseconds per step for G = 512, 768, 1024, 1280
// and nv = 52, 100 (j = 24, 48).
// Build: hipcc -O3 --offload-arch=gfx950 tools/syncprobe.hip -o tools/_build/syncprobe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

#ifndef NWIN
#define NWIN 4161   // C2 at one factor (n = 2^20); -DNWIN=525 for C4 (n = 2^17, bandwidth 3)
#endif
#define SPIN_MAX (1 << 24)

__device__ __forceinline__ void st_sc1(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ double ld_sc1(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ double row16(double s) {
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    s += __shfl_xor(s, 8);
    return s;
}

// the partials of windows b, b+G, ... (value v of window w at P[v * NWIN + w])
__device__ void publish(double* P, int nv, int step) {
    for (int w = blockIdx.x; w < NWIN; w += gridDim.x)
        for (int v = threadIdx.x; v < nv; v += blockDim.x) st_sc1(P + (size_t)v * NWIN + w, 1e-3 * (w + v + step));
}

// value v over the NWIN partials in k_reduce256's order
__device__ double reduce_value(const double* P, int v, double* rs) {
    const int t = threadIdx.x;
    double part[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) {
        const int b = t + 256 * i;
        part[i] = b < NWIN ? ld_sc1(P + (size_t)v * NWIN + b) : 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 24; ++i) s += part[i];
    s = row16(s);
    if ((t & 15) == 0) rs[t >> 4] = s;
    __syncthreads();
    double r = 0.0;
    for (int q = 0; q < 16; ++q) r += rs[q];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(256) void k_pub(double* P, int nv, int step) { publish(P, nv, step); }
__global__ __launch_bounds__(256) void k_red(const double* P, double* R, int nv) {
    __shared__ double rs[16];
    const double r = reduce_value(P, blockIdx.x, rs);
    if (threadIdx.x == 0) st_sc1(R + blockIdx.x, r);
}
__global__ __launch_bounds__(256) void k_use(const double* R, double* out, int nv) {
    double s = 0.0;
    for (int v = threadIdx.x & 63; v < nv; v += 64) s += ld_sc1(R + v);
    if (threadIdx.x == 0 && s == -1.0) out[blockIdx.x] = s;   // (keeps the loads)
}

// XCD-sharded grid barrier: shard = blockIdx % 8 (dispatch round-robin: the blocks of one XCD),
// monotonic counters, the last shard leader bumps the generation word
__device__ bool grid_barrier(unsigned* cnt, unsigned* top, unsigned* gen, unsigned target, unsigned* err) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        const unsigned sh = blockIdx.x & 7, per = gridDim.x >> 3;
        const unsigned old = __hip_atomic_fetch_add(cnt + 32 * sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == per * target) {
            const unsigned t = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t + 1 == 8 * target) __hip_atomic_store(gen, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int spins = 0;
        while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++spins < SPIN_MAX)
            __builtin_amdgcn_s_sleep(1);
        ok = spins < SPIN_MAX;
        if (!ok) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return ok;
}

__global__ __launch_bounds__(256) void k_persist(double* P, double* R, double* out, int nv, int steps, unsigned* cnt,
                                                 unsigned* top, unsigned* gen, unsigned* err) {
    __shared__ double rs[16];
    unsigned target = 0;
    for (int step = 0; step < steps; ++step) {
        publish(P, nv, step);
        if (!grid_barrier(cnt, top, gen, ++target, err)) return;
        if ((int)blockIdx.x < nv) {
            const double r = reduce_value(P, blockIdx.x, rs);
            if (threadIdx.x == 0) st_sc1(R + blockIdx.x, r);
        }
        if (!grid_barrier(cnt, top, gen, ++target, err)) return;
        double s = 0.0;
        for (int v = threadIdx.x & 63; v < nv; v += 64) s += ld_sc1(R + v);
        if (threadIdx.x == 0 && s == -1.0) out[blockIdx.x] = s;
    }
}

int main() {
    int dev = 0;
    CK(hipSetDevice(dev));
    int maxb = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&maxb, k_persist, 256, 0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, dev));
    printf("%s, %d CUs, k_persist resident blocks per CU (API) %d\n", prop.gcnArchName, prop.multiProcessorCount, maxb);
    double *P, *R, *out;
    unsigned *cnt, *top, *gen, *err;
    CK(hipMalloc(&P, (size_t)128 * NWIN * 8));
    CK(hipMalloc(&R, 128 * 8));
    CK(hipMalloc(&out, 4096 * 8));
    CK(hipMalloc(&cnt, 8 * 32 * 4));
    CK(hipMalloc(&top, 64));
    CK(hipMalloc(&gen, 64));
    CK(hipMalloc(&err, 64));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int steps = 50;
    for (int nv : {52, 100}) {
        for (int G : {512, 768, 1024, 1280}) {
            if (G > (maxb - 1) * prop.multiProcessorCount) continue;   // (one block per CU of margin)
            // launch-based
            float best = 1e9;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipEventRecord(a, s));
                for (int st = 0; st < steps; ++st) {
                    hipLaunchKernelGGL(k_pub, dim3(G), dim3(256), 0, s, P, nv, st);
                    hipLaunchKernelGGL(k_red, dim3(nv), dim3(256), 0, s, P, R, nv);
                    hipLaunchKernelGGL(k_use, dim3(G), dim3(256), 0, s, R, out, nv);
                }
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep) best = ms < best ? ms : best;
            }
            const float tl = best * 1e3f / steps;
            // persistent
            best = 1e9;
            unsigned e = 0;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipMemsetAsync(cnt, 0, 8 * 32 * 4, s));
                CK(hipMemsetAsync(top, 0, 64, s));
                CK(hipMemsetAsync(gen, 0, 64, s));
                CK(hipMemsetAsync(err, 0, 64, s));
                int nvv = nv, stp = steps;
                void* args[] = {&P, &R, &out, &nvv, &stp, &cnt, &top, &gen, &err};
                CK(hipEventRecord(a, s));
                CK(hipLaunchCooperativeKernel((const void*)k_persist, dim3(G), dim3(256), args, 0, s));
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
                if (e) break;
                if (rep) best = ms < best ? ms : best;
            }
            printf("nv=%3d G=%4d  launch-based %6.2f us/step   persistent %6.2f us/step%s\n", nv, G, tl,
                   best * 1e3f / steps, e ? "  (barrier timed out: not all blocks resident)" : "");
        }
    }
    return 0;
}
