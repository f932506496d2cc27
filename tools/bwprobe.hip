// bwprobe.hip -- microbenchmark of the Arnoldi pass-2 access pattern on gfx950 (tile-major
// V, thread-per-row, V^T u block reductions) to decide how to restructure the pass kernels.
// Not part of the library.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bwprobe.hip
// Run: ./bwprobe [ncols]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define TPB 256
#define CH 16
#define TSTR (TPB + 16)
typedef __amdgpu_buffer_rsrc_t rsrc_t;
#define GP(T, p) ((__attribute__((address_space(1))) T*)(p))

__device__ __forceinline__ rsrc_t mkrsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
template <int AUX = 0>
__device__ __forceinline__ double bld(rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double row16_sum(double s) {
    s += dpp<0x128>(s);
    s += dpp<0x124>(s);
    s += dpp<0x122>(s);
    s += dpp<0x121>(s);
    return s;
}
__device__ __forceinline__ void chunk_reduce(const double (&x)[CH], double* tr, double* acc, int base, bool first) {
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

struct Args {
    double* V;      // [nf][ntiles][KC][256]
    double* W;      // [nf][ld]
    double* U;      // [nf][ld]
    double* P;      // [nf][nv][npart]
    const double* h;
    int ntiles, KC, nc, npart;
    int64_t ld;
};

// MODE 0: no reduction (u = w - V h only)
// MODE 1: per-tile block reduction (current library scheme)
// MODE 2: per-thread register accumulation over the block's tiles, one block reduction at the end
template <int MAXC, int MODE, int AUX, int LAY = 0>
__global__ __launch_bounds__(TPB) void k_pass2(Args a) {
    __shared__ double tr[CH * TSTR];
    __shared__ double hs[64];
    __shared__ double acc[80];
    const int f = blockIdx.y;
    const int64_t TS = (int64_t)TPB * a.KC;
    for (int c = threadIdx.x; c < 64; c += TPB) hs[c] = c < a.nc ? a.h[c] : 0.0;
    __syncthreads();
    double racc[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) racc[c] = 0.0;
    bool first = true;
    for (int tile = blockIdx.x; tile < a.ntiles; tile += a.npart, first = false) {
        double v[MAXC];
        if (LAY == 0) {
            const double* Vt = a.V + ((int64_t)f * a.ntiles + tile) * TS;
            const rsrc_t tv = mkrsrc(Vt, (uint32_t)a.nc * TPB * 8);
            const uint32_t toff = threadIdx.x * 8u;
#pragma unroll
            for (int c = 0; c < MAXC; ++c) v[c] = bld<AUX>(tv, toff + (uint32_t)c * (TPB * 8));
        } else if (LAY == 2) {
            // paired columns: (r, c) at tile*TS + (c>>1)*512 + r*2 + (c&1); 16 B per lane
            const double* Vt = a.V + ((int64_t)f * a.ntiles + tile) * TS;
            const rsrc_t tv = mkrsrc(Vt, (uint32_t)((a.nc + 1) / 2) * TPB * 16);
            const uint32_t toff = threadIdx.x * 16u;
#pragma unroll
            for (int c = 0; c < MAXC; c += 2) {
                typedef double d2 __attribute__((ext_vector_type(2)));
                const d2 x = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(tv, toff + (uint32_t)(c / 2) * (TPB * 16), 0, AUX));
                v[c] = x.x;
                v[c + 1] = x.y;
            }
        } else {
            // column-major per factor: V[c*ld + r]; resource covers nc columns
            const double* Vf = a.V + (int64_t)f * a.ld * a.KC;
            const rsrc_t tv = mkrsrc(Vf, (uint32_t)(a.nc * a.ld * 8));
            const uint32_t roff = (uint32_t)(((int64_t)tile * TPB + threadIdx.x) * 8);
#pragma unroll
            for (int c = 0; c < MAXC; ++c) v[c] = bld<AUX>(tv, roff + (uint32_t)(c * a.ld * 8));
        }
        const int64_t r = (int64_t)tile * TPB + threadIdx.x;
        const double w = GP(const double, a.W)[f * a.ld + r];
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < MAXC; ++c) s += v[c] * hs[c];
        const double u = w - s;
        GP(double, a.U)[f * a.ld + r] = u;
        if (MODE == 1) {
#pragma unroll
            for (int c0 = 0; c0 < MAXC; c0 += CH) {
                if (c0 < a.nc) {
                    double x[CH];
#pragma unroll
                    for (int q = 0; q < CH; ++q) x[q] = v[c0 + q] * u;
                    chunk_reduce(x, tr, acc, c0, first);
                }
            }
        } else if (MODE == 2) {
#pragma unroll
            for (int c = 0; c < MAXC; ++c) racc[c] += v[c] * u;
        }
    }
    if (MODE == 2) {
#pragma unroll
        for (int c0 = 0; c0 < MAXC; c0 += CH) {
            double x[CH];
#pragma unroll
            for (int q = 0; q < CH; ++q) x[q] = racc[c0 + q];
            chunk_reduce(x, tr, acc, c0, true);
        }
    }
    if (MODE != 0) {
        __syncthreads();
        for (int c = threadIdx.x; c < a.nc; c += TPB)
            GP(double, a.P)[((int64_t)f * 64 + c) * a.npart + blockIdx.x] = acc[c];
    }
}


// double-buffered: the next tile's row is loaded before this tile's compute + reduction
template <int MAXC>
__device__ __forceinline__ void ld_row(double (&v)[MAXC], const Args& a, int f, int tile, int64_t TS) {
    const double* Vt = a.V + ((int64_t)f * a.ntiles + tile) * TS;
    const rsrc_t tv = mkrsrc(Vt, (uint32_t)((a.nc + 1) / 2) * TPB * 16);
    const uint32_t toff = threadIdx.x * 16u;
#pragma unroll
    for (int c = 0; c < MAXC; c += 2) {
        typedef double d2 __attribute__((ext_vector_type(2)));
        const d2 x = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(tv, toff + (uint32_t)(c / 2) * (TPB * 16), 0, 2));
        v[c] = x.x;
        v[c + 1] = x.y;
    }
}
template <int MAXC>
__device__ __forceinline__ void do_tile(const double (&v)[MAXC], const Args& a, int f, int tile, const double* hs,
                                        double* tr, double* acc, bool first) {
    const int64_t r = (int64_t)tile * TPB + threadIdx.x;
    const double w = GP(const double, a.W)[f * a.ld + r];
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) s += v[c] * hs[c];
    const double u = w - s;
    GP(double, a.U)[f * a.ld + r] = u;
#pragma unroll
    for (int c0 = 0; c0 < MAXC; c0 += CH) {
        if (c0 < a.nc) {
            double x[CH];
#pragma unroll
            for (int q = 0; q < CH; ++q) x[q] = c0 + q < MAXC ? v[c0 + q < MAXC ? c0 + q : 0] * u : 0.0;
            chunk_reduce(x, tr, acc, c0, first);
        }
    }
}
template <int MAXC>
__global__ __launch_bounds__(TPB) void k_pass2_db(Args a) {
    __shared__ double tr[CH * TSTR];
    __shared__ double hs[64];
    __shared__ double acc[80];
    const int f = blockIdx.y;
    const int64_t TS = (int64_t)TPB * a.KC;
    for (int c = threadIdx.x; c < 64; c += TPB) hs[c] = c < a.nc ? a.h[c] : 0.0;
    __syncthreads();
    double A[MAXC], B[MAXC];
    int tile = blockIdx.x;
    bool first = true;
    if (tile < a.ntiles) ld_row<MAXC>(A, a, f, tile, TS);
    for (; tile < a.ntiles; tile += 2 * a.npart) {
        const int t2 = tile + a.npart, t3 = t2 + a.npart;
        if (t2 < a.ntiles) ld_row<MAXC>(B, a, f, t2, TS);
        do_tile<MAXC>(A, a, f, tile, hs, tr, acc, first);
        first = false;
        if (t2 < a.ntiles) {
            if (t3 < a.ntiles) ld_row<MAXC>(A, a, f, t3, TS);
            do_tile<MAXC>(B, a, f, t2, hs, tr, acc, false);
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.nc; c += TPB)
        GP(double, a.P)[((int64_t)f * 64 + c) * a.npart + blockIdx.x] = acc[c];
}

// pure read of the same bytes with 16 B/lane loads (flat column-contiguous sweep)
__global__ __launch_bounds__(TPB) void k_read(const double2* __restrict__ p, int64_t n2, double* out) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n2; i += (int64_t)gridDim.x * TPB) {
        typedef double d2 __attribute__((ext_vector_type(2)));
        d2 x = __builtin_nontemporal_load((const d2*)(p + i));
        s += x.x + x.y;
    }
    if (s == 12345.678) out[0] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

template <class F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int nc = argc > 1 ? atoi(argv[1]) : 40;
    const int nf = 8, KC = 52, ntiles = 4096;
    const int64_t ld = (int64_t)ntiles * TPB;
    Args a;
    const size_t vbytes = (size_t)nf * ntiles * KC * TPB * 8;
    CK(hipMalloc(&a.V, vbytes));
    CK(hipMalloc(&a.W, nf * ld * 8));
    CK(hipMalloc(&a.U, nf * ld * 8));
    CK(hipMalloc(&a.P, (size_t)nf * 64 * 4096 * 8));
    double* h;
    CK(hipMalloc(&h, 64 * 8));
    CK(hipMemset(a.V, 0, vbytes));
    CK(hipMemset(a.W, 0, nf * ld * 8));
    CK(hipMemset(h, 0, 64 * 8));
    a.h = h;
    a.ntiles = ntiles;
    a.KC = KC;
    a.nc = nc;
    a.ld = ld;
    // bytes moved by one pass-2 launch: V cols + W read + U write
    const double bytes = (double)nf * ld * 8 * (nc + 2);
    auto rep = [&](const char* name, float ms) {
        printf("%-44s nc=%2d  %8.1f us  %6.2f TB/s\n", name, nc, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    };
    a.KC = 52;   // paired layout needs an even column count
    for (int npart : {1024, 512}) {
        a.npart = npart;
        dim3 g(npart, nf);
        char nm[128];
        snprintf(nm, sizeof nm, "paired MAXC48 single  npart=%d", npart);
        if (nc > 16) rep(nm, timeit([&] { k_pass2<48, 1, 2, 2><<<g, TPB>>>(a); }, 20));
        snprintf(nm, sizeof nm, "paired MAXC48 dbuf    npart=%d", npart);
        if (nc > 16) rep(nm, timeit([&] { k_pass2_db<48><<<g, TPB>>>(a); }, 20));
        snprintf(nm, sizeof nm, "paired MAXC16 single  npart=%d", npart);
        if (nc <= 16) rep(nm, timeit([&] { k_pass2<16, 1, 2, 2><<<g, TPB>>>(a); }, 20));
        snprintf(nm, sizeof nm, "paired MAXC16 dbuf    npart=%d", npart);
        if (nc <= 16) rep(nm, timeit([&] { k_pass2_db<16><<<g, TPB>>>(a); }, 20));
        snprintf(nm, sizeof nm, "paired MAXC8 single   npart=%d", npart);
        if (nc <= 8) rep(nm, timeit([&] { k_pass2<8, 1, 2, 2><<<g, TPB>>>(a); }, 20));
        snprintf(nm, sizeof nm, "paired MAXC8 dbuf     npart=%d", npart);
        if (nc <= 8) rep(nm, timeit([&] { k_pass2_db<8><<<g, TPB>>>(a); }, 20));
    }
    {
        // whole-V read with nontemporal 16 B loads: same byte count as nc columns over all tiles
        const int64_t n2 = (int64_t)nf * ntiles * nc * TPB / 2;
        double* out;
        CK(hipMalloc(&out, 8));
        float ms = timeit([&] { k_read<<<8192, TPB>>>((const double2*)a.V, n2, out); }, 20);
        printf("%-44s nc=%2d  %8.1f us  %6.2f TB/s\n", "flat 16B nt read (V bytes only)", nc, ms * 1e3,
               (double)n2 * 16 / (ms * 1e-3) / 1e12);
    }
    return 0;
}
