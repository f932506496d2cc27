// Achievable-bandwidth probe for the end-of-solve V*Y shape (C2): each 256-row tile reads its
// whole basis slab (KC columns, contiguous, 16 B per lane) and writes a t-column X slab
// (contiguous, 16 B per lane) that depends on what it read -- the byte pattern of k_fin_vy /
// k_basis_mul with no arithmetic.  Reports TB/s of (read + write) bytes.
// Build: hipcc -O3 --offload-arch=gfx950 tools/rwprobe.hip -o tools/_build/rwprobe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define TPB 256
typedef double d2 __attribute__((ext_vector_type(2)));

// one block per tile; RD = 16-B reads per lane (KC/2), WR = 16-B writes per lane ceil(t*256/2/256)
template <int NT>
__global__ __launch_bounds__(TPB) void k_rw(const d2* __restrict__ V, d2* __restrict__ X, int rd, int wr) {
    const int64_t tile = blockIdx.x;
    const d2* v = V + tile * (int64_t)rd * TPB;
    d2* x = X + tile * (int64_t)wr * TPB;
    d2 s = {0.0, 0.0};
    d2 r[32];
#pragma unroll
    for (int i = 0; i < 32; ++i)
        if (i < rd) r[i] = __builtin_nontemporal_load(v + i * TPB + threadIdx.x);
#pragma unroll
    for (int i = 0; i < 32; ++i)
        if (i < rd) s += r[i];
    for (int i = 0; i < wr; ++i) {
        d2 o = s * (double)(i + 1);
        if (NT) __builtin_nontemporal_store(o, x + i * TPB + threadIdx.x);
        else x[i * TPB + threadIdx.x] = o;
    }
}

__global__ __launch_bounds__(TPB) void k_rd(const d2* __restrict__ V, double* out, int rd) {
    const int64_t tile = blockIdx.x;
    const d2* v = V + tile * (int64_t)rd * TPB;
    d2 s = {0.0, 0.0};
    d2 r[32];
#pragma unroll
    for (int i = 0; i < 32; ++i)
        if (i < rd) r[i] = __builtin_nontemporal_load(v + i * TPB + threadIdx.x);
#pragma unroll
    for (int i = 0; i < 32; ++i)
        if (i < rd) s += r[i];
    if (s.x == 12345.678) out[0] = s.y;
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
    const int kc = argc > 1 ? atoi(argv[1]) : 50;     // basis columns read
    const int t = argc > 2 ? atoi(argv[2]) : 17;      // X columns written
    const int ntile = 8 * 4096;                       // C2: 8 factors x 2^20 rows
    const int rd = kc / 2, wr = (t + 1) / 2;
    if (rd > 32) { printf("kc <= 64\n"); return 1; }
    d2 *V, *X;
    double* out;
    CK(hipMalloc(&V, (size_t)ntile * rd * TPB * 16));
    CK(hipMalloc(&X, (size_t)ntile * wr * TPB * 16));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(V, 0, (size_t)ntile * rd * TPB * 16));
    const double rb = (double)ntile * rd * TPB * 16, wb = (double)ntile * t * TPB * 8;
    float ms = timeit([&] { k_rd<<<ntile, TPB>>>(V, out, rd); }, 10);
    printf("read only            kc=%d        %8.1f us  %6.2f TB/s\n", kc, ms * 1e3, rb / (ms * 1e-3) / 1e12);
    ms = timeit([&] { k_rw<0><<<ntile, TPB>>>(V, X, rd, wr); }, 10);
    printf("read+write           kc=%d t=%d  %8.1f us  %6.2f TB/s\n", kc, t, ms * 1e3, (rb + wb) / (ms * 1e-3) / 1e12);
    ms = timeit([&] { k_rw<1><<<ntile, TPB>>>(V, X, rd, wr); }, 10);
    printf("read+write (nt st)   kc=%d t=%d  %8.1f us  %6.2f TB/s\n", kc, t, ms * 1e3, (rb + wb) / (ms * 1e-3) / 1e12);
    return 0;
}
