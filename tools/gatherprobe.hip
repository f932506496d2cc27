// Ceiling probe for C3's shared-matrix SpMV (k_spmv_mf): replays the SELL-256 index stream of
// config C3's A_s (dumped by tools/c3_sell_dump.py) over an interleaved vector block Uint
// (5 factors, rows padded to 64 B) and times variants of the same access pattern:
//   kernel   one thread per row, 3 x 16-B gathers per nonzero (k_spmv_mf's form), sums in order
//   coop4    four lanes per row, one 16-B piece of the 64-B row each (factors 2p, 2p+1)
//   matrix   the index / value stream alone (no gathers): the matrix-read floor
//   seqgath  kernel's loads with every gathered row replaced by the thread's own row
//            (sequential 64-B rows): what the same bytes cost without the random pattern
//   split40  the 40-B entry as 32 B (factors 0-3, rows at a 32-B pitch) + 8 B (factor 4, its
//            own array): lanes 0, 1 of a quad gather 16 B each of the 32-B piece, lane 2 the 8 B
//   pack40   the 40-B entry packed (rows at a 40-B pitch, no padding): lanes 0, 1 16 B each
//            (8-B aligned), lane 2 the last 8 B -- a row may straddle two 64-B segments
//   gath64   one 64-B gather per nonzero, no index/value loads (indices precomputed per
//            thread in registers is impossible; instead col = hash(row, q)): random-gather floor
// Reports microseconds (mean of 20) and the algorithmic bytes rate of the SpMV
// (12 nnz + 4 (n+1) matrix + 5 * 8n gathered vector + 5 * 8n written).
// Build: hipcc -O3 --offload-arch=gfx950 tools/gatherprobe.hip -o tools/_build/gatherprobe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define TPB 256
#define NF 5
#define NP 8   // Uint pitch (doubles)
typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Sell {
    int64_t n;
    const long long* sptr;
    const int* swidth;
    const int* rowlen;
    const int* scol;
    const double* sval;
};

__device__ __forceinline__ double mul_rn(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b) {
#pragma clang fp contract(off)
    return a + b;
}

// MODE 0: kernel form; 1: matrix only; 2: sequential gathers
template <int MODE>
__global__ __launch_bounds__(TPB) void k_thread(Sell A, const double* __restrict__ Ui, double* __restrict__ AU, int64_t ld) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r >= ld) return;
    double s[NF] = {0, 0, 0, 0, 0};
    if (r < A.n) {
        const int64_t t = r >> 8;
        const int l = (int)(r & 255);
        const int64_t base = A.sptr[t];
        const int w = A.swidth[t];
        const int len = A.rowlen[r];
        constexpr int SG = 4;
        for (int q0 = 0; q0 < w; q0 += SG) {
            int64_t cc[SG];
            double vv[SG];
#pragma unroll
            for (int g = 0; g < SG; ++g) {
                const int64_t e = base + (int64_t)(q0 + g) * TPB + l;
                const bool in = q0 + g < len;
                cc[g] = in ? (MODE == 2 ? r : (int64_t)A.scol[e]) : -1;
                if (MODE == 2 && in) (void)A.scol[e];
                vv[g] = in ? A.sval[e] : 0.0;
            }
            if (MODE == 1) {
#pragma unroll
                for (int g = 0; g < SG; ++g) s[0] += vv[g] * (double)cc[g];
                continue;
            }
            double u[SG][NF];
#pragma unroll
            for (int g = 0; g < SG; ++g)
#pragma unroll
                for (int f = 0; f < NF; f += 2) {
                    const d2 x = cc[g] >= 0 ? ((const d2*)(Ui + cc[g] * NP))[f >> 1] : (d2){0.0, 0.0};
                    u[g][f] = x.x;
                    if (f + 1 < NF) u[g][f + 1] = x.y;
                }
#pragma unroll
            for (int g = 0; g < SG; ++g)
                if (cc[g] >= 0)
#pragma unroll
                    for (int f = 0; f < NF; ++f) s[f] = add_rn(s[f], mul_rn(vv[g], u[g][f]));
        }
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) AU[(int64_t)f * ld + r] = s[f];
}

// four lanes per row: lane p of the quad gathers piece p (16 B) of the 64-B row
template <int SG>
__global__ __launch_bounds__(TPB) void k_coop4(Sell A, const double* __restrict__ Ui, double* __restrict__ AU, int64_t ld) {
    const int p = threadIdx.x & 3;
    const int64_t r = (int64_t)blockIdx.x * (TPB / 4) + (threadIdx.x >> 2);
    if (r >= ld) return;
    double s0 = 0.0, s1 = 0.0;
    if (r < A.n && p < 3) {
        const int64_t t = r >> 8;
        const int l = (int)(r & 255);
        const int64_t base = A.sptr[t];
        const int w = A.swidth[t];
        const int len = A.rowlen[r];
        for (int q0 = 0; q0 < w; q0 += SG) {
            int64_t cc[SG];
            double vv[SG];
#pragma unroll
            for (int g = 0; g < SG; ++g) {
                const int64_t e = base + (int64_t)(q0 + g) * TPB + l;
                const bool in = q0 + g < len;
                cc[g] = in ? (int64_t)A.scol[e] : -1;
                vv[g] = in ? A.sval[e] : 0.0;
            }
            d2 x[SG];
#pragma unroll
            for (int g = 0; g < SG; ++g) x[g] = cc[g] >= 0 ? ((const d2*)(Ui + cc[g] * NP))[p] : (d2){0.0, 0.0};
#pragma unroll
            for (int g = 0; g < SG; ++g)
                if (cc[g] >= 0) {
                    s0 = add_rn(s0, mul_rn(vv[g], x[g].x));
                    s1 = add_rn(s1, mul_rn(vv[g], x[g].y));
                }
        }
    }
    if (p < 3) {
        AU[(int64_t)(2 * p) * ld + r] = s0;
        if (2 * p + 1 < NF) AU[(int64_t)(2 * p + 1) * ld + r] = s1;
    }
}

// the 40-byte entry: SPLIT 1 -> U4 (32-B rows) + U1 (8-B rows); SPLIT 0 -> one 40-B-pitch array
template <int SPLIT>
__global__ __launch_bounds__(TPB) void k_e40(Sell A, const double* __restrict__ U4, const double* __restrict__ U1,
                                             double* __restrict__ AU, int64_t ld) {
    constexpr int SG = 4;
    const int p = threadIdx.x & 3;
    const int64_t r = (int64_t)blockIdx.x * (TPB / 4) + (threadIdx.x >> 2);
    if (r >= ld) return;
    double s0 = 0.0, s1 = 0.0;
    if (r < A.n && p < 3) {
        const int64_t t = r >> 8;
        const int l = (int)(r & 255);
        const int64_t base = A.sptr[t];
        const int w = A.swidth[t];
        const int len = A.rowlen[r];
        for (int q0 = 0; q0 < w; q0 += SG) {
            int64_t cc[SG];
            double vv[SG];
#pragma unroll
            for (int g = 0; g < SG; ++g) {
                const int64_t e = base + (int64_t)(q0 + g) * TPB + l;
                const bool in = q0 + g < len;
                cc[g] = in ? (int64_t)A.scol[e] : -1;
                vv[g] = in ? A.sval[e] : 0.0;
            }
            d2 x[SG];
#pragma unroll
            for (int g = 0; g < SG; ++g) {
                if (cc[g] < 0) {
                    x[g] = (d2){0.0, 0.0};
                } else if (SPLIT) {
                    x[g] = p < 2 ? ((const d2*)(U4 + cc[g] * 4))[p] : (d2){U1[cc[g]], 0.0};
                } else {
                    const double* row = U4 + cc[g] * 5;
                    x[g] = p < 2 ? *(const d2*)__builtin_assume_aligned(row + 2 * p, 8) : (d2){row[4], 0.0};
                }
            }
#pragma unroll
            for (int g = 0; g < SG; ++g)
                if (cc[g] >= 0) {
                    s0 = add_rn(s0, mul_rn(vv[g], x[g].x));
                    s1 = add_rn(s1, mul_rn(vv[g], x[g].y));
                }
        }
    }
    if (p < 3) {
        AU[(int64_t)(2 * p) * ld + r] = s0;
        if (2 * p + 1 < NF) AU[(int64_t)(2 * p + 1) * ld + r] = s1;
    }
}

// one 64-B (4 x 16 B) random gather per nonzero slot, columns from a hash: no matrix stream
__global__ __launch_bounds__(TPB) void k_gath64(int64_t n, int w, const double* __restrict__ Ui, double* __restrict__ AU, int64_t ld) {
    const int p = threadIdx.x & 3;
    const int64_t r = (int64_t)blockIdx.x * (TPB / 4) + (threadIdx.x >> 2);
    if (r >= ld) return;
    d2 s = {0.0, 0.0};
    uint32_t h = (uint32_t)r * 2654435761u;
    for (int q = 0; q < w; q += 4) {
        d2 x[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            h = h * 1664525u + 1013904223u;
            const int64_t c = (int64_t)(h % (uint32_t)n);
            x[g] = ((const d2*)(Ui + c * NP))[p];
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) s += x[g];
    }
    AU[(int64_t)p * ld + r] = s.x + s.y;
}

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

template <class T>
static T* up(const std::vector<T>& v) {
    T* d;
    CK(hipMalloc(&d, std::max<size_t>(v.size(), 1) * sizeof(T)));
    CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char** argv) {
    if (argc < 2) { printf("usage: gatherprobe SELL.bin\n"); return 1; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { printf("cannot open %s\n", argv[1]); return 1; }
    int64_t hdr[3];
    if (fread(hdr, 8, 3, f) != 3) return 1;
    const int64_t n = hdr[0], slots = hdr[1], nt = hdr[2];
    std::vector<long long> sptr(nt);
    std::vector<int> sw(nt), rl(nt * 256), scol(slots);
    std::vector<double> sval(slots);
    if (fread(sptr.data(), 8, nt, f) != (size_t)nt || fread(sw.data(), 4, nt, f) != (size_t)nt ||
        fread(rl.data(), 4, nt * 256, f) != (size_t)(nt * 256) || fread(scol.data(), 4, slots, f) != (size_t)slots ||
        fread(sval.data(), 8, slots, f) != (size_t)slots) { printf("short file\n"); return 1; }
    fclose(f);
    int64_t nnz = 0;
    int wmax = 0;
    for (int64_t i = 0; i < n; ++i) nnz += rl[i];
    for (int64_t t = 0; t < nt; ++t) wmax = std::max(wmax, sw[t]);
    const int64_t ld = nt * 256;
    Sell A{n, up(sptr), up(sw), up(rl), up(scol), up(sval)};
    std::vector<double> u(ld * NP);
    for (size_t i = 0; i < u.size(); ++i) u[i] = (double)((i * 2654435761u) % 1000) * 1e-3;
    double* Ui = up(u);
    double* AU;
    CK(hipMalloc(&AU, (size_t)NF * ld * 8));
    const double alg = 12.0 * nnz + 4.0 * (n + 1) + 2.0 * NF * 8.0 * n;
    const double gath = 64.0 * nnz;
    printf("n=%lld nnz=%lld (%.2f/row) slots=%lld (%.2f x nnz) max width %d; algorithmic %.1f MB, 64-B gathers %.1f MB\n",
           (long long)n, (long long)nnz, (double)nnz / n, (long long)slots, (double)slots / nnz, wmax, alg / 1e6, gath / 1e6);
    const int reps = 20;
    auto rep = [&](const char* name, float ms) {
        printf("%-10s %8.1f us  alg %6.2f TB/s  (64-B gathers %6.2f TB/s)\n", name, ms * 1e3, alg / (ms * 1e-3) / 1e12,
               gath / (ms * 1e-3) / 1e12);
    };
    const int nb = (int)(ld / TPB);
    rep("kernel", timeit([&] { k_thread<0><<<nb, TPB>>>(A, Ui, AU, ld); }, reps));
    rep("coop4", timeit([&] { k_coop4<4><<<(int)(ld / 64), TPB>>>(A, Ui, AU, ld); }, reps));
    rep("coop4sg8", timeit([&] { k_coop4<8><<<(int)(ld / 64), TPB>>>(A, Ui, AU, ld); }, reps));
    {
        std::vector<double> u4(ld * 4), u1(ld), u5(ld * 5);
        for (int64_t i = 0; i < ld; ++i) {
            for (int q = 0; q < 4; ++q) u4[i * 4 + q] = u[i * NP + q];
            u1[i] = u[i * NP + 4];
            for (int q = 0; q < 5; ++q) u5[i * 5 + q] = u[i * NP + q];
        }
        double* U4 = up(u4);
        double* U1 = up(u1);
        double* U5 = up(u5);
        const double g40 = 40.0 * nnz;
        auto rep40 = [&](const char* name, float ms) {
            printf("%-10s %8.1f us  alg %6.2f TB/s  (40-B entries %6.2f TB/s)\n", name, ms * 1e3,
                   alg / (ms * 1e-3) / 1e12, g40 / (ms * 1e-3) / 1e12);
        };
        rep40("split40", timeit([&] { k_e40<1><<<(int)(ld / 64), TPB>>>(A, U4, U1, AU, ld); }, reps));
        rep40("pack40", timeit([&] { k_e40<0><<<(int)(ld / 64), TPB>>>(A, U5, nullptr, AU, ld); }, reps));
        CK(hipFree(U4));
        CK(hipFree(U1));
        CK(hipFree(U5));
    }
    rep("matrix", timeit([&] { k_thread<1><<<nb, TPB>>>(A, Ui, AU, ld); }, reps));
    rep("seqgath", timeit([&] { k_thread<2><<<nb, TPB>>>(A, Ui, AU, ld); }, reps));
    const int wavg = (int)((nnz + n - 1) / n);
    rep("gath64", timeit([&] { k_gath64<<<(int)(ld / 64), TPB>>>(n, wavg, Ui, AU, ld); }, reps));
    CK(hipDeviceSynchronize());
    return 0;
}
