// tk_host.cpp -- host-native compressed side of tensorkrylov!:
// the k-sized work of each iteration that never touches n-length data.
//
//   * tk_compressed_solve  solve_compressed_system (src/tensor_krylov_method.jl:10-34,
//                          src/utils.jl:501-523): Y_s[:, j] = exp(-alpha_j/lmin * first(H)) b~_s,
//                          lambda_j = omega_j / lmin.  For SymInstance first(H) is
//                          Symmetric(H_1, :L) (src/tensor_struct.jl:259) and all t exponentials
//                          come from ONE eigendecomposition; for NonSymInstance each term is a
//                          Pade scaling-and-squaring matrix exponential, as Julia's exp(::Matrix).
//   * tk_residualnorm      residualnorm! + compressed_residual (src/utils.jl:371-443,
//                          Lemma 3.4) with the O(d^3 t^2) masked products of the reference as
//                          leave-one-out / leave-two-out elementwise products.
//
// Plain C++ (no LAPACK in the image): symmetric eigensolver = Householder tridiagonalisation
// + implicit QL with Wilkinson shifts; general exponential = Higham's degree-13 Pade with
// scaling and squaring.  Results agree with the NumPy/SciPy oracle to rounding
// (tests/test_host.py).
#include <immintrin.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "../../include/tk.h"
#include "tk_host.h"

namespace tkh {

// ------------------------------------------------------------------ symmetric eigen
// A (n x n, column-major, symmetric; only the lower triangle is read) -> eigenvalues w
// (ascending) and orthonormal eigenvectors Q (columns).
static void tridiagonalize(int n, Vec& Q, Vec& diag, Vec& off) {
    // Householder reduction Q' A Q = T (A overwritten by the accumulated Q)
    diag.assign(n, 0.0);
    off.assign(n, 0.0);
#define A_(i, j) Q[(size_t)(j) * n + (i)]
    for (int i = n - 1; i > 0; --i) {
        const int l = i - 1;
        double h = 0.0, scale = 0.0;
        if (l > 0) {
            for (int k = 0; k <= l; ++k) scale += fabs(A_(i, k));
            if (scale == 0.0) {
                off[i] = A_(i, l);
            } else {
                for (int k = 0; k <= l; ++k) {
                    A_(i, k) /= scale;
                    h += A_(i, k) * A_(i, k);
                }
                double f = A_(i, l);
                double g = f >= 0.0 ? -sqrt(h) : sqrt(h);
                off[i] = scale * g;
                h -= f * g;
                A_(i, l) = f - g;
                f = 0.0;
                for (int j = 0; j <= l; ++j) {
                    A_(j, i) = A_(i, j) / h;
                    g = 0.0;
                    for (int k = 0; k <= j; ++k) g += A_(j, k) * A_(i, k);
                    for (int k = j + 1; k <= l; ++k) g += A_(k, j) * A_(i, k);
                    off[j] = g / h;
                    f += off[j] * A_(i, j);
                }
                const double hh = f / (h + h);
                for (int j = 0; j <= l; ++j) {
                    f = A_(i, j);
                    off[j] = g = off[j] - hh * f;
                    for (int k = 0; k <= j; ++k) A_(j, k) -= (f * off[k] + g * A_(i, k));
                }
            }
        } else {
            off[i] = A_(i, l);
        }
        diag[i] = h;
    }
    diag[0] = 0.0;
    off[0] = 0.0;
    for (int i = 0; i < n; ++i) {
        const int l = i - 1;
        if (diag[i] != 0.0) {
            for (int j = 0; j <= l; ++j) {
                double g = 0.0;
                for (int k = 0; k <= l; ++k) g += A_(i, k) * A_(k, j);
                for (int k = 0; k <= l; ++k) A_(k, j) -= g * A_(k, i);
            }
        }
        diag[i] = A_(i, i);
        A_(i, i) = 1.0;
        for (int j = 0; j <= l; ++j) A_(j, i) = A_(i, j) = 0.0;
    }
#undef A_
}

// sqrt(a^2 + b^2) without libm's hypot (its overflow-safe scaling costs more than the rest
// of a QL rotation); falls back to hypot outside the range where the squares are exact-safe
static inline double fast_hypot(double a, double b) {
    const double m = std::max(fabs(a), fabs(b));
    if (m > 1e-150 && m < 1e150) return sqrt(a * a + b * b);
    return hypot(a, b);
}

static bool tql(int n, Vec& d, Vec& e, Vec& Z) {
    // implicit QL on the tridiagonal (d, e[1..n-1]) accumulating into Z
    for (int i = 1; i < n; ++i) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    for (int l = 0; l < n; ++l) {
        int iter = 0, m;
        do {
            for (m = l; m < n - 1; ++m) {
                const double dd = fabs(d[m]) + fabs(d[m + 1]);
                if (fabs(e[m]) <= 2.220446049250313e-16 * dd) break;
            }
            if (m != l) {
                if (++iter > 60) return false;
                double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
                double r = fast_hypot(g, 1.0);
                g = d[m] - d[l] + e[l] / (g + (g >= 0.0 ? fabs(r) : -fabs(r)));
                double s = 1.0, c = 1.0, p = 0.0;
                int i;
                for (i = m - 1; i >= l; --i) {
                    double f = s * e[i];
                    const double b = c * e[i];
                    e[i + 1] = (r = fast_hypot(f, g));
                    if (r == 0.0) {
                        d[i + 1] -= p;
                        e[m] = 0.0;
                        break;
                    }
                    s = f / r;
                    c = g / r;
                    g = d[i + 1] - p;
                    r = (d[i] - g) * s + 2.0 * c * b;
                    d[i + 1] = g + (p = s * r);
                    g = c * r - b;
                    double* __restrict zi = &Z[(size_t)i * n];
                    double* __restrict zn = &Z[(size_t)(i + 1) * n];
                    for (int k = 0; k < n; ++k) {
                        const double a = zi[k], b2 = zn[k];
                        zn[k] = s * a + c * b2;
                        zi[k] = c * a - s * b2;
                    }
                }
                if (r == 0.0 && i >= l) continue;
                d[l] -= p;
                e[l] = g;
                e[m] = 0.0;
            }
        } while (m != l);
    }
    return true;
}

bool sym_eig(int n, const double* A, int lda, Vec& w, Vec& Q) {
    Q.assign((size_t)n * n, 0.0);
    // Symmetric(H, :L) of an upper-Hessenberg H (Arnoldi) or of a Lanczos T is already
    // tridiagonal: QL directly on (diag, subdiag), Q starting from the identity
    bool tri = true;
    for (int j = 0; j < n && tri; ++j)
        for (int i = j + 2; i < n; ++i)
            if (A[(size_t)j * lda + i] != 0.0) {
                tri = false;
                break;
            }
    Vec e;
    if (tri) {
        w.assign(n, 0.0);
        e.assign(n, 0.0);
        for (int i = 0; i < n; ++i) {
            w[i] = A[(size_t)i * lda + i];
            if (i > 0) e[i] = A[(size_t)(i - 1) * lda + i];
            Q[(size_t)i * n + i] = 1.0;
        }
    } else {
        for (int j = 0; j < n; ++j)
            for (int i = j; i < n; ++i) Q[(size_t)j * n + i] = Q[(size_t)i * n + j] = A[(size_t)j * lda + i];   // lower
        tridiagonalize(n, Q, w, e);
    }
    if (!tql(n, w, e, Q)) return false;
    // ascending order
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return w[a] < w[b]; });
    Vec w2(n), Q2((size_t)n * n);
    for (int c = 0; c < n; ++c) {
        w2[c] = w[idx[c]];
        memcpy(&Q2[(size_t)c * n], &Q[(size_t)idx[c] * n], n * sizeof(double));
    }
    w.swap(w2);
    Q.swap(Q2);
    return true;
}

// ------------------------------------------------------------------ general exponential
static void gemm_nn(int m, int n, int kk, const double* __restrict A, int lda, const double* __restrict B, int ldb,
                    double* __restrict C, int ldc);
// C = A B (n x n, column-major): the register-blocked AVX2 kernel below (the plain triple loop
// ran at ~4 GFMA/s at n = 50, the Pade / squaring products being most of a nonsymmetric
// iteration's host time at C4)
static void matmul(int n, const double* A, const double* B, double* C) { gemm_nn(n, n, n, A, n, B, n, C, n); }

static bool lu_solve(int n, Vec& A, Vec& B) {
    // solve A X = B (n x n each), partial pivoting; B overwritten by X.  Columns are separate
    // arrays to the compiler (restrict): every inner loop is an axpy it vectorizes.
    std::vector<int> piv(n);
    double* __restrict Ad = A.data();
    for (int k = 0; k < n; ++k) {
        double* __restrict ak = Ad + (size_t)k * n;
        int p = k;
        for (int i = k + 1; i < n; ++i)
            if (fabs(ak[i]) > fabs(ak[p])) p = i;
        if (ak[p] == 0.0) return false;
        piv[k] = p;
        if (p != k) {
            for (int j = 0; j < n; ++j) std::swap(A[(size_t)j * n + k], A[(size_t)j * n + p]);
            for (int j = 0; j < n; ++j) std::swap(B[(size_t)j * n + k], B[(size_t)j * n + p]);
        }
        const double inv = 1.0 / ak[k];
        for (int i = k + 1; i < n; ++i) ak[i] *= inv;
        for (int j = k + 1; j < n; ++j) {
            double* __restrict aj = Ad + (size_t)j * n;
            const double a = aj[k];
            if (a != 0.0)
                for (int i = k + 1; i < n; ++i) aj[i] -= ak[i] * a;
        }
    }
    // the triangular solves for all n right-hand sides at once on a row-major copy of B:
    // row updates X[i, :] -= L[i, k] X[k, :] are full-length contiguous axpys
    Vec T((size_t)n * n);
    double* __restrict X = T.data();
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) X[(size_t)i * n + j] = B[(size_t)j * n + i];
    for (int k = 0; k < n; ++k) {
        const double* __restrict xk = X + (size_t)k * n;
        const double* __restrict ak = Ad + (size_t)k * n;
        for (int i = k + 1; i < n; ++i) {
            const double l = ak[i];
            if (l == 0.0) continue;
            double* __restrict xi = X + (size_t)i * n;
            for (int j = 0; j < n; ++j) xi[j] -= l * xk[j];
        }
    }
    for (int k = n - 1; k >= 0; --k) {
        double* __restrict xk = X + (size_t)k * n;
        const double* __restrict ak = Ad + (size_t)k * n;
        const double dk = ak[k];
        for (int j = 0; j < n; ++j) xk[j] /= dk;
        for (int i = 0; i < k; ++i) {
            const double u = ak[i];
            if (u == 0.0) continue;
            double* __restrict xi = X + (size_t)i * n;
            for (int j = 0; j < n; ++j) xi[j] -= u * xk[j];
        }
    }
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) B[(size_t)j * n + i] = X[(size_t)i * n + j];
    return true;
}

// exp(c A) by Pade approximants of degree 3/5/7/9/13 with scaling and squaring (Higham 2005,
// the method of Julia's LinearAlgebra.exp!).  The even powers A^2, A^4, A^6, A^8 of the
// UNSCALED matrix are formed once (ExpmPowers) and reused by every scalar c: (cA)^2k =
// c^2k A^2k, so the exponential-sum terms of one iteration, exp(g_j H) for j = 1..t, share
// them (the products then differ from (cA)(cA) by rounding only).  Scratch in ExpmPowers.
void ExpmPowers::reset(int n_, const double* A_) {
    n = n_;
    A = A_;
    have = 0;
    norm1 = 0.0;
    for (int j = 0; j < n; ++j) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += fabs(A[(size_t)j * n + i]);
        norm1 = std::max(norm1, s);
    }
}

static const double kTheta[] = {1.495585217958292e-2, 2.539398330063230e-1, 9.504178996162932e-1,
                                2.097847961257068e0, 5.371920351148152e0};

int ExpmPowers::needs(double c) const {
    const double nrm = fabs(c) * norm1;
    static const int top[] = {2, 4, 6, 8};   // Pade degree 3/5/7/9 reads powers up to m - 1
    for (int q = 0; q < 4; ++q)
        if (nrm <= kTheta[q]) return top[q];
    return 6;                                // degree 13: A^2, A^4, A^6
}

const double* ExpmPowers::pw(int k) {
    const size_t nn = (size_t)n * n;
    if (have < 2) { P2.resize(nn); matmul(n, A, A, P2.data()); have = 2; }
    if (k >= 4 && have < 4) { P4.resize(nn); matmul(n, P2.data(), P2.data(), P4.data()); have = 4; }
    if (k >= 6 && have < 6) { P6.resize(nn); matmul(n, P4.data(), P2.data(), P6.data()); have = 6; }
    if (k >= 8 && have < 8) { P8.resize(nn); matmul(n, P4.data(), P4.data(), P8.data()); have = 8; }
    return k == 2 ? P2.data() : k == 4 ? P4.data() : k == 6 ? P6.data() : P8.data();
}

static bool expm_scaled(ExpmPowers& pw, ExpmScratch& xs, double c, Vec& E) {
    static const double b13[] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                                 1187353796428800.0,  129060195264000.0,   10559470521600.0,
                                 670442572800.0,      33522128640.0,       1323241920.0,
                                 40840800.0,          960960.0,            16380.0,
                                 182.0,               1.0};
    const double* theta = kTheta;
    static const double bd[4][10] = {{120.0, 60.0, 12.0, 1.0},
                                     {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0},
                                     {17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0},
                                     {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
                                      2162160.0, 110880.0, 3960.0, 90.0, 1.0}};
    const int n = pw.n;
    const size_t nn = (size_t)n * n;
    const double* A = pw.A;
    const double norm1 = fabs(c) * pw.norm1;
    for (Vec* v : {&xs.U, &xs.V, &xs.T, &xs.Num, &xs.Den}) v->resize(nn);
    double* U = xs.U.data();
    double* V = xs.V.data();
    double* T = xs.T.data();
    static const int degs[] = {3, 5, 7, 9};
    int m = 13, s = 0;
    for (int q = 0; q < 4; ++q)
        if (norm1 <= theta[q]) {
            m = degs[q];
            break;
        }
    if (m < 13) {
        // U = cA * sum_{odd k} b_k (cA)^{k-1},  V = sum_{even k} b_k (cA)^k
        const double* b = bd[m == 3 ? 0 : m == 5 ? 1 : m == 7 ? 2 : 3];
        for (size_t i = 0; i < nn; ++i) T[i] = V[i] = 0.0;
        for (int i = 0; i < n; ++i) {
            T[(size_t)i * n + i] = b[1];
            V[(size_t)i * n + i] = b[0];
        }
        double ck = 1.0;
        for (int k = 2; k <= m - 1; k += 2) {
            ck *= c * c;
            const double* P = pw.pw(k);
            const double bu = b[k + 1] * ck, bv = b[k] * ck;
            for (size_t i = 0; i < nn; ++i) {
                T[i] += bu * P[i];
                V[i] += bv * P[i];
            }
        }
        matmul(n, A, T, U);
        for (size_t i = 0; i < nn; ++i) U[i] *= c;
    } else {
        if (norm1 > theta[4]) s = std::max(0, (int)ceil(log2(norm1 / theta[4])));
        const double sc = ldexp(c, -s), s2 = sc * sc, s4 = s2 * s2, s6 = s4 * s2;
        const double* B2 = pw.pw(2);
        const double* B4 = pw.pw(4);
        const double* B6 = pw.pw(6);
        const double* b = b13;
        // U = As (B6 (b13 B6 + b11 B4 + b9 B2) + b7 B6 + b5 B4 + b3 B2 + b1 I),
        // V = B6 (b12 B6 + b10 B4 + b8 B2) + b6 B6 + b4 B4 + b2 B2 + b0 I   (B2k = (sc A)^2k)
        double* W = xs.Num.data();
        for (size_t i = 0; i < nn; ++i) T[i] = b[13] * s6 * B6[i] + b[11] * s4 * B4[i] + b[9] * s2 * B2[i];
        matmul(n, B6, T, W);
        for (size_t i = 0; i < nn; ++i) W[i] = s6 * W[i] + b[7] * s6 * B6[i] + b[5] * s4 * B4[i] + b[3] * s2 * B2[i];
        for (int i = 0; i < n; ++i) W[(size_t)i * n + i] += b[1];
        matmul(n, A, W, U);
        for (size_t i = 0; i < nn; ++i) U[i] *= sc;
        for (size_t i = 0; i < nn; ++i) T[i] = b[12] * s6 * B6[i] + b[10] * s4 * B4[i] + b[8] * s2 * B2[i];
        matmul(n, B6, T, V);
        for (size_t i = 0; i < nn; ++i) V[i] = s6 * V[i] + b[6] * s6 * B6[i] + b[4] * s4 * B4[i] + b[2] * s2 * B2[i];
        for (int i = 0; i < n; ++i) V[(size_t)i * n + i] += b[0];
    }
    Vec& Num = xs.Num;
    Vec& Den = xs.Den;
    for (size_t i = 0; i < nn; ++i) {
        Num[i] = V[i] + U[i];
        Den[i] = V[i] - U[i];
    }
    if (!lu_solve(n, Den, Num)) return false;
    for (int q = 0; q < s; ++q) {
        matmul(n, Num.data(), Num.data(), T);
        memcpy(Num.data(), T, nn * sizeof(double));
    }
    E.assign(Num.begin(), Num.end());
    return true;
}

bool expm(int n, const double* A, Vec& E) {
    ExpmPowers pw;
    ExpmScratch xs;
    pw.reset(n, A);
    return expm_scaled(pw, xs, 1.0, E);
}


// ------------------------------------------------------------------ compressed solve / residual
// Dot product with four independent accumulators (vectorizable without reassociation flags).
static inline double dot4(int n, const double* a, const double* b) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int i = 0;
    for (; i + 4 <= n; i += 4) {
        s0 += a[i] * b[i];
        s1 += a[i + 1] * b[i + 1];
        s2 += a[i + 2] * b[i + 2];
        s3 += a[i + 3] * b[i + 3];
    }
    for (; i < n; ++i) s0 += a[i] * b[i];
    return (s0 + s1) + (s2 + s3);
}

// C[0:m, 0:n] = A[0:m, 0:kk] * B[0:kk, 0:n] (column-major; lda, ldb, ldc): AVX2 register blocks
// of 8 rows x 4 columns (eight ymm accumulators; each k step two A loads, four broadcasts,
// eight FMAs), then 4-row and single-row / single-column edges.  Every C entry is one
// accumulation in k order (a fused multiply-add per term), whatever block it falls in.
// The same products with zmm registers (AVX-512F, both the box's EPYC 9575F and this image's
// build host have it): blocks of 16 rows x 4 columns, the row edge through masked loads and
// stores.  Each C entry is the same k-ordered chain of fused multiply-adds as in the AVX2
// kernel, so the two give the same bits (TKHIP_HOST_AVX512=0 selects the AVX2 kernel).
__attribute__((target("avx512f"))) static void gemm_nn_512(int m, int n, int kk, const double* __restrict A, int lda,
                                                           const double* __restrict B, int ldb, double* __restrict C,
                                                           int ldc) {
    int j0 = 0;
    for (; j0 + 4 <= n; j0 += 4) {
        const double* b0 = B + (size_t)j0 * ldb;
        const double* b1 = b0 + ldb;
        const double* b2 = b1 + ldb;
        const double* b3 = b2 + ldb;
        for (int i0 = 0; i0 < m; i0 += 16) {
            const int r = m - i0;
            const __mmask8 k0 = (__mmask8)(r >= 8 ? 0xFF : (1u << r) - 1u);
            const __mmask8 k1 = (__mmask8)(r >= 16 ? 0xFF : (r > 8 ? (1u << (r - 8)) - 1u : 0u));
            __m512d c00 = _mm512_setzero_pd(), c01 = _mm512_setzero_pd(), c10 = _mm512_setzero_pd(),
                    c11 = _mm512_setzero_pd(), c20 = _mm512_setzero_pd(), c21 = _mm512_setzero_pd(),
                    c30 = _mm512_setzero_pd(), c31 = _mm512_setzero_pd();
            for (int c = 0; c < kk; ++c) {
                const double* a = A + (size_t)c * lda + i0;
                const __m512d a0 = _mm512_maskz_loadu_pd(k0, a), a1 = _mm512_maskz_loadu_pd(k1, a + 8);
                __m512d bv = _mm512_set1_pd(b0[c]);
                c00 = _mm512_fmadd_pd(a0, bv, c00);
                c01 = _mm512_fmadd_pd(a1, bv, c01);
                bv = _mm512_set1_pd(b1[c]);
                c10 = _mm512_fmadd_pd(a0, bv, c10);
                c11 = _mm512_fmadd_pd(a1, bv, c11);
                bv = _mm512_set1_pd(b2[c]);
                c20 = _mm512_fmadd_pd(a0, bv, c20);
                c21 = _mm512_fmadd_pd(a1, bv, c21);
                bv = _mm512_set1_pd(b3[c]);
                c30 = _mm512_fmadd_pd(a0, bv, c30);
                c31 = _mm512_fmadd_pd(a1, bv, c31);
            }
            double* cc = C + (size_t)j0 * ldc + i0;
            _mm512_mask_storeu_pd(cc, k0, c00);
            _mm512_mask_storeu_pd(cc + 8, k1, c01);
            _mm512_mask_storeu_pd(cc + ldc, k0, c10);
            _mm512_mask_storeu_pd(cc + ldc + 8, k1, c11);
            _mm512_mask_storeu_pd(cc + 2 * (size_t)ldc, k0, c20);
            _mm512_mask_storeu_pd(cc + 2 * (size_t)ldc + 8, k1, c21);
            _mm512_mask_storeu_pd(cc + 3 * (size_t)ldc, k0, c30);
            _mm512_mask_storeu_pd(cc + 3 * (size_t)ldc + 8, k1, c31);
        }
    }
    for (; j0 < n; ++j0) {
        const double* bj = B + (size_t)j0 * ldb;
        double* cj = C + (size_t)j0 * ldc;
        for (int i0 = 0; i0 < m; i0 += 8) {
            const int r = m - i0;
            const __mmask8 k0 = (__mmask8)(r >= 8 ? 0xFF : (1u << r) - 1u);
            __m512d c0 = _mm512_setzero_pd();
            for (int c = 0; c < kk; ++c)
                c0 = _mm512_fmadd_pd(_mm512_maskz_loadu_pd(k0, A + (size_t)c * lda + i0), _mm512_set1_pd(bj[c]), c0);
            _mm512_mask_storeu_pd(cj + i0, k0, c0);
        }
    }
}

static bool use_avx512() {
    static const bool v = [] {
        const char* e = getenv("TKHIP_HOST_AVX512");
        return !(e && e[0] == '0') && __builtin_cpu_supports("avx512f");
    }();
    return v;
}

static void gemm_nn(int m, int n, int kk, const double* __restrict A, int lda, const double* __restrict B, int ldb,
                    double* __restrict C, int ldc) {
    if (use_avx512()) {
        gemm_nn_512(m, n, kk, A, lda, B, ldb, C, ldc);
        return;
    }
    int j0 = 0;
    for (; j0 + 4 <= n; j0 += 4) {
        const double* b0 = B + (size_t)j0 * ldb;
        const double* b1 = b0 + ldb;
        const double* b2 = b1 + ldb;
        const double* b3 = b2 + ldb;
        int i0 = 0;
        for (; i0 + 8 <= m; i0 += 8) {
            __m256d c00 = _mm256_setzero_pd(), c01 = _mm256_setzero_pd(), c10 = _mm256_setzero_pd(),
                    c11 = _mm256_setzero_pd(), c20 = _mm256_setzero_pd(), c21 = _mm256_setzero_pd(),
                    c30 = _mm256_setzero_pd(), c31 = _mm256_setzero_pd();
            for (int c = 0; c < kk; ++c) {
                const double* a = A + (size_t)c * lda + i0;
                const __m256d a0 = _mm256_loadu_pd(a), a1 = _mm256_loadu_pd(a + 4);
                __m256d bv = _mm256_broadcast_sd(b0 + c);
                c00 = _mm256_fmadd_pd(a0, bv, c00);
                c01 = _mm256_fmadd_pd(a1, bv, c01);
                bv = _mm256_broadcast_sd(b1 + c);
                c10 = _mm256_fmadd_pd(a0, bv, c10);
                c11 = _mm256_fmadd_pd(a1, bv, c11);
                bv = _mm256_broadcast_sd(b2 + c);
                c20 = _mm256_fmadd_pd(a0, bv, c20);
                c21 = _mm256_fmadd_pd(a1, bv, c21);
                bv = _mm256_broadcast_sd(b3 + c);
                c30 = _mm256_fmadd_pd(a0, bv, c30);
                c31 = _mm256_fmadd_pd(a1, bv, c31);
            }
            double* cc = C + (size_t)j0 * ldc + i0;
            _mm256_storeu_pd(cc, c00);
            _mm256_storeu_pd(cc + 4, c01);
            _mm256_storeu_pd(cc + ldc, c10);
            _mm256_storeu_pd(cc + ldc + 4, c11);
            _mm256_storeu_pd(cc + 2 * (size_t)ldc, c20);
            _mm256_storeu_pd(cc + 2 * (size_t)ldc + 4, c21);
            _mm256_storeu_pd(cc + 3 * (size_t)ldc, c30);
            _mm256_storeu_pd(cc + 3 * (size_t)ldc + 4, c31);
        }
        for (; i0 + 4 <= m; i0 += 4) {
            __m256d c0 = _mm256_setzero_pd(), c1 = _mm256_setzero_pd(), c2 = _mm256_setzero_pd(),
                    c3 = _mm256_setzero_pd();
            for (int c = 0; c < kk; ++c) {
                const __m256d a0 = _mm256_loadu_pd(A + (size_t)c * lda + i0);
                c0 = _mm256_fmadd_pd(a0, _mm256_broadcast_sd(b0 + c), c0);
                c1 = _mm256_fmadd_pd(a0, _mm256_broadcast_sd(b1 + c), c1);
                c2 = _mm256_fmadd_pd(a0, _mm256_broadcast_sd(b2 + c), c2);
                c3 = _mm256_fmadd_pd(a0, _mm256_broadcast_sd(b3 + c), c3);
            }
            double* cc = C + (size_t)j0 * ldc + i0;
            _mm256_storeu_pd(cc, c0);
            _mm256_storeu_pd(cc + ldc, c1);
            _mm256_storeu_pd(cc + 2 * (size_t)ldc, c2);
            _mm256_storeu_pd(cc + 3 * (size_t)ldc, c3);
        }
        for (; i0 < m; ++i0) {
            double acc[4] = {};
            for (int c = 0; c < kk; ++c) {
                const double av = A[(size_t)c * lda + i0];
                acc[0] = fma(av, b0[c], acc[0]);
                acc[1] = fma(av, b1[c], acc[1]);
                acc[2] = fma(av, b2[c], acc[2]);
                acc[3] = fma(av, b3[c], acc[3]);
            }
            for (int q = 0; q < 4; ++q) C[(size_t)(j0 + q) * ldc + i0] = acc[q];
        }
    }
    for (; j0 < n; ++j0) {
        const double* bj = B + (size_t)j0 * ldb;
        double* cj = C + (size_t)j0 * ldc;
        int i0 = 0;
        for (; i0 + 4 <= m; i0 += 4) {
            __m256d c0 = _mm256_setzero_pd();
            for (int c = 0; c < kk; ++c)
                c0 = _mm256_fmadd_pd(_mm256_loadu_pd(A + (size_t)c * lda + i0), _mm256_broadcast_sd(bj + c), c0);
            _mm256_storeu_pd(cj + i0, c0);
        }
        for (; i0 < m; ++i0) {
            double acc = 0.0;
            for (int c = 0; c < kk; ++c) acc = fma(A[(size_t)c * lda + i0], bj[c], acc);
            cj[i0] = acc;
        }
    }
}

// C[i, j] = <A[:, i], B[:, j]> for i < m, j < n (A: kk x m, B: kk x n, column-major, leading
// dimension kk; C row-major with stride ldc) through row-major copies: rows of A' and B'
// are broadcast against contiguous output rows.
static void gemm_tn(int m, int n, int kk, const double* A, const double* B, double* C, int ldc, Vec& tmp) {
    // Bt[r][j] = B[r, j]  (kk x n, row stride n)
    tmp.resize((size_t)kk * n);
    double* __restrict Bt = tmp.data();
    for (int j = 0; j < n; ++j)
        for (int r = 0; r < kk; ++r) Bt[(size_t)r * n + j] = B[(size_t)j * kk + r];
    for (int i = 0; i < m; ++i) {
        double* __restrict ci = C + (size_t)i * ldc;
        for (int j = 0; j < n; ++j) ci[j] = 0.0;
        const double* ai = A + (size_t)i * kk;
        for (int r = 0; r < kk; ++r) {
            const double av = ai[r];
            const double* br = Bt + (size_t)r * n;
            for (int j = 0; j < n; ++j) ci[j] += av * br[j];
        }
    }
}

bool compressed_solve(int d, int k, const double* H1, int ldh, int symmetric, const double* bt, int ldb,
                      int t, const double* alpha, const double* omega, double lmin, double* lambda, double* Y,
                      Work& ws) {
    const double inv = 1.0 / lmin;                                    // src/utils.jl:507
    for (int j = 0; j < t; ++j) lambda[j] = inv * omega[j];
    if (symmetric) {
        // exp(g Symmetric(H1, :L)) = Q exp(g w) Q' for every term: one eigendecomposition
        if (!sym_eig(k, H1, ldh, ws.w, ws.Q)) return false;
        const double* Q = ws.Q.data();
        ws.C.resize((size_t)k * d);
        for (int s = 0; s < d; ++s)                                   // C = Q' B
            for (int c = 0; c < k; ++c) ws.C[(size_t)s * k + c] = dot4(k, Q + (size_t)c * k, bt + (size_t)s * ldb);
        ws.E.resize((size_t)k * t);
        for (int j = 0; j < t; ++j) {
            const double g = -alpha[j] * inv;
            for (int c = 0; c < k; ++c) ws.E[(size_t)j * k + c] = exp(ws.w[c] * g);
        }
        // M[:, (s, j)] = exp(g_j w) .* C[:, s];  Y_s[:, j] = Q M[:, (s, j)]
        ws.M.resize((size_t)k * t * d);
        for (int s = 0; s < d; ++s)
            for (int j = 0; j < t; ++j) {
                double* m = &ws.M[((size_t)s * t + j) * k];
                const double* e = &ws.E[(size_t)j * k];
                const double* cs = &ws.C[(size_t)s * k];
                for (int c = 0; c < k; ++c) m[c] = e[c] * cs[c];
            }
        // (with helpers: column blocks of Y = Q M, each column the same arithmetic)
        const int ncol = t * d, nth = std::max(1, std::min(std::min(ws.nthreads, 4), ncol / 8));
        auto part = [&](int q) {
            const int c0 = q * ncol / nth, c1 = (q + 1) * ncol / nth;
            gemm_nn(k, c1 - c0, k, Q, k, ws.M.data() + (size_t)c0 * k, k, Y + (size_t)c0 * k, k);
        };
        par_for(ws.par, nth, part);
    } else {
        // every term exp(g_j H1) from the same powers of H1 (ExpmPowers); with ws.nthreads > 1
        // the terms are spread over helper tasks (the powers formed first, then read-only;
        // each term's arithmetic is the same whichever thread runs it)
        ws.G.resize((size_t)k * k);
        for (int c = 0; c < k; ++c)
            for (int i = 0; i < k; ++i) ws.G[(size_t)c * k + i] = H1[(size_t)c * ldh + i];
        ws.pw.reset(k, ws.G.data());
        auto term = [&](int j, ExpmScratch& xs) -> bool {
            const double g = -alpha[j] * inv;
            if (!expm_scaled(ws.pw, xs, g, xs.Ex)) return false;
            for (int s = 0; s < d; ++s) {
                double* y = Y + (size_t)s * k * t + (size_t)j * k;
                for (int i = 0; i < k; ++i) y[i] = 0.0;
                for (int c = 0; c < k; ++c) {
                    const double b = bt[(size_t)s * ldb + c];
                    const double* e = &xs.Ex[(size_t)c * k];
                    for (int i = 0; i < k; ++i) y[i] += e[i] * b;
                }
            }
            return true;
        };
        const int nth = std::min(std::min(ws.nthreads, t), 4);
        if (nth <= 1) {
            for (int j = 0; j < t; ++j)
                if (!term(j, ws.xs[0])) return false;
        } else {
            int top = 2;
            for (int j = 0; j < t; ++j) top = std::max(top, ws.pw.needs(-alpha[j] * inv));
            ws.pw.pw(top);
            bool ok[4] = {true, true, true, true};
            auto part = [&](int q) {
                for (int j = q; j < t; j += nth) ok[q] = ok[q] && term(j, ws.xs[q]);
            };
            par_for(ws.par, nth, part);
            for (int q = 0; q < nth; ++q)
                if (!ok[q]) return false;
        }
    }
    return true;
}

int residual(int d, int k, int t, const double* H, int ldh, size_t hs, const double* lambda, const double* Y,
             const double* subdiag, const double* bt, int ldb, double bnorm, double* r_comp, double* r_norm,
             Work& ws) {
    const size_t tt = (size_t)t * t, kt = (size_t)k * t;
    auto y = [&](int s, int i, int j) { return Y[(size_t)s * kt + (size_t)j * k + i]; };
    // Z_s = H_s Y_s;  Ly_s = lower(Y_s' Y_s), Lz_s = lower(Z_s' Z_s), X_s = Y_s' Z_s  ([i*t+j])
    ws.Z.assign((size_t)d * kt, 0.0);
    ws.Ly.assign(d * tt, 0.0);
    ws.Lz.assign(d * tt, 0.0);
    ws.X.assign(d * tt, 0.0);
    // per factor: Z_s = H_s Y_s and the Gram blocks of [Y_s Z_s]; independent over s, so with
    // helper threads (ws.nthreads) the factors are split over them (each factor's arithmetic
    // unchanged; scratch per thread)
    auto factor = [&](int s, Vec& G2, Vec& YZv, Vec& tmp) {
        const double* Hs = H + (size_t)s * hs;
        double* Zs = &ws.Z[(size_t)s * kt];
        const double* Ys = Y + (size_t)s * kt;
        // (the minors are upper Hessenberg or tridiagonal; a dense GEMM in register blocks
        // is still cheaper than a column-by-column band update)
        gemm_nn(k, t, k, Hs, ldh, Ys, k, Zs, k);
        // G = [Y Z]' [Y Z]  (2t x 2t, row-major): Ly = lower(G11), X = G12, Lz = lower(G22)
        double* YZ = YZv.data();
        memcpy(YZ, Ys, kt * sizeof(double));
        memcpy(YZ + kt, Zs, kt * sizeof(double));
        gemm_tn(2 * t, 2 * t, k, YZ, YZ, G2.data(), 2 * t, tmp);
        double* Ly = &ws.Ly[s * tt];
        double* Lz = &ws.Lz[s * tt];
        double* X = &ws.X[s * tt];
        const double* G = G2.data();
        for (int i = 0; i < t; ++i)
            for (int j = 0; j < t; ++j) {
                X[(size_t)i * t + j] = G[(size_t)i * 2 * t + t + j];
                if (j <= i) {
                    Ly[(size_t)i * t + j] = G[(size_t)i * 2 * t + j];
                    Lz[(size_t)i * t + j] = G[(size_t)(t + i) * 2 * t + t + j];
                }
            }
    };
    const int nth = std::max(1, std::min(std::min(ws.nthreads, 4), d));
    for (int q = 0; q < nth; ++q) {
        ws.G2[q].resize((size_t)4 * tt);
        ws.YZ[q].resize((size_t)2 * kt);
    }
    auto part = [&](int q) {
        for (int s = q; s < d; s += nth) factor(s, ws.G2[q], ws.YZ[q], ws.tmp[q]);
    };
    par_for(ws.par, nth, part);
    auto W = [&](int i, int j) { return i == j ? 1.0 : 2.0; };   // lower triangle only
    // first term: sum_s beta_s^2 * sum W .* Gamma_s .* prod_{q != s} Ly_q  (prefix/suffix)
    ws.pre.assign(d * tt, 1.0);
    ws.suf.assign(d * tt, 1.0);
    double* pre = ws.pre.data();
    double* suf = ws.suf.data();
    const double* Ly = ws.Ly.data();
    const double* Lz = ws.Lz.data();
    const double* X = ws.X.data();
    for (int s = 1; s < d; ++s)
        for (size_t e = 0; e < tt; ++e) pre[s * tt + e] = pre[(s - 1) * tt + e] * Ly[(s - 1) * tt + e];
    for (int s = d - 2; s >= 0; --s)
        for (size_t e = 0; e < tt; ++e) suf[s * tt + e] = suf[(s + 1) * tt + e] * Ly[(s + 1) * tt + e];
    double res = 0.0;
    for (int s = 0; s < d; ++s) {
        double acc = 0.0;
        for (int i = 0; i < t; ++i)
            for (int j = 0; j <= i; ++j) {
                const double gam = y(s, k - 1, i) * y(s, k - 1, j) * (lambda[i] * lambda[j]);
                acc += W(i, j) * gam * (pre[s * tt + (size_t)i * t + j] * suf[s * tt + (size_t)i * t + j]);
            }
        res += subdiag[s] * subdiag[s] * acc;
    }
    // compressed residual ||Hy||^2: per element e = (i, j), j <= i,
    //   sum_s Lz_s prod_{q != s} Ly_q + sum_{s != r} X_s[e] X_r[e'] prod_{q != s, r} Ly_q
    // accumulated in one pass over the factors (states: no factor chosen, one Lz chosen,
    // one X_s[e] / one X_r[e'] chosen, two chosen) -- O(d t^2) instead of O(d^3 t^2)
    double hy_norm = 0.0;
    for (int i = 0; i < t; ++i)
        for (int j = 0; j <= i; ++j) {
            const size_t e = (size_t)i * t + j, et = (size_t)j * t + i;
            double s0 = 1.0, sl = 0.0, sa = 0.0, sb = 0.0, s2 = 0.0;
            for (int q = 0; q < d; ++q) {
                const double ly = Ly[q * tt + e], xe = X[q * tt + e], xt = X[q * tt + et];
                s2 = s2 * ly + sa * xt + sb * xe;
                sa = sa * ly + s0 * xe;
                sb = sb * ly + s0 * xt;
                sl = sl * ly + s0 * Lz[q * tt + e];
                s0 = s0 * ly;
            }
            hy_norm += W(i, j) * (lambda[i] * lambda[j]) * (sl + s2);
        }
    // <Hy, b>: first rows of Y_s and Z_s
    double hy_b = 0.0;
    for (int j = 0; j < t; ++j)
        for (int s = 0; s < d; ++s) {
            double p = ws.Z[(size_t)s * kt + (size_t)j * k];
            for (int q = 0; q < d; ++q)
                if (q != s) p *= y(q, 0, j);
            hy_b += lambda[j] * p;
        }
    hy_b *= bnorm;
    double bn2 = 1.0;
    for (int s = 0; s < d; ++s) {
        double acc = 0.0;
        for (int i = 0; i < k; ++i) acc += bt[(size_t)s * ldb + i] * bt[(size_t)s * ldb + i];
        bn2 *= acc;
    }
    const double rc = hy_norm - 2 * hy_b + bn2;
    *r_comp = rc;
    if (rc < 0.0) {
        *r_norm = NAN;
        return 1;
    }
    *r_norm = sqrt(res + rc);
    return 0;
}

}  // namespace tkh

using namespace tkh;

tk_status tk_fail_internal(int code, const char* msg);   // tk_abi.cpp: tk_last_error()'s store

// nothing throws across the ABI (include/tk.h): host containers' exceptions become statuses
#define TK_API_BEGIN try {
#define TK_API_END                                                                            \
    }                                                                                         \
    catch (const std::bad_alloc&) { return tk_fail_internal(TK_ERR_ALLOC, "host allocation failed"); } \
    catch (...) { return tk_fail_internal(TK_ERR_INTERNAL, "unknown C++ exception"); }

extern "C" {

tk_status tk_compressed_solve(int d, int k, const double* H1, int symmetric, const double* bt, int t,
                              const double* alpha, const double* omega, double lmin, double* lambda, double* Y) { TK_API_BEGIN
    if (d < 1 || k < 1 || t < 1 || !H1 || !bt || !alpha || !omega || !lambda || !Y) return TK_ERR_ARG;
    Work ws;
    if (!compressed_solve(d, k, H1, k, symmetric, bt, k, t, alpha, omega, lmin, lambda, Y, ws)) return TK_ERR_STATE;
    return TK_OK;
    TK_API_END
}

tk_status tk_residualnorm(int d, int k, int t, const double* H, const double* lambda, const double* Y,
                          const double* subdiag, const double* bt, double bnorm, double* r_comp, double* r_norm) { TK_API_BEGIN
    if (d < 1 || k < 1 || t < 1 || !H || !lambda || !Y || !subdiag || !bt || !r_comp || !r_norm) return TK_ERR_ARG;
    Work ws;
    return residual(d, k, t, H, k, (size_t)k * k, lambda, Y, subdiag, bt, k, bnorm, r_comp, r_norm, ws)
               ? TK_BREAKDOWN : TK_OK;
    TK_API_END
}

}  // extern "C"
