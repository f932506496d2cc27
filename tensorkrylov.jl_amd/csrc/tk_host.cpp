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
#include <math.h>
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
static void matmul(int n, const double* A, const double* B, double* C) {
    for (int j = 0; j < n; ++j) {
        double* c = C + (size_t)j * n;
        for (int i = 0; i < n; ++i) c[i] = 0.0;
        for (int k = 0; k < n; ++k) {
            const double b = B[(size_t)j * n + k];
            const double* a = A + (size_t)k * n;
            for (int i = 0; i < n; ++i) c[i] += a[i] * b;
        }
    }
}

static bool lu_solve(int n, Vec& A, Vec& B) {
    // solve A X = B (n x n each), partial pivoting; B overwritten by X
    std::vector<int> piv(n);
    for (int k = 0; k < n; ++k) {
        int p = k;
        for (int i = k + 1; i < n; ++i)
            if (fabs(A[(size_t)k * n + i]) > fabs(A[(size_t)k * n + p])) p = i;
        if (A[(size_t)k * n + p] == 0.0) return false;
        piv[k] = p;
        if (p != k) {
            for (int j = 0; j < n; ++j) std::swap(A[(size_t)j * n + k], A[(size_t)j * n + p]);
            for (int j = 0; j < n; ++j) std::swap(B[(size_t)j * n + k], B[(size_t)j * n + p]);
        }
        const double inv = 1.0 / A[(size_t)k * n + k];
        for (int i = k + 1; i < n; ++i) A[(size_t)k * n + i] *= inv;
        for (int j = k + 1; j < n; ++j) {
            const double a = A[(size_t)j * n + k];
            if (a != 0.0)
                for (int i = k + 1; i < n; ++i) A[(size_t)j * n + i] -= A[(size_t)k * n + i] * a;
        }
    }
    for (int j = 0; j < n; ++j) {
        double* b = &B[(size_t)j * n];
        for (int k = 0; k < n; ++k)
            for (int i = k + 1; i < n; ++i) b[i] -= A[(size_t)k * n + i] * b[k];
        for (int k = n - 1; k >= 0; --k) {
            b[k] /= A[(size_t)k * n + k];
            for (int i = 0; i < k; ++i) b[i] -= A[(size_t)k * n + i] * b[k];
        }
    }
    return true;
}

// exp(A) by Pade approximants of degree 3/5/7/9/13 with scaling and squaring (Higham 2005,
// the method of Julia's LinearAlgebra.exp!)
bool expm(int n, const double* A, Vec& E) {
    static const double b13[] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                                 1187353796428800.0,  129060195264000.0,   10559470521600.0,
                                 670442572800.0,      33522128640.0,       1323241920.0,
                                 40840800.0,          960960.0,            16380.0,
                                 182.0,               1.0};
    static const double theta[] = {1.495585217958292e-2, 2.539398330063230e-1, 9.504178996162932e-1,
                                   2.097847961257068e0, 5.371920351148152e0};
    static const double bd[4][10] = {{120.0, 60.0, 12.0, 1.0},
                                     {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0},
                                     {17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0},
                                     {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
                                      2162160.0, 110880.0, 3960.0, 90.0, 1.0}};
    const size_t nn = (size_t)n * n;
    double norm1 = 0.0;
    for (int j = 0; j < n; ++j) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += fabs(A[(size_t)j * n + i]);
        norm1 = std::max(norm1, s);
    }
    Vec Id(nn, 0.0);
    for (int i = 0; i < n; ++i) Id[(size_t)i * n + i] = 1.0;
    Vec U(nn), V(nn), A2(nn);
    matmul(n, A, A, A2.data());
    static const int degs[] = {3, 5, 7, 9};
    for (int q = 0; q < 4; ++q) {
        if (norm1 <= theta[q]) {
            const int m = degs[q];
            const double* b = bd[q];
            Vec P(Id), Ut(nn, 0.0), Vt(nn, 0.0), tmp(nn);
            // U = A * sum_{odd} b_k A^{k-1},  V = sum_{even} b_k A^k
            for (size_t i = 0; i < nn; ++i) {
                Ut[i] = b[1] * P[i];
                Vt[i] = b[0] * P[i];
            }
            for (int k = 2; k <= m; k += 2) {
                matmul(n, P.data(), A2.data(), tmp.data());
                P.swap(tmp);
                for (size_t i = 0; i < nn; ++i) {
                    Ut[i] += b[k + 1] * P[i];
                    Vt[i] += b[k] * P[i];
                }
            }
            matmul(n, A, Ut.data(), U.data());
            Vec Num(nn), Den(nn);
            for (size_t i = 0; i < nn; ++i) {
                Num[i] = Vt[i] + U[i];
                Den[i] = Vt[i] - U[i];
            }
            if (!lu_solve(n, Den, Num)) return false;
            E.swap(Num);
            return true;
        }
    }
    int s = 0;
    if (norm1 > theta[4]) s = std::max(0, (int)ceil(log2(norm1 / theta[4])));
    const double sc = ldexp(1.0, -s);
    Vec As(nn);
    for (size_t i = 0; i < nn; ++i) As[i] = A[i] * sc;
    Vec B2(nn), B4(nn), B6(nn), tmp(nn);
    matmul(n, As.data(), As.data(), B2.data());
    matmul(n, B2.data(), B2.data(), B4.data());
    matmul(n, B4.data(), B2.data(), B6.data());
    const double* b = b13;
    for (size_t i = 0; i < nn; ++i) tmp[i] = b[13] * B6[i] + b[11] * B4[i] + b[9] * B2[i];
    matmul(n, B6.data(), tmp.data(), U.data());
    for (size_t i = 0; i < nn; ++i) U[i] += b[7] * B6[i] + b[5] * B4[i] + b[3] * B2[i] + b[1] * Id[i];
    matmul(n, As.data(), U.data(), tmp.data());
    U.swap(tmp);
    for (size_t i = 0; i < nn; ++i) tmp[i] = b[12] * B6[i] + b[10] * B4[i] + b[8] * B2[i];
    matmul(n, B6.data(), tmp.data(), V.data());
    for (size_t i = 0; i < nn; ++i) V[i] += b[6] * B6[i] + b[4] * B4[i] + b[2] * B2[i] + b[0] * Id[i];
    Vec Num(nn), Den(nn);
    for (size_t i = 0; i < nn; ++i) {
        Num[i] = V[i] + U[i];
        Den[i] = V[i] - U[i];
    }
    if (!lu_solve(n, Den, Num)) return false;
    for (int q = 0; q < s; ++q) {
        matmul(n, Num.data(), Num.data(), tmp.data());
        Num.swap(tmp);
    }
    E.swap(Num);
    return true;
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

// C[0:m, 0:n] = A[0:m, 0:kk] * B[0:kk, 0:n] (column-major; lda, ldb, ldc); register blocks of
// 8 rows x 4 columns, the inner dimension streamed (vectorized over rows).
static void gemm_nn(int m, int n, int kk, const double* __restrict A, int lda, const double* __restrict B, int ldb,
                    double* __restrict C, int ldc) {
    int j0 = 0;
    for (; j0 + 4 <= n; j0 += 4) {
        const double* b0 = B + (size_t)j0 * ldb;
        int i0 = 0;
        for (; i0 + 8 <= m; i0 += 8) {
            double acc[4][8] = {};
            for (int c = 0; c < kk; ++c) {
                const double* a = A + (size_t)c * lda + i0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const double bv = b0[(size_t)q * ldb + c];
#pragma unroll
                    for (int r = 0; r < 8; ++r) acc[q][r] += a[r] * bv;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 8; ++r) C[(size_t)(j0 + q) * ldc + i0 + r] = acc[q][r];
        }
        for (; i0 < m; ++i0) {
            double acc[4] = {};
            for (int c = 0; c < kk; ++c) {
                const double av = A[(size_t)c * lda + i0];
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] += av * b0[(size_t)q * ldb + c];
            }
            for (int q = 0; q < 4; ++q) C[(size_t)(j0 + q) * ldc + i0] = acc[q];
        }
    }
    for (; j0 < n; ++j0) {
        const double* bj = B + (size_t)j0 * ldb;
        double* cj = C + (size_t)j0 * ldc;
        for (int i = 0; i < m; ++i) cj[i] = 0.0;
        for (int c = 0; c < kk; ++c) {
            const double* a = A + (size_t)c * lda;
            const double bv = bj[c];
            for (int i = 0; i < m; ++i) cj[i] += a[i] * bv;
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
        gemm_nn(k, t * d, k, Q, k, ws.M.data(), k, Y, k);
    } else {
        ws.G.resize((size_t)k * k);
        for (int j = 0; j < t; ++j) {
            const double g = -alpha[j] * inv;
            for (int c = 0; c < k; ++c)
                for (int i = 0; i < k; ++i) ws.G[(size_t)c * k + i] = g * H1[(size_t)c * ldh + i];
            if (!expm(k, ws.G.data(), ws.Ex)) return false;
            for (int s = 0; s < d; ++s) {
                double* y = Y + (size_t)s * k * t + (size_t)j * k;
                for (int i = 0; i < k; ++i) y[i] = 0.0;
                for (int c = 0; c < k; ++c) {
                    const double b = bt[(size_t)s * ldb + c];
                    const double* e = &ws.Ex[(size_t)c * k];
                    for (int i = 0; i < k; ++i) y[i] += e[i] * b;
                }
            }
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
    ws.G.resize((size_t)4 * tt);
    ws.M.resize((size_t)2 * kt);
    for (int s = 0; s < d; ++s) {
        const double* Hs = H + (size_t)s * hs;
        double* Zs = &ws.Z[(size_t)s * kt];
        const double* Ys = Y + (size_t)s * kt;
        // (the minors are upper Hessenberg or tridiagonal; a dense GEMM in register blocks
        // is still cheaper than a column-by-column band update)
        gemm_nn(k, t, k, Hs, ldh, Ys, k, Zs, k);
        // G = [Y Z]' [Y Z]  (2t x 2t, row-major): Ly = lower(G11), X = G12, Lz = lower(G22)
        double* YZ = ws.M.data();
        memcpy(YZ, Ys, kt * sizeof(double));
        memcpy(YZ + kt, Zs, kt * sizeof(double));
        gemm_tn(2 * t, 2 * t, k, YZ, YZ, ws.G.data(), 2 * t, ws.Ex);
        double* Ly = &ws.Ly[s * tt];
        double* Lz = &ws.Lz[s * tt];
        double* X = &ws.X[s * tt];
        const double* G = ws.G.data();
        for (int i = 0; i < t; ++i)
            for (int j = 0; j < t; ++j) {
                X[(size_t)i * t + j] = G[(size_t)i * 2 * t + t + j];
                if (j <= i) {
                    Ly[(size_t)i * t + j] = G[(size_t)i * 2 * t + j];
                    Lz[(size_t)i * t + j] = G[(size_t)(t + i) * 2 * t + t + j];
                }
            }
    }
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
