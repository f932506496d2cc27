/*
 * tk_ref.c -- TEST INFRASTRUCTURE ONLY (parity oracle / CPU baseline).
 *
 * Plain-C restatement of the reference's per-factor Krylov steps, in the reference's
 * operation order, compiled with -ffp-contract=off:
 *   - SpMV  mul!(y, A::SparseMatrixCSC, x): y zeroed, column scatter
 *           y[rowval[p]] += nzval[p] * x[j]   (Julia 1.9 SparseArrays _spmatmul!,
 *           used at src/orthogonal_bases.jl:20,45,103)
 *   - orthonormalize!(::Decomposition, k, ::MGS)  src/orthogonal_bases.jl:15-37
 *     (two sequential MGS passes, H[k+1,k] = norm(v), V[:,k+1] = v .* inv(H[k+1,k]))
 *   - orthonormalize!(::Lanczos, k, ::TTR)        src/orthogonal_bases.jl:39-67
 * Only tests/ and bench.py's cpu_baseline leg load it (through oracle/tk_ref.py).
 * Indices are 0-based; step j consumes V[:, j] and produces V[:, j+1].
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static void csc_matvec(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nz,
                       const double* x, double* y) {
    memset(y, 0, (size_t)n * sizeof(double));
    for (int64_t j = 0; j < n; ++j) {
        const double xj = x[j];
        for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) y[rowval[p]] += nz[p] * xj;
    }
}

static double dot(int64_t n, const double* a, const double* b) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

void tkref_matvec(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nz,
                  const double* x, double* y) {
    csc_matvec(n, colptr, rowval, nz, x, y);
}

/* V[:,0] = inv(norm(b)) .* b   (initialize_decomp!, src/decompositions.jl:112-118) */
void tkref_init(int64_t n, const double* b, double* V) {
    const double inv = 1.0 / sqrt(dot(n, b, b));
    for (int64_t i = 0; i < n; ++i) V[i] = inv * b[i];
}

/* MGS step j: H column-major with leading dimension ldh; w is an n-length scratch. */
void tkref_arnoldi_step(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nz,
                        double* V, int64_t ldv, double* H, int64_t ldh, int j, double* w) {
    const double* vj = V + (int64_t)j * ldv;
    csc_matvec(n, colptr, rowval, nz, vj, w);
    double* Hc = H + (int64_t)j * ldh;
    for (int i = 0; i <= j; ++i) {                         /* :22-26 */
        const double* vi = V + (int64_t)i * ldv;
        const double h = dot(n, w, vi);
        Hc[i] = h;
        for (int64_t r = 0; r < n; ++r) w[r] = w[r] - h * vi[r];
    }
    for (int i = 0; i <= j; ++i) {                         /* :28-33 */
        const double* vi = V + (int64_t)i * ldv;
        const double h = dot(n, w, vi);
        Hc[i] += h;
        for (int64_t r = 0; r < n; ++r) w[r] = w[r] - h * vi[r];
    }
    const double nrm = sqrt(dot(n, w, w));                 /* :35 */
    Hc[j + 1] = nrm;
    const double inv = 1.0 / nrm;                          /* :36 */
    double* vn = V + (int64_t)(j + 1) * ldv;
    for (int64_t r = 0; r < n; ++r) vn[r] = w[r] * inv;
}

/* TTR step j: u = A v_j - beta_prev v_{j-1}; alpha = <u, v_j>; v = u - alpha v_j;
 * beta = norm(v); V[:, j+1] = beta == 0 ? 0 : inv(beta) .* v.  Returns alpha, beta. */
void tkref_lanczos_step(int64_t n, const int64_t* colptr, const int64_t* rowval, const double* nz,
                        double* V, int64_t ldv, int j, double beta_prev, double* w,
                        double* alpha_out, double* beta_out) {
    const double* vj = V + (int64_t)j * ldv;
    csc_matvec(n, colptr, rowval, nz, vj, w);
    if (j > 0) {
        const double* vp = V + (int64_t)(j - 1) * ldv;
        for (int64_t r = 0; r < n; ++r) w[r] = w[r] - beta_prev * vp[r];
    }
    const double alpha = dot(n, w, vj);
    for (int64_t r = 0; r < n; ++r) w[r] = w[r] - alpha * vj[r];
    const double beta = sqrt(dot(n, w, w));
    double* vn = V + (int64_t)(j + 1) * ldv;
    if (beta == 0.0) {
        memset(vn, 0, (size_t)n * sizeof(double));
    } else {
        const double inv = 1.0 / beta;
        for (int64_t r = 0; r < n; ++r) vn[r] = inv * w[r];
    }
    *alpha_out = alpha;
    *beta_out = beta;
}

/* ------------------------------------------------------------------ all-cores baseline
 * The same K-step MGS2 sweep (src/orthogonal_bases.jl:15-37) with the rows split over
 * OpenMP threads -- what the reference's dot/axpy would run with a threaded BLAS
 * (test/tensor_krylov_method.jl:33 sets BLAS.set_num_threads(30)).  SpMV as CSR row sums
 * (each row's products added in ascending column order, bitwise the CSC scatter); every
 * MGS projection: per-thread partial dot, one barrier, every thread sums the partials in
 * thread order; the axpy of projection i is fused with the partial dot of projection i+1.
 * Only the dot reduction order differs from tkref_arnoldi_step (results equal to rounding).
 * V column-major (ldv), H column-major (ldh), V[:,0] = b/|b| on entry. */
#include <omp.h>
void tkref_arnoldi_sweep_omp(int64_t n, const int64_t* rowptr, const int64_t* colind, const double* val,
                             double* V, int64_t ldv, double* H, int64_t ldh, int K, double* w,
                             int nthreads, double* partial /* 2 * 8 * nthreads */) {
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
    {
        const int nt = omp_get_num_threads(), t = omp_get_thread_num();
        const int64_t r0 = n * t / nt, r1 = n * (t + 1) / nt;
        int buf = 0;
#define TK_PART(b, th) partial[((b) * nt + (th)) * 8]
#define TK_SUM(res)                                                   \
    do {                                                              \
        _Pragma("omp barrier");                                       \
        double s_ = 0.0;                                              \
        for (int q_ = 0; q_ < nt; ++q_) s_ += TK_PART(buf, q_);       \
        (res) = s_;                                                   \
        buf ^= 1;                                                     \
    } while (0)
        for (int j = 0; j < K; ++j) {
            const double* vj = V + (int64_t)j * ldv;
            double* Hc = H + (int64_t)j * ldh;
            double acc = 0.0;
            for (int64_t r = r0; r < r1; ++r) {           /* w = A v_j ; partial <w, v_0> */
                double y = 0.0;
                for (int64_t p = rowptr[r]; p < rowptr[r + 1]; ++p) y += val[p] * vj[colind[p]];
                w[r] = y;
                acc += y * V[r];
            }
            TK_PART(buf, t) = acc;
            for (int pass = 0; pass < 2; ++pass)
                for (int i = 0; i <= j; ++i) {
                    double h;
                    TK_SUM(h);
                    if (t == 0) Hc[i] = pass == 0 ? h : Hc[i] + h;
                    const double* vi = V + (int64_t)i * ldv;
                    const int last = pass == 1 && i == j;
                    const double* vn = last ? w : (i < j ? vi + ldv : V);  /* next projection's column */
                    acc = 0.0;
                    for (int64_t r = r0; r < r1; ++r) {
                        const double x = w[r] - h * vi[r];
                        w[r] = x;
                        acc += x * (last ? x : vn[r]);
                    }
                    TK_PART(buf, t) = acc;
                }
            double nrm2;
            TK_SUM(nrm2);
            const double nrm = sqrt(nrm2);
            if (t == 0) Hc[j + 1] = nrm;
            const double inv = 1.0 / nrm;
            double* vnew = V + (int64_t)(j + 1) * ldv;
            for (int64_t r = r0; r < r1; ++r) vnew[r] = w[r] * inv;
#pragma omp barrier
        }
#undef TK_SUM
#undef TK_PART
    }
}

int tkref_max_threads(void) { return omp_get_max_threads(); }
