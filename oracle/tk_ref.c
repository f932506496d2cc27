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
