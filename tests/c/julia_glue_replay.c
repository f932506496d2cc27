/*
 * julia_glue_replay.c -- a plain-C caller of libtkhip.so that replays, call for call, what
 * the Julia drop-in (tensorkrylov.jl_amd/julia/TensorKrylovHIP.jl) does inside
 * tensorkrylov! (src/tensor_krylov_method.jl:36-125), including its 1-based record
 * offsets, so the glue's ccall sequence is exercised without a Julia toolchain:
 *
 *   HIPMatrix(ctx, A)       tk_matrix_from_csc(..., one_based = 1)   (Julia's colptr/rowval as-is)
 *   HIPDecomp(...)          tk_decomp_create(ctx, method, d, 0, d, mats, b, n, kmax, 2)
 *   records(dc, :init)      tk_decomp_init      -> apply_records!(td, rec, -1)
 *   orthonormalize!(td, k)  tk_decomp_step(k-1) -> apply_records!(td, rec, k-1),  k = 1..nmax
 *
 * apply_records! below is TensorKrylovHIP.jl:227-255 with its 1-based indices kept
 * literally (R(i) is Julia's r[i]; HJ(s, i, j) is Julia's td.H.M[s][i, j]).
 *
 * usage: julia_glue_replay METHOD D N KMAX RHS_FILE OUT_FILE
 *   RHS_FILE: D*N doubles (b_1 .. b_D);  OUT_FILE receives, per factor s = 1..D,
 *   H_s ((kmax+2)^2, column-major), btilde_s (kmax+1), gram_s ((kmax+1)^2, column-major).
 * Matrix: assemble_matrix(N, Laplace) (src/tensor_struct.jl:48-57), built here 1-based.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tk.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        tk_status st_ = (x);                                                       \
        if (st_ != TK_OK) {                                                        \
            fprintf(stderr, "%s failed (%d): %s\n", #x, st_, tk_last_error());     \
            exit(2);                                                               \
        }                                                                          \
    } while (0)

static int kmax_, d_, method_;
static double *Hs, *bts, *grams;   /* host mirror, per factor */
#define HJ(s, i, j) Hs[(size_t)((s) - 1) * (kmax_ + 2) * (kmax_ + 2) + (size_t)((j) - 1) * (kmax_ + 2) + ((i) - 1)]
#define BT(s, c) bts[(size_t)((s) - 1) * (kmax_ + 1) + ((c) - 1)]
#define GR(s, i, j) grams[(size_t)((s) - 1) * (kmax_ + 1) * (kmax_ + 1) + (size_t)((j) - 1) * (kmax_ + 1) + ((i) - 1)]

/* TensorKrylovHIP.jl apply_records!(td, rec, j); rec is Julia's m x d column-major
 * matrix == C's [d][m]. */
static void apply_records(const double* rec, int m, int j) {
    const int kmax = kmax_;
    for (int s = 1; s <= d_; ++s) {
        const double* r0 = rec + (size_t)(s - 1) * m;
#define R(i) r0[(i) - 1]
        if (j >= 0) {
            if (method_ == TK_ARNOLDI) {
                for (int i = 1; i <= j + 2; ++i) HJ(s, i, j + 1) = R(i);          /* H[1:j+2, j+1] .= r[1:j+2] */
            } else {
                const int reorth = method_ == TK_LANCZOS_REORTH && R(2 * kmax + 9) > 0;
                double beta;
                if (reorth) {
                    for (int i = 1; i <= j + 2; ++i) HJ(s, i, j + 1) = R(i);
                    for (int i = 1; i <= (j - 1 > 0 ? j - 1 : 0); ++i) HJ(s, i, j + 1) = 0.0;
                    beta = HJ(s, j + 2, j + 1);
                } else {
                    HJ(s, j + 1, j + 1) = R(j + 1);
                    beta = R(j + 2);
                }
                HJ(s, j + 2, j + 1) = beta;                                         /* update_subdiagonals! */
                HJ(s, j + 1, j + 2) = beta;
            }
        }
        const int c = (int)R(2 * kmax + 6);
        if (c >= 0) {
            BT(s, c + 1) = R(2 * kmax + 5);
            if (R(2 * kmax + 10) > 0)
                for (int i = 1; i <= c + 1; ++i) GR(s, c + 1, i) = R(kmax + 3 + i - 1); /* gram[c+1, 1:c+1] .= r[kmax+3:kmax+3+c] */
        }
#undef R
    }
}

int main(int argc, char** argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: %s METHOD D N KMAX RHS_FILE OUT_FILE\n", argv[0]);
        return 1;
    }
    method_ = atoi(argv[1]);
    d_ = atoi(argv[2]);
    const int64_t n = atoll(argv[3]);
    kmax_ = atoi(argv[4]);
    const int kmax = kmax_, d = d_;

    double* b = malloc(sizeof(double) * (size_t)d * n);
    FILE* fb = fopen(argv[5], "rb");
    if (!fb || fread(b, sizeof(double), (size_t)d * n, fb) != (size_t)d * n) {
        fprintf(stderr, "cannot read %s\n", argv[5]);
        return 1;
    }
    fclose(fb);

    /* assemble_matrix(n, Laplace) as Julia's SparseMatrixCSC: 1-based colptr / rowval */
    const double h = 1.0 / (double)(n + 1), c2 = 1.0 / (h * h);
    int64_t* colptr = malloc(sizeof(int64_t) * (n + 1));
    int64_t* rowval = malloc(sizeof(int64_t) * 3 * n);
    double* nzval = malloc(sizeof(double) * 3 * n);
    int64_t p = 0;
    for (int64_t j = 0; j < n; ++j) {
        colptr[j] = p + 1;
        if (j > 0) { rowval[p] = j; nzval[p++] = c2 * -1.0; }
        rowval[p] = j + 1; nzval[p++] = c2 * 2.0;
        if (j + 1 < n) { rowval[p] = j + 2; nzval[p++] = c2 * -1.0; }
    }
    colptr[n] = p + 1;

    tk_ctx* ctx = NULL;
    tk_mat* A = NULL;
    tk_decomp* dc = NULL;
    CHECK(tk_ctx_create(0, &ctx));
    CHECK(tk_matrix_from_csc(ctx, n, colptr, rowval, nzval, 1, &A));   /* one_based = 1 */
    tk_mat** mats = malloc(sizeof(tk_mat*) * d);
    const double** bp = malloc(sizeof(double*) * d);
    for (int s = 0; s < d; ++s) {
        mats[s] = A;                    /* the glue's IdDict cache: one device matrix per A_s object */
        bp[s] = b + (size_t)s * n;
    }
    CHECK(tk_decomp_create(ctx, method_, d, 0, d, mats, bp, n, kmax, 2, &dc));
    const int m = tk_record_len(kmax);
    if (m != 2 * kmax + 10) {           /* reclen(kmax) = 2kmax + 10 in the glue */
        fprintf(stderr, "record length %d != 2kmax+10\n", m);
        return 3;
    }
    Hs = calloc((size_t)d * (kmax + 2) * (kmax + 2), sizeof(double));
    bts = calloc((size_t)d * (kmax + 1), sizeof(double));
    grams = calloc((size_t)d * (kmax + 1) * (kmax + 1), sizeof(double));
    double* rec = calloc((size_t)d * m, sizeof(double));

    CHECK(tk_decomp_init(dc, rec));                     /* orthonormalize!(td, b) */
    apply_records(rec, m, -1);
    for (int k = 1; k <= kmax; ++k) {                   /* orthonormalize!(td, 1), then k = 2:nmax */
        memset(rec, 0, sizeof(double) * (size_t)d * m);
        CHECK(tk_decomp_step(dc, k - 1, rec));
        apply_records(rec, m, k - 1);
    }

    FILE* fo = fopen(argv[6], "wb");
    for (int s = 0; s < d; ++s) {
        fwrite(Hs + (size_t)s * (kmax + 2) * (kmax + 2), sizeof(double), (size_t)(kmax + 2) * (kmax + 2), fo);
        fwrite(bts + (size_t)s * (kmax + 1), sizeof(double), (size_t)(kmax + 1), fo);
        fwrite(grams + (size_t)s * (kmax + 1) * (kmax + 1), sizeof(double), (size_t)(kmax + 1) * (kmax + 1), fo);
    }
    fclose(fo);
    CHECK(tk_decomp_destroy(dc));                       /* finalizers, any order */
    CHECK(tk_matrix_destroy(A));
    CHECK(tk_ctx_destroy(ctx));
    printf("replayed %d steps of %d factors\n", kmax, d);
    return 0;
}
