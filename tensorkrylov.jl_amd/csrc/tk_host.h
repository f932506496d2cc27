// tk_host.h -- host numerics shared by tk_host.cpp (compressed solve, residual) and
// tk_solver.cpp (the native per-iteration driver).  Plain C++, no GPU.
#pragma once
#include <stddef.h>
#include <vector>

namespace tkh {

typedef std::vector<double> Vec;

// A (n x n column-major, leading dimension lda; lower triangle read) -> ascending
// eigenvalues w and orthonormal eigenvectors Q (n x n column-major)
bool sym_eig(int n, const double* A, int lda, Vec& w, Vec& Q);
// exp(A) (n x n column-major): Pade 3/5/7/9/13 with scaling and squaring
bool expm(int n, const double* A, Vec& E);

// The even powers A^2..A^8 of one unscaled matrix, formed on demand and shared by every
// exp(c A) of an iteration (tk_host.cpp expm_scaled); read-only once formed.
struct ExpmPowers {
    int n = -1;
    const double* A = nullptr;
    double norm1 = 0.0;
    int have = 0;                       // highest even power formed (0, 2, 4, 6, 8)
    Vec P2, P4, P6, P8;
    void reset(int n_, const double* A_);
    const double* pw(int k);            // A^k, k in {2, 4, 6, 8}
    int needs(double c) const;          // the highest power exp(c A) reads
};
// per-thread scratch of one exp(c A)
struct ExpmScratch {
    Vec U, V, T, Num, Den, Ex;
};

// The data-parallel parts of one evaluation (exp-sum terms, column blocks of Y = Q M, the
// residual's factors): run(n, fn, ctx) calls fn(ctx, i) for every i < n on the calling thread
// and whichever helper threads are free, and returns when all n calls are done.  A task's
// arithmetic depends on i alone, so the result is bitwise the serial one.
struct ParFor {
    virtual ~ParFor() {}
    virtual void run(int n, void (*fn)(void*, int), void* ctx) = 0;
};
template <class F>
inline void par_for(ParFor* p, int n, F& f) {
    if (!p || n <= 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    p->run(n, [](void* c, int i) { (*static_cast<F*>(c))(i); }, &f);
}

// Scratch of the two functions below (grown on demand, reused across iterations).
struct Work {
    Vec w, Q, C, E, M, ec, G, Ex;
    Vec Z, Ly, Lz, X, pre, suf;
    Vec G2[4], YZ[4], tmp[4];
    ExpmPowers pw;
    ExpmScratch xs[4];
    // tasks (<= 4) the parts above are split into, and the helpers that run them (the native
    // loop sets both for the last iterations, when the other workers are idle)
    int nthreads = 1;
    ParFor* par = nullptr;
};

// solve_compressed_system (src/tensor_krylov_method.jl:10-34): lambda[j] = omega[j]/lmin and
// Y_s[:, j] = exp(-alpha_j/lmin * first(H)) btilde_s for every factor s.
//   H1: k x k (column-major, leading dimension ldh); bt: d vectors, stride ldb;
//   Y: [s][j][i] (k x t column-major per factor).  false: eigen/expm failure.
bool compressed_solve(int d, int k, const double* H1, int ldh, int symmetric, const double* bt, int ldb,
                      int t, const double* alpha, const double* omega, double lmin, double* lambda, double* Y,
                      Work& ws);

// residualnorm! + compressed_residual (src/utils.jl:371-443, Lemma 3.4).
//   H: d minors k x k, column-major, leading dimension ldh, factor stride hs;
//   Y: [s][j][i]; subdiag[s] = H_s[k+1, k]; bt: stride ldb.
// Returns 0 (ok) or 1 (compressed norm breakdown: r_comp < 0, r_norm = NaN).
int residual(int d, int k, int t, const double* H, int ldh, size_t hs, const double* lambda, const double* Y,
             const double* subdiag, const double* bt, int ldb, double bnorm, double* r_comp, double* r_norm,
             Work& ws);

}  // namespace tkh
