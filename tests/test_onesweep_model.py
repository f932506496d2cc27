"""CPU model of the device's one-sweep Arnoldi (CGS2 with the
reorthogonalization delayed one step) against the MGS2 oracle (src/orthogonal_bases.jl:15-37).

The model restates, column by column and in exact correspondence with k_arn_d1 + d1_coef +
bk_arn_d (tensorkrylov.jl_amd/csrc/tk_kernels.hip), the recurrences the GPU evaluates
row-wise.  Step J takes its coefficients straight from step J-1's dots
(c = V'u_J, q = V'A u_J, |u_J|^2, <u_J, A u_J>):
  beta = sqrt(|u|^2 - |c|^2);  gamma = (<u,Au> - c.q) / beta^2;
  v_J = (u_J - V c) / beta;    u_{J+1} = (A u_J - V q) / beta - gamma v_J
(CGS's u_{J+1} = A v_J - V h1 with h1 = (q - Hbar c) / beta, after the Arnoldi relation
A V c = V Hbar c cancels the Hbar terms).  The record of step J-1 (bookkeeping, off the
device's critical path) keeps the explicit first projection:
  H[:, J-1] = h1 + c;  h1' = [(q - Hbar c) / beta ; (<u,Au> - c.q) / beta^2 - (Hbar c)_J / beta].
It pins the algorithm's numerics independently of the GPU: H and V agree with MGS2 to the
parity tolerance of the GPU tests (1e-12 relative) -- and to ~1e-15 in practice -- for the
gallery's Laplace and convection-diffusion matrices, up to k close to n."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import tk_oracle as O


def onesweep_arnoldi(A, b, K):
    n = len(b)
    V = np.zeros((n, K + 1))
    H = np.zeros((K + 2, K + 1))
    v0 = (1.0 / np.linalg.norm(b)) * b
    V[:, 0] = v0
    U = v0.copy()                                        # k_init_bd / POST_INIT_B:
    c, q, uu, uz = np.zeros(0), np.zeros(0), 1.0, v0 @ (A @ v0)   # beta = 1, gamma = <v0,Av0>
    h1 = np.array([uz])
    for J in range(K):                                   # k_arn_d1 step J
        beta = np.sqrt(max(uu - c @ c, 0.0))             # d1_coef
        ib = 1.0 / beta
        t1 = (uz - c @ q) * ib
        gamma = t1 * ib
        if J >= 1:                                       # bk_arn_d of step J-1
            H[:J, J - 1] = h1 + c
            H[J, J - 1] = beta
            g = H[:J + 1, :J] @ c
            h1 = np.concatenate([(q - g[:J]) * ib, [(t1 - g[J]) * ib]])
        vj = (U - V[:, :J] @ c) * ib
        V[:, J] = vj
        u = ib * (A @ U - V[:, :J] @ q) - gamma * vj
        z = A @ u
        c, q, uu, uz = V[:, :J + 1].T @ u, V[:, :J + 1].T @ z, u @ u, u @ z
        U = u
    beta = np.sqrt(max(uu - c @ c, 0.0))                 # bk_arn_d of step K-1 + the flush
    H[:K, K - 1] = h1 + c
    H[K, K - 1] = beta
    V[:, K] = (U - V[:, :K] @ c) * (1.0 / beta)
    return V, H


@pytest.mark.parametrize("cls,n,K", [("Laplace", 200, 50), ("ConvDiff", 200, 50), ("Laplace", 200, 150),
                                     ("ConvDiff", 300, 120), ("Laplace", 3000, 60), ("ConvDiff", 3000, 60)])
def test_onesweep_model_matches_mgs2(cls, n, K):
    D = O.laplace_dense(n) if cls == "Laplace" else O.convdiff_dense(n)
    b = np.random.default_rng(n + K).random(n)
    b /= np.linalg.norm(b)
    ref = O.arnoldi_algorithm(O.dense_to_csc(D), b, K)
    V, H = onesweep_arnoldi(sp.csr_matrix(D), b, K)
    scale = np.abs(ref.H[:K + 1, :K]).max()
    assert np.abs(H[:K + 1, :K] - ref.H[:K + 1, :K]).max() <= 1e-12 * scale
    assert np.abs(V - ref.V[:, :K + 1]).max() <= 1e-12
    assert np.abs(V.T @ V - np.eye(K + 1)).max() <= 1e-13


def onesweep_lanczos(A, b, K):
    """k_lan_1s + k_reduce256 (RED_LAN): TTR (src/orthogonal_bases.jl:39-67) with the
    orthogonalization against v_j delayed into the next step; beta from the dots."""
    n = len(b)
    V = np.zeros((n, K + 1))
    alpha_, beta_ = np.zeros(K), np.zeros(K)
    U = (1.0 / np.linalg.norm(b)) * b                    # k_init_bd: U = v_0
    alpha, ib, betap, vprev = 0.0, 1.0, 0.0, np.zeros(n)  # POST_INIT_B
    for j in range(K):
        vj = ib * (U - alpha * vprev)                    # :53, :59
        V[:, j] = vj
        u = A @ vj - betap * vprev                       # :45-47
        a, uu, vv = u @ vj, u @ u, vj @ vj               # :50
        beta = np.sqrt(max((uu - (2.0 * a) * a) + (a * a) * vv, 0.0))   # :56
        alpha_[j], beta_[j] = a, beta
        alpha, ib, betap, vprev, U = a, (0.0 if beta == 0.0 else 1.0 / beta), beta, vj, u
    V[:, K] = ib * (U - alpha * vprev)                   # the flush (k_fin_d MODE 2)
    return V, alpha_, beta_


@pytest.mark.parametrize("n,K", [(200, 50), (200, 150), (3000, 60), (10000, 120)])
def test_onesweep_lanczos_model_matches_ttr(n, K):
    D = O.laplace_dense(n)
    b = np.random.default_rng(n + K).random(n)
    b /= np.linalg.norm(b)
    ref = O.lanczos_algorithm(O.dense_to_csc(D), b, K + 1)     # K TTR steps
    V, al, be = onesweep_lanczos(sp.csr_matrix(D), b, K)
    ra = np.array([ref.H[i, i] for i in range(K)])
    rb = np.array([ref.H[i + 1, i] for i in range(K)])
    scale = max(np.abs(ra).max(), np.abs(rb).max())
    assert np.abs(al - ra).max() <= 1e-13 * scale
    assert np.abs(be - rb).max() <= 1e-13 * scale
    assert np.abs(V - ref.V[:, :K + 1]).max() <= 1e-12
