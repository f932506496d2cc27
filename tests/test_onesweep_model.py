"""CPU model of the device's one-sweep Arnoldi (CGS2 with the
reorthogonalization delayed one step) against the MGS2 oracle (src/orthogonal_bases.jl:15-37).

The model restates, column by column and in exact correspondence with k_arn_d1 + post_arn_d
(tensorkrylov.jl_amd/csrc/tk_kernels.hip), the recurrences the GPU evaluates row-wise:
  v_j = (u_j - V c) / beta_j;  u_{j+1} = A v_j - V h1;  z = A u_{j+1};
  c' = V' u;  beta' = sqrt(|u|^2 - |c'|^2);  H[:, j] = h1 + c';
  h1' = [(q - Hbar c') / beta' ; ((<u,z> - c'.q) / beta' - (Hbar c')_{j+1}) / beta'].
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
    U, c, invb = v0.copy(), np.zeros(0), 1.0            # k_init_bd / POST_INIT_B
    h1 = np.array([v0 @ (A @ v0)])
    for j in range(K):                                   # k_arn_d1 step j
        vj = (U - V[:, :j] @ c) * invb
        V[:, j] = vj
        u = A @ vj - V[:, :j + 1] @ h1
        z = A @ u
        p, q = V[:, :j + 1].T @ u, V[:, :j + 1].T @ z
        uu, uz = u @ u, u @ z
        c = p                                            # post_arn_d
        beta = np.sqrt(max(uu - p @ p, 0.0))
        H[:j + 1, j] = h1 + c
        H[j + 1, j] = beta
        g = H[:j + 2, :j + 1] @ c
        h1 = np.concatenate([(q - g[:j + 1]) / beta, [((uz - c @ q) / beta - g[j + 1]) / beta]])
        U, invb = u, 1.0 / beta
    V[:, K] = (U - V[:, :K] @ c) * invb                  # k_arn_finalize (flush)
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
