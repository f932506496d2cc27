"""CPU stand-in for tkamd.device.DeviceDecomposition -- TEST INFRASTRUCTURE ONLY.

Used by the CPU test suite to exercise the product's HOST logic (record bookkeeping,
factor partitioning over ranks, the per-step exchange, the compressed solve) without
a GPU.  It produces records with exactly the layout and column semantics of
libtkhip (include/tk.h) from the oracle's per-factor steps, and sums them over ranks
with torch.distributed (gloo) the way tk_decomp_step does with RCCL.  The product
path never uses it (tkamd has no CPU fallback).
"""
import numpy as np

from oracle import tk_oracle as O


class FakeDecomposition:
    def __init__(self, td, b):
        self.kmax = td.kmax
        self.layout = td.layout
        self.m = td.layout.m
        self.d = td.d
        self.loc = list(td.part.local())
        self.method = td.name
        self.b = {s: np.asarray(b[s], dtype=np.float64) for s in self.loc}
        self.f = {s: O.Factor(td.A[s], self.b[s], td.kmax) for s in self.loc}
        self.replica = False
        # TK_FAKE_GRAM_DEFERRED=1: orthogonality_data from one Gram at the end (tk_decomp_gram),
        # with the ABI's rule that a multi-rank handle refuses a Gram while a column is pending
        # (the flush that would write it starts record all-reduces every rank must join)
        import os
        self.gram_deferred = os.environ.get("TK_FAKE_GRAM_DEFERRED") == "1"
        self.pending = False
        self.next_step = 0
        self.log = []

    def _world(self):
        import sys
        if "torch.distributed" not in sys.modules:
            return 1
        import torch.distributed as dist
        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    def set_replica(self):
        self.replica = True

    def _exchange(self, r):
        import sys
        if "torch.distributed" not in sys.modules:   # single process: nothing to sum
            return r
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            import torch
            # a replica sends zero rows (tk_decomp_set_replica); it receives everyone's
            t = torch.from_numpy(np.zeros_like(r) if self.replica else r)
            dist.all_reduce(t)
            return t.numpy()
        return r

    def _gram(self, r, s, c):
        lay = self.layout
        V = self.f[s].V
        r[s, lay.col] = c
        r[s, lay.bt] = float(np.dot(V[:, c], self.b[s]))
        tracked = s == 0 or self.method == "TensorLanczosReorth"
        r[s, lay.tracked] = 1.0 if tracked else 0.0
        if tracked:
            r[s, lay.gram:lay.gram + c + 1] = V[:, :c + 1].T @ V[:, c]

    def init(self, want=True):
        r = np.zeros((self.d, self.m))
        for s in self.loc:
            self._gram(r, s, 0)
        return self._exchange(r)

    def step(self, j, want=True):
        r = np.zeros((self.d, self.m))
        lay = self.layout
        k = j + 1
        for s in self.loc:
            f = self.f[s]
            if self.method == "TensorArnoldi":
                f.arnoldi_mgs(k)
                r[s, :j + 2] = f.H[:j + 2, j]
                self._gram(r, s, j)
            elif self.method == "TensorLanczos":
                f.lanczos_ttr(k)
                r[s, j] = f.H[j, j]
                r[s, j + 1] = f.H[j + 1, j]
                if j > 0:
                    self._gram(r, s, j)
                else:
                    r[s, lay.col] = -1
            else:
                # the record carries the raw MGS column when re-orthogonalized; the
                # oracle has already applied the reference bookkeeping to H, so
                # re-expand: rows 0..j-2 are zeroed by both, rows j-1..j+1 are MGS values
                loss, re = f.lanczos_reorth(k)
                r[s, :j + 2] = f.H[:j + 2, j]
                r[s, lay.loss] = loss
                r[s, lay.flag] = 1.0 if re else 0.0
                self._gram(r, s, j + 1)
            r[s, lay.beta] = f.H[j + 1, j]
        self.pending = True
        self.next_step = j + 1
        return self._exchange(r)

    def flush(self, want=True):
        # the flush slot's records all-reduce (tk_decomp_flush), on every rank alike
        if self.pending:
            self.log.append("flush")
            self._exchange(np.zeros((self.d, self.m)))
            self.pending = False
        return np.zeros((self.d, self.m))

    def allreduce_host(self, x):
        return self._exchange(np.asarray(x, dtype=np.float64))

    def gram(self, f, k, want=True):
        # the ABI's rule (tk_decomp_gram): refused when the product would read the pending
        # column -- v_{j+1} after step j, or column j itself while it waits in the one-sweep
        # column buffer (even j, Arnoldi / Lanczos)
        j = self.next_step - 1
        in_e = self.method in ("TensorArnoldi", "TensorLanczos") and j % 2 == 0
        if self.pending and self._world() > 1 and k - 1 >= j + (0 if in_e else 1):
            raise RuntimeError("tk_decomp_gram: column pending; call tk_decomp_flush on every rank first")
        self.log.append("gram")
        V = self.f[self.loc[f]].V[:, :k]
        return V.T @ V

    def basis(self, f, c0, nc):
        return self.f[self.loc[f]].V[:, c0:c0 + nc].copy()

    def basis_mul(self, k, Ys, want=True):
        self.flush(False)   # (tk_decomp_basis_mul finalizes a pending column first)
        return [self.f[s].V[:, :k] @ Ys[i] for i, s in enumerate(self.loc)]

    def close(self):
        pass


def backend(td, b):
    """Factory for TensorDecomposition(backend=...)."""
    return FakeDecomposition(td, b)
