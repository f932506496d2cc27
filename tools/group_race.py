"""Diagnostic (GPU): factor groups under a records exchange with group 0 held back
(TKHIP_TEST_GROUP_DELAY_US), one shared signal word (TKHIP_TEST_SHARED_XSIG=1, the round-4
form) against per-factor words (the default).  Prints how many exchanged record rows differ
from the one-stream local run -- the shared word's count shows the race the per-factor words
close (tests/test_gpu_groups.py::test_factor_groups_exchange_waits_for_every_group)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tensorkrylov.jl_amd"))
import tkamd as tk  # noqa: E402


def run(c, G, d, n, K, bs, mat):
    os.environ["TKHIP_FACTOR_GROUPS"] = G
    A = tk.DeviceMatrix(c, mat)
    dev = tk.DeviceDecomposition(c, 0, d, 0, [A] * d, bs, K)
    dev.init(False)
    dev.sweep(0, K)
    r = dev.records(0, K + 1)
    dev.close()
    A.close()
    return r


def main():
    d, n, K = 3, 1 << 15, 30
    rng = np.random.default_rng(12)
    mat = tk.assemble_matrix(n, "ConvDiff")
    bs = [v / np.linalg.norm(v) for v in (rng.random(n) for _ in range(d))]
    ctx = tk.Context(0)
    local = run(ctx, "1", d, n, K, bs, mat)
    c2 = tk.Context(0)
    c2.init_comm(tk.unique_id(), 1, 0)
    os.environ["TKHIP_EXCHANGE_ALWAYS"] = "1"
    os.environ["TKHIP_TEST_GROUP_DELAY_US"] = os.environ.get("DELAY", "300")
    for fuse in ("0", "1"):
        os.environ["TKHIP_D1_FUSE"] = fuse
        for shared in ("1", "0"):
            os.environ["TKHIP_TEST_SHARED_XSIG"] = shared
            bad = []
            for _ in range(3):
                r = run(c2, "2", d, n, K, bs, mat)
                bad.append(int(sum(not np.array_equal(local[s, f], r[s, f]) for s in range(K + 1) for f in range(d))))
            print("fuse=%s shared_word=%s differing record rows per run: %s" % (fuse, shared, bad), flush=True)
    c2.close()
    ctx.close()


if __name__ == "__main__":
    main()
