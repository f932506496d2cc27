#!/usr/bin/env python3
"""Block timeline of one k_arn_d1 launch (diagnostic; needs a library built with
`tools/build_variant.sh trace - -DTK_D1_TRACE=1`, selected by TKHIP_LIB).

usage: TKHIP_LIB=tools/_build/libtkhip_trace.so d1_trace.py NF J [J ...]
NF factors of the C2 Laplace problem (n = 2^20, K = 50); for each J prints the launch span,
block duration percentiles, how many blocks ran at once over time and per-XCD spans."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tensorkrylov.jl_amd"))
import tkamd  # noqa: E402
from tkamd import _lib as L  # noqa: E402


def main():
    nf = int(sys.argv[1])
    js = [int(x) for x in sys.argv[2:]]
    n, K = 1 << 20, 50
    lib = ctypes.CDLL(os.environ["TKHIP_LIB"])
    fn = lib.tk_debug_d1_trace
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    ctx = tkamd.Context(0)
    csc = tkamd.assemble_matrix(n, "Laplace")
    A = tkamd.DeviceMatrix(ctx, csc)
    bs = []
    for s in range(nf):
        b = np.random.default_rng(1000 + s).random(n)
        bs.append(b / np.linalg.norm(b))
    dev = tkamd.DeviceDecomposition(ctx, L.TK_ARNOLDI, nf, 0, [A] * nf, bs, K)
    for j in js:
        for rep in range(2):
            fn(j, None, 0)
            dev.init(False)
            dev.sweep(0, K)
            dev.flush(False)
            ctx.sync()
        buf = np.zeros(7 * 8192, dtype=np.uint64)
        fn(-1, buf.ctypes.data, 8192)
        tr = buf[:3 * 8192].reshape(-1, 3)
        ph = buf[3 * 8192:].reshape(-1, 4)
        keep = tr[:, 0] > 0
        tr, ph = tr[keep], ph[keep]
        t0 = tr[:, 0].min()
        st = (tr[:, 0] - t0).astype(np.float64) / 100.0    # us (100 MHz)
        en = (tr[:, 1] - t0).astype(np.float64) / 100.0
        du = en - st
        xcc = (tr[:, 2] >> np.uint64(32)).astype(np.int64) & 0xF
        hw = (tr[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        cu = (hw >> 8) & 0xF
        se = (hw >> 13) & 0x7
        print("j=%d blocks %d span %.2f us  dur p10/50/90/max %.2f %.2f %.2f %.2f  first-end %.2f  last-start %.2f"
              % (j, len(tr), en.max(), *np.percentile(du, [10, 50, 90]), du.max(), en.min(), st.max()))
        if ph[:, 3].min() > 0:   # phase clocks: median time from block start to each phase
            rel = (ph.astype(np.float64) - tr[:, :1].astype(np.float64)) / 100.0
            print("  phases (median us from block start): loads %.2f  spmv1 %.2f  spmv2 %.2f  dots %.2f  end %.2f"
                  % (*np.median(rel, axis=0), np.median(du)))
        # the XCD-aware slot map assumes the dispatcher deals blocks round-robin over the XCDs, so
        # slot range s // ceil(nwin / 8) runs on one XCD (XCC_ID numbers them in another order):
        # the share of each range's blocks on its most common XCD
        slots = np.nonzero(keep)[0]
        per = max(1, (len(tr) + 7) // 8)
        rng = slots // per
        held = sum(np.bincount(xcc[rng == r], minlength=16).max() for r in np.unique(rng))
        print("  slot ranges of %d on one XCD: %.1f %% of blocks" % (per, 100.0 * held / len(tr)))
        grid = np.arange(0, en.max() + 1.0, 1.0)
        act = [int(((st <= g) & (en > g)).sum()) for g in grid]
        print("  active blocks per us:", " ".join(str(a) for a in act))
        for x in range(8):
            m = xcc == x
            if m.any():
                print("  xcc %d: %4d blocks, start %.2f..%.2f end %.2f..%.2f, cus %d"
                      % (x, m.sum(), st[m].min(), st[m].max(), en[m].min(), en[m].max(),
                         len(set(zip(se[m].tolist(), cu[m].tolist())))))
    dev.close()
    A.close()
    ctx.close()


if __name__ == "__main__":
    main()
