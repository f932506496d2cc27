#!/usr/bin/env python3
"""Dump config C3's A_s in the SELL-256 layout libtkhip builds (tk_abi.cpp build_sell: slice =
256-row tile, entry q of row r at sptr[r/256] + q*256 + r%256, ascending columns per row,
padding slots repeat the row index) for tools/gatherprobe.hip, which replays the SpMV's exact
index stream.  usage: c3_sell_dump.py OUT.bin [n]

File: int64 n, int64 slots, int64 ntiles; int64 sptr[ntiles]; int32 swidth[ntiles];
int32 rowlen[ntiles*256]; int32 scol[slots]; float64 sval[slots].
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tensorkrylov.jl_amd"))
import tkamd  # noqa: E402


def sell(n, colptr, rowval, nzval):
    # CSC -> CSR with ascending columns per row (the scatter mul!'s order)
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(colptr))
    order = np.lexsort((cols, rowval))
    r, c, v = rowval[order], cols[order], nzval[order]
    rl = np.bincount(r, minlength=n).astype(np.int32)
    rp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(rl, out=rp[1:])
    nt = (n + 255) // 256
    rlp = np.zeros(nt * 256, dtype=np.int32)
    rlp[:n] = rl
    sw = rlp.reshape(nt, 256).max(axis=1).astype(np.int32)
    sptr = np.zeros(nt, dtype=np.int64)
    np.cumsum(sw[:-1].astype(np.int64) * 256, out=sptr[1:])
    slots = int(sw.astype(np.int64).sum() * 256)
    scol = np.zeros(slots, dtype=np.int32)
    sval = np.zeros(slots)
    rows = np.arange(nt * 256)
    scol_default = np.minimum(rows, n - 1)
    for t in range(nt):
        w = int(sw[t])
        base = int(sptr[t])
        for q in range(w):
            rr = rows[t * 256:(t + 1) * 256]
            e = base + q * 256 + np.arange(256)
            inrow = (rr < n) & (q < rlp[t * 256:(t + 1) * 256])
            src = rp[np.minimum(rr, n - 1)] + q
            scol[e] = np.where(inrow, c[np.minimum(src, len(c) - 1)], scol_default[t * 256:(t + 1) * 256])
            sval[e] = np.where(inrow, v[np.minimum(src, len(v) - 1)], 0.0)
    return sptr, sw, rlp, scol, sval


def main():
    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 19
    colptr, rowval, nzval = tkamd.assemble_matrix(n, "RandSparseSPD")
    sptr, sw, rl, scol, sval = sell(n, colptr, rowval, nzval)
    with open(out, "wb") as f:
        np.array([n, len(scol), len(sptr)], dtype=np.int64).tofile(f)
        sptr.tofile(f)
        sw.tofile(f)
        rl.tofile(f)
        scol.tofile(f)
        sval.tofile(f)
    print("n=%d nnz=%d slots=%d (%.2f x nnz) mean width %.1f" % (n, len(nzval), len(scol), len(scol) / len(nzval),
                                                               sw.mean()))


if __name__ == "__main__":
    main()
