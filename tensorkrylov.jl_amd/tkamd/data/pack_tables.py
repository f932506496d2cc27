#!/usr/bin/env python3
"""Pack the reference's exponential-sum coefficient tables into one compact .npz.

Data, not code: `coefficients_data/output_data/tabelle_complete.csv` (max error of the
best rank-t exponential sum 1/x ~ sum_j w_j exp(-a_j x) on [1, R], rows R, columns
t = 1..63) and the 2,771 `coefficients_data/1_xk{t:02d}.{digit}_{order}` files
(first t numbers = w, next t = a), read by src/approximation.jl:44-54 and :119-147.

Run ONLY in the build container (reads /root/reference).  The .npz it writes ships
with the package so the GPU box never needs the reference tree.  Numbers are parsed
with Python's correctly rounded float(), the same value CSV.jl/Parsers.jl yields.
"""
import os
import sys

import numpy as np

SRC = "/root/reference/coefficients_data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "expsum_tables.npz")


def main():
    if not os.path.isdir(SRC):
        sys.exit("reference tables not present (build container only)")
    lines = open(os.path.join(SRC, "output_data", "tabelle_complete.csv")).read().strip().split("\n")
    header = lines[0].split(",")
    assert header[0] == "R" and header[1:] == [str(t) for t in range(1, 64)]
    rows = [[float(x) for x in ln.split(",")] for ln in lines[1:]]
    tab = np.array(rows, dtype=np.float64)
    arrays = {"R": tab[:, 0].copy(), "err": tab[:, 1:].copy()}
    for f in sorted(os.listdir(SRC)):
        if not f.startswith("1_xk"):
            continue
        t = int(f[4:6])
        vals = [float(ln.split("{")[0]) for ln in open(os.path.join(SRC, f)).read().strip().split("\n")]
        assert len(vals) == 2 * t, f
        arrays["xk" + f[4:]] = np.array(vals, dtype=np.float64)   # key e.g. 'xk05.1_2'
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, len(arrays) - 2, "coefficient sets")


if __name__ == "__main__":
    main()
