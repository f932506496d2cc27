#!/usr/bin/env python3
"""Extract golden fixtures from the reference's own recorded experiment data.

Run ONLY in the build container (it reads /root/reference, which does not exist on
the GPU box).  It writes small JSON fixtures next to this script; those fixtures are
committed and are what the tests read.

Source data (reference, read-only):
  experiments/data/reproduction_data/laplace_new  (Laplace, TensorLanczosReorth)
  experiments/data/reproduction_data/nonsym_new   (ConvDiff, TensorArnoldi)
written by experiments/reproduction.jl:9-23 -> experiments/experiment_common.jl:73-98
(`run_experiments!`) and :138-151 (`serialize_to_file`, Julia 1.9 `Serialization`).

The stream holds an `Experiment` (experiment_common.jl:37-62): dims=[5,10,50,100],
matrixsize=200, nmax, ..., `rhs_vec` (for each d, d normalized copies of one
rand(200) vector: src/system.jl:5-11 + :33-37), then one `ConvergenceData`
(src/convergence.jl:3-23) per d: niterations, iterations::Vector{Int},
relative_residual_norm, projected_residual_norm, orthogonality_data (all Float64).

We do not implement a full Julia deserializer; we use the fixed tags of the
concrete payloads (documented in SURVEY.md section 8c):
  Float64 array : 0x15 0x00 0x0e <len>   (len = 0x31 <int32>  or  1-byte 0xdf+len)
  Int64   array : 0x15 0x00 0x08 <len>
"""
import json
import os
import struct
import sys

REF = "/root/reference/experiments/data/reproduction_data"
HERE = os.path.dirname(os.path.abspath(__file__))
DIMS = [5, 10, 50, 100]


def _read_len(buf, p):
    tag = buf[p]
    if tag == 0x31:                      # Int32 follows
        return struct.unpack_from("<i", buf, p + 1)[0], p + 5
    if 0xdf <= tag < 0xdf + 32:          # small-int short form
        return tag - 0xdf, p + 1
    raise ValueError("unknown length tag 0x%02x at %d" % (tag, p))


def scan_arrays(buf):
    """Yield (offset, kind, values) for every Float64/Int64 1-d array in the stream."""
    p = 0
    n = len(buf)
    while p < n - 4:
        if buf[p] == 0x15 and buf[p + 1] == 0x00 and buf[p + 2] in (0x0E, 0x08):
            kind = "f64" if buf[p + 2] == 0x0E else "i64"
            try:
                L, q = _read_len(buf, p + 3)
            except ValueError:
                p += 1
                continue
            if 0 <= L <= 100000 and q + 8 * L <= n:
                fmt = "<%d%s" % (L, "d" if kind == "f64" else "q")
                vals = list(struct.unpack_from(fmt, buf, q))
                yield p, kind, vals
                p = q + 8 * L
                continue
        p += 1


def decode(fname):
    buf = open(os.path.join(REF, fname), "rb").read()
    arrs = list(scan_arrays(buf))
    # first Int64 array is `dims`
    assert arrs[0][1] == "i64" and arrs[0][2] == DIMS, arrs[0]
    f64 = [a for a in arrs if a[1] == "f64"]
    n_rhs = sum(DIMS)
    rhs = [a[2] for a in f64[:n_rhs]]
    assert all(len(r) == 200 for r in rhs)
    groups = {}
    p = 0
    for d in DIMS:
        g = rhs[p:p + d]
        p += d
        # random_rhs shares one vector; normalize! rebinds each slot to an equal copy
        assert all(x == g[0] for x in g), "rhs copies differ for d=%d" % d
        groups[d] = g[0]
    # ConvergenceData records: Int64 iterations array followed by 3 Float64 arrays
    rest = [a for a in arrs if a[0] > f64[n_rhs - 1][0]]
    conv = {}
    i = 0
    for d in DIMS:
        while rest[i][1] != "i64":
            i += 1
        its = rest[i][2]
        relres, proj, orth = (rest[i + 1][2], rest[i + 2][2], rest[i + 3][2])
        assert len(its) == len(relres) == len(proj) == len(orth)
        assert its == list(range(1, len(its) + 1))
        conv[d] = dict(niterations=len(its), relative_residual_norm=relres,
                       projected_residual_norm=proj, orthogonality_data=orth)
        i += 4
    return groups, conv


def main():
    if not os.path.isdir(REF):
        sys.exit("reference data not present (this script runs in the build container only)")
    out = {}
    for fname, cls, method in (("laplace_new", "Laplace", "TensorLanczosReorth"),
                               ("nonsym_new", "ConvDiff", "TensorArnoldi")):
        groups, conv = decode(fname)
        out[fname] = dict(
            source="/root/reference/experiments/data/reproduction_data/" + fname,
            matrix_class=cls, method=method, n=200, tol=1e-9,
            rhs={str(d): groups[d] for d in DIMS},
            convergence={str(d): conv[d] for d in DIMS})
        print(fname, {d: conv[d]["niterations"] for d in DIMS})
    with open(os.path.join(HERE, "reproduction.json"), "w") as f:
        json.dump(out, f)
    print("wrote", os.path.join(HERE, "reproduction.json"))


if __name__ == "__main__":
    main()
