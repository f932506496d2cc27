#!/usr/bin/env python3
"""Per-kernel achieved bandwidth of the Arnoldi pass kernels from a rocprofv3 kernel-stats
CSV of bench.py (C2 defaults): each template instance covers a known range of steps j,
so its algorithmic bytes follow from DESIGN.md section 4.
usage: kstats_bw.py KERNEL_STATS.csv [n d K]"""
import csv
import re
import sys

path = sys.argv[1]
n, d, K = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (1 << 20, 8, 50)


def jrange(kind, M):
    # which steps j use MAXC = M (see launchers: a1_fused by j, a2/finalize by j+1)
    lo = M - 8
    if kind == "a1_fused":
        js = [j for j in range(1, K) if lo < j <= M]
    elif kind == "a1_plain":
        js = [0]
    else:
        js = [j for j in range(K) if lo < j + 1 <= M]
    return js


for r in csv.DictReader(open(path)):
    m = re.search(r"k_arn_(a1_fused|a1_plain|a2)<(\d+)", r["Name"])
    if not m:
        continue
    kind, M = m.group(1), int(m.group(2))
    js = jrange(kind, M)
    if not js:
        continue
    calls = int(r["Calls"])
    avg_us = float(r["AverageNs"]) / 1e3
    jm = sum(js) / len(js)
    if kind == "a1_fused":      # V[:,0..j) + write v_j, W; read U (+gathers), dval 3n
        cols = jm + 1 + 1 + 1 + 3
    elif kind == "a1_plain":
        cols = 1 + 1 + 3
    else:                       # V[:,0..j], W, b, write U
        cols = jm + 1 + 3
    byts = 8.0 * n * cols * d
    print("%-9s MAXC=%2d j~%5.1f calls=%3d avg=%8.1f us  %.2f TB/s" % (kind, M, jm, calls, avg_us,
                                                                     byts / (avg_us * 1e-6) / 1e12))
