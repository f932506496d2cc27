#!/usr/bin/env python3
"""Per-instance achieved bandwidth of the one-sweep Arnoldi kernel (k_arn_d1<MAXC,FMT>)
from a rocprofv3 kernel-stats CSV of bench.py: MAXC = M serves steps j in (M-8, M]
(j <= 8 for M = 8), and one factor-step moves 8n(j + 3) algorithmic bytes (V[:,0..j),
u in, u out, v_j).
usage: kstats_d1.py KERNEL_STATS.csv [n d K]"""
import csv
import re
import sys

path = sys.argv[1]
n, d, K = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (1 << 20, 8, 50)
for r in csv.DictReader(open(path)):
    m = re.search(r"k_arn_d1<(\d+)", r["Name"])
    if not m:
        continue
    M = int(m.group(1))
    js = [j for j in range(K) if (j <= 8 if M == 8 else M - 8 < j <= M)]
    byts = sum(8 * n * (j + 3) for j in js) / len(js) * d
    avg_ns = float(r["AverageNs"])
    print("k_arn_d1<%2d>  j %2d..%2d  calls %4s  avg %8.1f us  %6.0f GB/s" %
          (M, js[0], js[-1], r["Calls"], avg_ns / 1e3, byts / avg_ns))
