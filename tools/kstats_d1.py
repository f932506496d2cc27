#!/usr/bin/env python3
"""Per-launch achieved bandwidth of the one-sweep Arnoldi kernel (k_arn_d1<MAXC,FMT,MODE>)
from a rocprofv3 kernel-stats CSV of bench.py: MAXC = M serves steps j in (M-8, M]
(j <= 8 for M = 8), and one factor-step moves 8n(j + 3) algorithmic bytes (V[:,0..j),
u in, u out, v_j).  One launch carries d / G factors: with G = 2 factor
groups (tk_decomp_factor_groups; C2 at N = 1) each group's launch carries half of them, so the
bytes per launch are 8n(j+3) * d / G.  This is each launch's own rate; the two groups' launches
run concurrently, so the step's rate is in tools/trace_span.py (start / end timestamps).
usage: kstats_d1.py KERNEL_STATS.csv [n d K G]      (defaults: C2, 2^20 8 50 2)"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
n, d, K, G = (int(x) for x in sys.argv[2:6]) if len(sys.argv) > 5 else (1 << 20, 8, 50, 2)
agg = defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(path)):
    m = re.search(r"k_arn_d1<(\d+)", r["Name"])
    if not m:
        continue
    M = int(m.group(1))
    agg[M][0] += int(r["Calls"])
    agg[M][1] += float(r["TotalDurationNs"])
for M in sorted(agg):
    js = [j for j in range(K) if (j <= 8 if M == 8 else M - 8 < j <= M)]
    if not js:
        continue
    byts = sum(8 * n * (j + 3) for j in js) / len(js) * d / G
    calls, tot = agg[M]
    avg_ns = tot / calls
    print("k_arn_d1<%2d>  j %2d..%2d  calls %4d  avg %8.1f us  %6.0f GB/s per launch (%d factors)" %
          (M, js[0], js[-1], calls, avg_ns / 1e3, byts / avg_ns, d // G))
