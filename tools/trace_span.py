#!/usr/bin/env python3
"""Per-step SPAN of the one-sweep Arnoldi sweep from a rocprofv3 --kernel-trace CSV of
bench.py (start / end timestamps, not summed durations: with two factor groups the groups'
launches run concurrently on two streams, so summing their durations double-counts).

A sweep is the run of step kernels (k_arn_d1, k_reduce256, k_post) between a k_init_bd and
the next k_fin_vy / k_basis_mul.  Its span is the first k_arn_d1 start to the last step
kernel's end -- what bench.py's event pair around tk_decomp_sweep brackets -- and span / K is
comparable with the bench line's roofline.avg_launch_us.  Step j's span is the earliest
start of the j-th k_arn_d1 on any queue to the latest end of that queue's j-th step
kernels; with the algorithmic bytes of the step (8 n (j + 3) per factor, DESIGN.md section
4) it gives each register-row tier's effective bandwidth with both groups overlapped.

usage: trace_span.py KERNEL_TRACE.csv [K n d]     (defaults: C2, 50 2^20 8)"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    K, n, d = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (50, 1 << 20, 8)
    rows = list(csv.DictReader(open(path)))
    qk = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(qk, "0")) for r in rows)
    sweeps, cur = [], None
    for s, e, name, q in ks:
        if "k_init_bd" in name:
            cur = []
            sweeps.append(cur)
        elif cur is not None and ("k_fin_vy" in name or "k_basis_mul" in name):
            cur = None
        elif cur is not None and any(k in name for k in ("k_arn_d1", "k_reduce256", "k_post")):
            cur.append((s, e, name, q))
    spans, tiers = [], defaultdict(list)
    for sw in sweeps:
        d1 = [x for x in sw if "k_arn_d1" in x[2]]
        if len(d1) < K:
            continue
        spans.append((max(x[1] for x in sw) - min(x[0] for x in d1)) / K)
        # per queue: the j-th k_arn_d1 and the step kernels after it up to the next k_arn_d1
        perq = defaultdict(list)
        for x in sw:
            perq[x[3]].append(x)
        steps = defaultdict(lambda: [float("inf"), 0, None])
        for q, xs in perq.items():
            j = -1
            for s, e, name, _ in xs:
                if "k_arn_d1" in name:
                    j += 1
                    st = steps[j]
                    st[0] = min(st[0], s)
                    st[2] = int(re.search(r"k_arn_d1<(\d+)", name).group(1))
                if j >= 0:
                    steps[j][1] = max(steps[j][1], e)
        for j, (s, e, m) in steps.items():
            if j < K:
                tiers[m].append((j, e - s))
    if not spans:
        print("no complete sweep of %d steps found" % K)
        return
    print("sweeps: %d   per-step span (sweep span / K): median %.2f us, mean %.2f us, min %.2f us" %
          (len(spans), statistics.median(spans) / 1e3, statistics.mean(spans) / 1e3, min(spans) / 1e3))
    print("%-10s %8s %12s %10s" % ("tier", "steps", "span us", "TB/s"))
    for m in sorted(tiers):
        v = tiers[m]
        byts = statistics.mean(8.0 * n * (j + 3) * d for j, _ in v)
        dt = statistics.median(x for _, x in v)
        print("MAXC %-5d %8d %12.1f %10.2f" % (m, len(v), dt / 1e3, byts / dt / 1e3))


if __name__ == "__main__":
    main()
