#!/usr/bin/env python3
"""Per-kernel mean duration and mean idle gap before it (start minus the previous kernel's
end, same queue) from a rocprofv3 --kernel-trace CSV: where an iteration's time goes
between launches (e.g. bench.py --emulate-ranks 8, one factor per GPU).

usage: trace_gaps.py KERNEL_TRACE.csv [MIN_CALLS]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main():
    path = sys.argv[1]
    mincalls = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows = list(csv.DictReader(open(path)))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    by_q = defaultdict(list)
    for r in rows:
        by_q[r.get(qkey, "0")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    dur = defaultdict(list)
    gap = defaultdict(list)
    for q, ks in by_q.items():
        ks.sort()
        for i, (s, e, n) in enumerate(ks):
            dur[n].append(e - s)
            if i:
                g = s - ks[i - 1][1]
                if g < 200000:   # ignore host-side pauses between sweeps
                    gap[n].append(g)
    print("%-34s %7s %10s %10s" % ("kernel", "calls", "avg us", "gap us"))
    for n in sorted(dur, key=lambda n: -sum(dur[n])):
        if len(dur[n]) < mincalls:
            continue
        g = gap[n]
        print("%-34s %7d %10.2f %10.2f" % (n, len(dur[n]), sum(dur[n]) / len(dur[n]) / 1e3,
                                          (sum(g) / len(g) / 1e3) if g else float("nan")))


if __name__ == "__main__":
    main()
