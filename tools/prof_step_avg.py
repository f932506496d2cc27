#!/usr/bin/env python3
"""Average duration of one Arnoldi factor-step launch group (pass 1 + reduce + pass 2 +
reduce + post, or the one-sweep k_arn_d1 + reduce + post; all local factors) from a rocprofv3 --kernel-trace --stats summary, for
comparison with bench.py's live HIP-event figure (roofline.avg_launch_us).

usage: prof_step_avg.py KERNEL_STATS.csv SWEEPS K
"""
import csv
import sys

STEP = ("k_arn_a1", "k_arn_a2", "k_arn_d1", "k_reduce", "k_post")


def main():
    path, sweeps, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    tot = 0.0
    for r in csv.DictReader(open(path)):
        if any(s in r["Name"] for s in STEP):
            tot += float(r["TotalDurationNs"])
    # the init call issues one reduce + post pair of its own; it is a small share
    print("step-group avg over %d sweeps x %d steps: %.1f us" % (sweeps, K, tot / (sweeps * K) / 1e3))


if __name__ == "__main__":
    main()
