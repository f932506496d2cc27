#!/usr/bin/env python3
"""k_arn_d1 launches of the first timed sweep in a rocprofv3 --kernel-trace CSV: per step, each
launch's duration and the gap from the previous step kernel's end on any queue (diagnostic for
launch-order experiments).  usage: launch_gaps.py KERNEL_TRACE.csv [j ...]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    js = [int(x) for x in sys.argv[2:]] or [4, 10, 20, 30, 40, 48]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # the last complete sweep: from the last k_init_bd
    i0 = max(i for i, k in enumerate(ks) if "k_init_bd" in k[2])
    sw = [k for k in ks[i0:] if any(x in k[2] for x in ("k_arn_d1", "k_reduce256", "k_red_d1", "k_post"))]
    arn = [k for k in sw if "k_arn_d1" in k[2]]
    per = len(arn) // 50 if len(arn) >= 50 else 1
    print("sweep kernels %d, k_arn_d1 launches %d (%d per step)" % (len(sw), len(arn), per))
    for j in js:
        for q in range(per):
            s, e, name = arn[j * per + q]
            prev_end = max((k[1] for k in sw if k[1] <= s), default=s)
            print("j=%2d launch %d: %8.2f us  gap %6.2f us  %s" % (j, q, (e - s) / 1e3, (s - prev_end) / 1e3,
                                                                   name.split("<")[1].split(">")[0] if "<" in name else ""))
    span = (max(k[1] for k in sw) - min(k[0] for k in arn)) / 1e3
    print("sweep span %.1f us, per step %.2f us" % (span, span / 50))


if __name__ == "__main__":
    main()
