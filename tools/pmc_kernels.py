#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 --pmc counters (one or more counter_collection.csv files),
plus derived ratios when the usual SQ counters are present.

usage: pmc_kernels.py COUNTER_COLLECTION.csv [...] [--match SUBSTR]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main():
    args = sys.argv[1:]
    match = None
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        args = args[:i] + args[i + 2:]
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in args:
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if match and match not in k:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    for k in sorted(tot):
        c = tot[k]
        n = len(disp[k])
        line = ["%-28s dispatches %4d" % (k, n)]
        for name in sorted(c):
            line.append("%s=%.4g" % (name, c[name] / n))
        if c.get("SQ_BUSY_CYCLES") and c.get("SQ_ACTIVE_INST_VALU"):
            # per-SIMD VALU issue share (SQ_ACTIVE_INST_VALU is summed over waves; per the
            # guide's convention divided by 4 SIMDs x CUs is left to the reader)
            line.append("valu/busy=%.3f" % (c["SQ_ACTIVE_INST_VALU"] / c["SQ_BUSY_CYCLES"]))
        if c.get("SQ_INSTS_LDS") and c.get("SQ_LDS_BANK_CONFLICT") is not None:
            line.append("lds_conflict/lds_inst=%.3f" % (c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_INSTS_LDS"], 1)))
        print("  ".join(line))


if __name__ == "__main__":
    main()
