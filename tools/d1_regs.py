#!/usr/bin/env python3
"""Resource usage of every k_arn_d1 instantiation from a `hipcc -Rpass-analysis=kernel-resource-usage`
log (tools/d1_regs.sh writes it): MAXC, FMT, MODE, VGPRs, waves/SIMD, SGPR / VGPR spills."""
import re
import sys

cur, rows = None, []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: _ZN2tk8k_arn_d1ILi(\d+)ELi(\d+)ELi(\d+)E", line)
    if m:
        cur = {"k": tuple(int(x) for x in m.groups())}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("sspill", r"SGPRs Spill: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
for r in sorted(rows, key=lambda r: (r["k"][1], r["k"][0], r["k"][2])):
    print("k_arn_d1<%2d,%d,%d>  vgpr %3d  waves %d  sgpr-spill %3d  vgpr-spill %3d" %
          (r["k"] + (r.get("vgpr", -1), r.get("occ", -1), r.get("sspill", -1), r.get("vspill", -1))))
