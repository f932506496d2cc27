#!/usr/bin/env python3
"""Summarize a TKHIP_SOLVER_TRACE file of the native loop (tk_solver_run): per iteration the
time its record was in hand, its evaluation start / end and its consumption (us from the loop
start), the record cadence, the evaluation times and where the loop's end goes.
usage: python tools/e2e_trace.py TRACE.csv [device_us_per_iteration]"""
import csv
import sys

lines = open(sys.argv[1]).read().splitlines()
if lines and lines[0].startswith("#"):
    print("native loop:", lines[0][1:].strip())
    lines = lines[1:]
rows = [{k: float(v) for k, v in r.items()} for r in csv.DictReader(lines)]
dev = float(sys.argv[2]) if len(sys.argv) > 2 else None
ks = [int(r["k"]) for r in rows]
rec = [r["record_us"] for r in rows]
ev = [r["eval_end_us"] - r["eval_start_us"] for r in rows]
wait = [r["eval_start_us"] - r["record_us"] for r in rows]
end = rows[-1]["consumed_us"]
print("iterations %d..%d, loop %.0f us; last record at %.0f us (%.0f us before the end)" % (ks[0], ks[-1], end, rec[-1], end - rec[-1]))
gaps = [b - a for a, b in zip(rec, rec[1:])]
print("record cadence: mean %.1f us (first half %.1f, second half %.1f)%s" % (
    sum(gaps) / len(gaps), sum(gaps[:len(gaps) // 2]) / (len(gaps) // 2), sum(gaps[len(gaps) // 2:]) / (len(gaps) - len(gaps) // 2),
    "; device %.1f us per iteration" % dev if dev else ""))
print("evaluation: mean %.1f us, max %.1f us (k=%d); submit -> start mean %.1f us" % (
    sum(ev) / len(ev), max(ev), ks[ev.index(max(ev))], sum(wait) / len(wait)))
for r in rows[-6:]:
    print("  k=%d record %.0f start %.0f end %.0f consumed %.0f" % (r["k"], r["record_us"], r["eval_start_us"], r["eval_end_us"], r["consumed_us"]))
