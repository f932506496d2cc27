# round 4: why emulated N=8 rank 0 (factor 1, its Gram) is slower than rank 5: kernel stats of both
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for r in 0 5; do
  rm -rf $R/gpurun_out/prof_rk$r
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_rk$r -o run -- python3 $R/bench.py --emulate-ranks 8 --emulate-rank $r --no-cpu-baseline --no-end-to-end --steps 5 --warmup 1 > $R/gpurun_out/prof_rk$r.log 2>&1 || { echo "prof $r failed"; tail -5 $R/gpurun_out/prof_rk$r.log; exit 1; }
done
cd $R
python3 - <<'PY'
import csv
for r in (0, 5):
    rows = list(csv.DictReader(open("gpurun_out/prof_rk%d/run_kernel_stats.csv" % r)))
    tot = sum(float(x["TotalDurationNs"]) for x in rows)
    print("rank", r, "total kernel ms %.2f" % (tot / 1e6))
    for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:12]:
        print("   %-60s %5s calls %9.1f us total %7.1f us avg" % (x["Name"][:60], x["Calls"], float(x["TotalDurationNs"]) / 1e3, float(x["AverageNs"]) / 1e3))
PY
