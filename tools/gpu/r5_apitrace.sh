# host-side HIP API cost per Krylov iteration of an emulated N-rank step (CFG, RK; default C4 rank 0):
# rocprofv3 --hip-trace --stats (no counters), summarized per API call
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
export TKHIP_RED_MM=0
rm -rf $R/gpurun_out/api_tr
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $R/gpurun_out/api_tr -o run -- python3 $R/bench.py --config ${CFG:-C4} --emulate-ranks ${N:-8} --emulate-rank ${RK:-0} --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/api_tr.log 2>&1 || { echo "trace failed"; tail -5 $R/gpurun_out/api_tr.log; exit 1; }
cd $R
tail -1 gpurun_out/api_tr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'host_issue_us', d['host_issue_us_per_iteration'], 'step_us', d['roofline']['avg_launch_us'])"
ls gpurun_out/api_tr
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/api_tr/*stats*.csv")):
    rows = list(csv.DictReader(open(f)))
    print("==", f, len(rows))
    rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0) or 0))
    for r in rows[:25]:
        print("%-45s %8s %12.1f us avg %10.3f" % (r["Name"][:45], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
PY
