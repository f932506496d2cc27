# host time per part of a step's issue (TKHIP_HOST_PROFILE=1, printed at exit): C2 at N = 1 and
# the emulated C4 ranks 0 / 7 and C2 rank 0 of N = 8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for spec in "C2 1 0" "C4 8 0" "C4 8 7" "C2 8 0"; do set -- $spec
  TKHIP_HOST_PROFILE=1 timeout -k 10 200 python bench.py --config $1 --emulate-ranks $2 --emulate-rank $3 --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/hp_$1_$2_$3.log 2> gpurun_out/hp_$1_$2_$3.err || { echo "$spec failed"; tail -5 gpurun_out/hp_$1_$2_$3.err; exit 1; }
  echo "== $1 N=$2 rank $3: $(tail -1 gpurun_out/hp_$1_$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'it/s, host issue', d['host_issue_us_per_iteration'], 'us/step, device', d['roofline']['avg_launch_us'], 'us/step')")"
  grep -A 12 "tkhip host profile" gpurun_out/hp_$1_$2_$3.err
done
