# kernel stats of the C2 bench on one stream (TKHIP_FACTOR_GROUPS=1) and with the default groups
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 2; do
  TKHIP_FACTOR_GROUPS=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/os$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/os$v.log 2>&1 || { tail gpurun_out/os$v.log; exit 1; }
  echo "== groups $v"; tail -1 gpurun_out/os$v.log | cut -c1-160
  head -12 $(find gpurun_out/os$v -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
done
