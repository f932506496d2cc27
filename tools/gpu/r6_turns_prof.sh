# kernel traces of the C2 bench with factor groups taking turns (default) and on two streams
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp; cd $R
for v in 1 0; do
  TKHIP_D1_TURNS=$v timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tp$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/tp$v.log 2>&1 || { tail gpurun_out/tp$v.log; exit 1; }
  f=$(find gpurun_out/tp$v -name "*kernel_trace.csv" | head -1)
  echo "== TKHIP_D1_TURNS=$v"; tail -1 gpurun_out/tp$v.log | cut -c1-200
  python3 tools/launch_gaps.py $f
done
