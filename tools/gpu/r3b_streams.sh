# does a second stream overlap launch drains / reduce latency? (tools/stream_probe.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for cfg in "2 20" "4 18" "8 20" "10 17"; do
  timeout -k 10 200 python tools/stream_probe.py $cfg >> gpurun_out/streams.log 2>&1 || { echo "probe $cfg failed"; tail -5 gpurun_out/streams.log; exit 1; }
done
cat gpurun_out/streams.log
