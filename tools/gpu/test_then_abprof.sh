# GPU tests, then per-instance one-sweep kernel stats of variant libraries (args: names)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_gpu.log | head -20; exit 1; }
bash tools/gpu/abprof_d1.sh "$@"
