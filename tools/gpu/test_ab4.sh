set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^FAILED|Error" gpurun_out/t_gpu.log | head -5; tail -5 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
bash tools/gpu/ab4.sh prev cur occ3
