# GPU tests (thread timeouts so a hang names its test), then full.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
bash tools/gpu/full.sh
