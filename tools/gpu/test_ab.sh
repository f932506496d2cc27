# full GPU suite on the working-tree library, then the same-box A/B (ab4.sh) of the named variants
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
bash tools/gpu/ab4.sh "$@"
