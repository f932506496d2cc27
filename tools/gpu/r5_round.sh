# GPU suite (all of it), then the given extra command file steps (args: scripts to source)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_gpu.log | head -30; exit 1; }
