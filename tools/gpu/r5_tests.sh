# GPU suite, then the north-star parity tests again with their printed errors kept
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_northstar.py -v -s -m gpu --timeout 240 --timeout-method thread > gpurun_out/northstar.log 2>&1 || { tail -20 gpurun_out/northstar.log; exit 1; }
grep -E "C2 |PASS|passed" gpurun_out/northstar.log
