# round 6: the new multi-process / test-build tests
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_boundary.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/t_new.log | tail -30
exit $rc
