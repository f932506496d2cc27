# round 6: the new multi-process / test-build tests first, then the whole GPU suite
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_boundary.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1; rc=$?
tail -15 gpurun_out/t_new.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/t_gpu.log
exit $rc
