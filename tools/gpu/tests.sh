# pytest -m gpu (all GPU parity tests; -s keeps the per-config error prints), then the
# default bench line (C2 + the 1-core / all-cores CPU baselines)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_gpu.log 2>&1
rc=$?; echo "pytest EXIT $rc" >> gpurun_out/t_gpu.log
grep -E "factor [0-9]+:|PASSED|FAILED|ERROR" gpurun_out/t_gpu.log | tail -60
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || exit 1
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
