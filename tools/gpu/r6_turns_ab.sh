# factor groups taking turns: GPU tests, launch gaps, A/B against two streams
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_groups.py} -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tp1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/tp1.log 2>&1 || { tail gpurun_out/tp1.log; exit 1; }
python3 tools/launch_gaps.py $(find gpurun_out/tp1 -name "*kernel_trace.csv" | head -1)
CASES="${CASES:-C2:1 C1:1 C4:1 C2:2 C2:4}" bash tools/gpu/r6_ab.sh "$@"
