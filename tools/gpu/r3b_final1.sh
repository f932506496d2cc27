# round-end rehearsal at HEAD: the GPU suite, smoke and the default bench (what the driver runs)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu/r3_tests.sh || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_default.log; exit 1; }
tail -c 600 gpurun_out/bench_default.log
