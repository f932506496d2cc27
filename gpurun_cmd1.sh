set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/t1.log 2>&1; echo "pytest EXIT $?" >> gpurun_out/t1.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_c2.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c2.log 2>&1
echo "chain EXIT $?"
tail -3 $R/gpurun_out/t1.log; cat $R/gpurun_out/smoke.log | tail -2; cat $R/gpurun_out/bench_c2.log | tail -2
