set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/ -q -m gpu > gpurun_out/t_gpu.log 2>&1; echo "pytest EXIT $?" >> gpurun_out/t_gpu.log
for C in C1 C3 C4; do timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$C.log 2>&1 || echo "bench $C failed" ; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_write.log 2>&1
echo "pmc EXIT $?"
cd $R; tail -3 gpurun_out/t_gpu.log; for C in C1 C3 C4; do tail -1 gpurun_out/bench_$C.log | cut -c1-400; done
