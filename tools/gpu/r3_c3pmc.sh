# C3: parity of the shared-matrix path, the bench line, kernel stats, and PMC passes
# (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) of one sweep -> gpurun_out/pmc_C3_n1.json
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "shared_matrix or C3 or RandSparse" --timeout 300 --timeout-method thread > gpurun_out/t_c3.log 2>&1
rc=$?; tail -2 gpurun_out/t_c3.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --config C3 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_C3.log 2>&1 || { echo "bench C3 failed"; tail -5 gpurun_out/bench_C3.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_C3.log').read().strip().split('\n')[-1]); print('C3', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_c3 $R/gpurun_out/pmc_c3_*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -o run -- python3 $R/bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/prof_c3.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_c3_fetch -o run -- python3 $R/bench.py --config C3 --pmc-mode > $R/gpurun_out/pmc_c3_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_c3_write -o run -- python3 $R/bench.py --config C3 --pmc-mode > $R/gpurun_out/pmc_c3_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc_c3_tcc -o run -- python3 $R/bench.py --config C3 --pmc-mode > $R/gpurun_out/pmc_c3_tcc.log 2>&1 || { echo "pmc tcc failed"; exit 1; }
cd $R
python3 tools/pmc_traffic.py gpurun_out/pmc_c3_fetch gpurun_out/pmc_c3_write C3 1 50 gpurun_out/pmc_C3_n1.json
find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs head -8
