# iteration script: GPU tests, bench of all configs, kernel stats of C2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu -x > gpurun_out/t_gpu.log 2>&1; echo "pytest EXIT $?" >> gpurun_out/t_gpu.log
tail -1 gpurun_out/t_gpu.log | grep -q "EXIT 0" || { tail -30 gpurun_out/t_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --force-comm > gpurun_out/bench_C2_xch.log 2>&1 || { echo "bench force-comm failed"; tail -5 gpurun_out/bench_C2_xch.log; exit 1; }
for C in C2 C1 C3 C4; do timeout -k 10 300 python bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -5 gpurun_out/bench_$C.log; exit 1; }; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c2.log 2>&1
echo "prof EXIT $?"
cd $R; tail -2 gpurun_out/t_gpu.log
for C in C2_xch C2 C1 C3 C4; do python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$C.log').read().strip().split('\n')[-1]); print('$C', d['value'], d['roofline']['achieved'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()}, 'e2e', (d.get('end_to_end') or {}).get('iterations_s'))"; done
head -14 gpurun_out/prof_c2/run_kernel_stats.csv | cut -d, -f1-4
