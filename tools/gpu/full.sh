# smoke, the default bench line (C2 + CPU baseline), the other configs, rocprofv3 kernel
# stats of the default bench, and the two PMC passes (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_default.log; exit 1; }
for C in C1 C3 C4; do
  timeout -k 10 300 python bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -5 gpurun_out/bench_$C.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
# (profiles: the reduce hand-off's startup self-check runs a small one-sweep job of its own,
# whose kernels would be counted in with the workload's -- relaxed form forced, no check)
export TKHIP_RED_MM=0
rm -rf $R/gpurun_out/prof_c2 $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/prof_c2.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R
tail -1 gpurun_out/smoke.log
for C in default C1 C3 C4; do python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$C.log').read().strip().split('\n')[-1]); print('$C', d['value'], d['roofline']['achieved'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()}, 'e2e', (d.get('end_to_end') or {}).get('iterations_s'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; done
