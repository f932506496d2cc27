set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/ -q -m gpu > gpurun_out/t_gpu.log 2>&1; echo "pytest EXIT $?" >> gpurun_out/t_gpu.log
for C in C2 C3; do timeout -k 10 300 python bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$C.log 2>&1 || echo "bench $C failed" ; done
cd $R; tail -3 gpurun_out/t_gpu.log; for C in C2 C3; do python -c "
import json; d=json.loads(open('gpurun_out/bench_$C.log').read().strip().split('\n')[-1]); print('$C', d['value'], d['roofline']['achieved'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})"; done
