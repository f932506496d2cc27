# predicted strong scaling: per-rank work of an N-GPU run, on one GPU (device rate and the
# end-to-end native loop with the other ranks' records overlaid from a full run)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/scale_1.log 2>&1 || { tail -5 gpurun_out/scale_1.log; exit 1; }
for N in 2 4 8; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --emulate-ranks $N > gpurun_out/scale_$N.log 2>&1 || { tail -5 gpurun_out/scale_$N.log; exit 1; }
done
for N in 1 2 4 8; do python3 -c "
import json; d=json.loads(open('gpurun_out/scale_$N.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}
print('$N', d['value'], d['ms_per_step'], d['roofline']['achieved'], {k:v['avg_us'] for k,v in d['kernels'].items()}, 'e2e', e.get('iterations_s'), e.get('vs_device_steps_only'), 'relres==n1', e.get('relres_bitwise_equal_to_n1'), 'split', e.get('eval_split'))"; done
