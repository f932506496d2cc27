# round-6 evidence, part B: emulated strong scaling (C2 N = 1, 2, 4, 8, end-to-end with the
# evaluation split), per-rank N = 8 lines (C2 ranks 1, 5; C4 ranks 0, 7), the three methods at C2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu/scale.sh || exit 1
for r in 1 5; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --emulate-ranks 8 --emulate-rank $r > gpurun_out/rk8_$r.log 2>&1 || { echo "rank $r failed"; tail -5 gpurun_out/rk8_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/rk8_$r.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}
print('C2 rank $r', d['value'], d['ms_per_step'], 'e2e', e.get('iterations_s'), e.get('vs_device_steps_only'), {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done
for r in 0 7; do
  timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline --emulate-ranks 8 --emulate-rank $r > gpurun_out/c4rk8_$r.log 2>&1 || { echo "C4 rank $r failed"; tail -5 gpurun_out/c4rk8_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c4rk8_$r.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}
print('C4 rank $r', d['value'], d['ms_per_step'], d['roofline']['factor_groups'], 'e2e', e.get('iterations_s'), e.get('vs_device_steps_only'), e.get('eval_split'), {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done
for m in TensorArnoldi TensorLanczos TensorLanczosReorth; do
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --method $m > gpurun_out/method_$m.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/method_$m.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/method_$m.log').read().strip().split('\n')[-1]); print('$m', d['value'], d['roofline']['frac'], 'e2e', (d.get('end_to_end') or {}).get('iterations_s'), (d.get('end_to_end') or {}).get('vs_device_steps_only'))"
done
