# C2 with each orthonormalization type (device sweep rate + end-to-end loop)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for m in TensorArnoldi TensorLanczos TensorLanczosReorth; do
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --method $m > gpurun_out/method_$m.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/method_$m.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/method_$m.log').read().strip().split('\n')[-1]); print('$m', d['value'], d['roofline']['achieved'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()}, 'e2e', (d.get('end_to_end') or {}).get('iterations_s'), 'host', d['host_issue_us_per_iteration'])"
done
