set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --emulate-ranks 8 > gpurun_out/e8_$i.log 2>&1 || { tail -5 gpurun_out/e8_$i.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e8_$i.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}
print('$i', d['value'], 'e2e', e.get('iterations_s'), e.get('relres_bitwise_equal_to_n1'))"
done
