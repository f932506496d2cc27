set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for N in 8 2; do
TKHIP_SOLVER_STATS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-ranks $N > gpurun_out/e2e_$N.log 2>&1 || { tail -5 gpurun_out/e2e_$N.log; exit 1; }
grep tk_solver_run gpurun_out/e2e_$N.log
python3 -c "
import json; d=json.loads(open('gpurun_out/e2e_$N.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}
print('$N', d['value'], 'e2e', e.get('iterations_s'), e.get('relres_bitwise_equal_to_n1'))"
done
