# quick: default bench (no CPU baseline) + C1 / C4 lines
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for C in C2 C1 C4; do
  TKHIP_SOLVER_STATS=1 timeout -k 10 300 python bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bq_$C.log 2>gpurun_out/bq_$C.err || { echo "bench $C failed"; tail -5 gpurun_out/bq_$C.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bq_$C.log').read().strip().split('\n')[-1]); print('$C', d['value'], d['roofline']['frac'], 'e2e', d['end_to_end']['iterations_s'], d['end_to_end']['phases_s'], d['orthogonality_gram'].get('avg_us'))"; cat gpurun_out/bq_$C.err
done
