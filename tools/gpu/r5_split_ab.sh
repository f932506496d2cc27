# end-to-end with and without the evaluation split (emulated N = 8 ranks)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for spec in "C4 7" "C4 0" "C2 0"; do set -- $spec; cfg=$1; rk=$2
  for sp in 1 0; do
    TKHIP_EVAL_SPLIT=$sp timeout -k 10 300 python bench.py --config $cfg --emulate-ranks 8 --emulate-rank $rk --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/spl_${cfg}_${rk}_$sp.log 2>&1 || { echo "$cfg $rk $sp failed"; tail -3 gpurun_out/spl_${cfg}_${rk}_$sp.log; exit 1; }
    tail -1 gpurun_out/spl_${cfg}_${rk}_$sp.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d.get('end_to_end') or {}
print('$cfg rank $rk split=$sp device', d['value'], 'host_issue', d['host_issue_us_per_iteration'], 'e2e', e.get('iterations_s'), e.get('iterations_s_all'), 'vs_steps', e.get('vs_device_steps_only'), e.get('eval_split'), e.get('split_table_eval_us'))"
  done
done
