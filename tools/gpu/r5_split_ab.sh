# end-to-end of the emulated N = 8 ranks: evaluation split with the owners' calibrated times
# (default), split with the full run's times, and no split
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for spec in "${@:-C4:7}"; do cfg=${spec%%:*}; rk=${spec##*:}
  for v in "cal 1 1" "full 1 0" "nosplit 0 1"; do set -- $v; nm=$1; sp=$2; cb=$3
    TKHIP_EVAL_SPLIT=$sp TKHIP_EVAL_CALIBRATE=$cb timeout -k 10 300 python bench.py --config $cfg --emulate-ranks 8 --emulate-rank $rk --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/spl_${cfg}_${rk}_$nm.log 2>&1 || { echo "$cfg $rk $nm failed"; tail -3 gpurun_out/spl_${cfg}_${rk}_$nm.log; exit 1; }
    tail -1 gpurun_out/spl_${cfg}_${rk}_$nm.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d.get('end_to_end') or {}
print('$cfg rank $rk $nm device', d['value'], 'host_issue', d['host_issue_us_per_iteration'], 'e2e', e.get('iterations_s'), e.get('iterations_s_all'), 'vs_steps', e.get('vs_device_steps_only'), e.get('eval_split'), e.get('split_table_eval_us'))"
  done
done
