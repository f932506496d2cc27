# records-exchange grouping at emulated N = 8: device rate and end-to-end per TKHIP_XCH_GROUP
# (slots per all-reduce), plus the no-exchange bound (TK_EMULATE_NOCOMM=1)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in a b; do for cf in "C4 7" "C4 0" "C2 0"; do set -- $cf
  VARS=("g4 TKHIP_XCH_GROUP=4" "g8 TKHIP_XCH_GROUP=8" "g16 TKHIP_XCH_GROUP=16" "nocomm TK_EMULATE_NOCOMM=1")
  [ -n "$QUICK" ] && VARS=("g4 TKHIP_XCH_GROUP=4" "nocomm TK_EMULATE_NOCOMM=1")
  for v in "${VARS[@]}"; do set -- $cf $v
    env $4 timeout -k 10 300 python bench.py --config $1 --emulate-ranks 8 --emulate-rank $2 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/xg_$3_$1_$2_$rep.log 2>&1 || { echo "$3 $1 $2 failed"; tail -3 gpurun_out/xg_$3_$1_$2_$rep.log; exit 1; }
    tail -1 gpurun_out/xg_$3_$1_$2_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d.get('end_to_end') or {}
print('$rep $1 rank $2 $3', d['value'], d['roofline']['avg_launch_us'], 'e2e', e.get('iterations_s'), e.get('vs_device_steps_only'), {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
  done
done; done
