# Collective latency in the scaling prediction: emulated N=8 ranks with every
# records all-reduce held back TKHIP_TEST_XCH_DELAY_US on the exchange stream (a 1-rank
# communicator's all-reduce is a local copy; an 8-peer xGMI one costs tens of us).
# Device rate and end-to-end per delay; C2 rank 0, C4 ranks 0 (2 factors) and 7 (1 factor).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for spec in "C2 0" "C4 0" "C4 7"; do set -- $spec; cfg=$1; rk=$2
  for dl in 0 10 25 50; do
    TKHIP_TEST_XCH_DELAY_US=$dl timeout -k 10 300 python bench.py --config $cfg --emulate-ranks 8 --emulate-rank $rk --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/dly_${cfg}_${rk}_$dl.log 2>&1 || { echo "$cfg $rk $dl failed"; tail -3 gpurun_out/dly_${cfg}_${rk}_$dl.log; exit 1; }
    tail -1 gpurun_out/dly_${cfg}_${rk}_$dl.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d.get('end_to_end') or {}
print('$cfg rank $rk delay_us=$dl device', d['value'], 'step_us', d['roofline']['avg_launch_us'], 'xch_us', d['kernels']['exchange']['avg_us'], 'e2e', e.get('iterations_s'), 'e2e/dev %.3f' % (e.get('iterations_s', 0) / d['value']), 'relres==n1', e.get('relres_bitwise_equal_to_n1'))"
  done
done
