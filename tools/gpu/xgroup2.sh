# emulated N=8 device and end-to-end rates per record-exchange group size (two repetitions)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  BARGS="--emulate-ranks 8" bash tools/gpu/ab_env.sh n8g4:TKHIP_XCH_GROUP=4 n8g8:TKHIP_XCH_GROUP=8 n8g16:TKHIP_XCH_GROUP=16 n8nc:TK_EMULATE_NOCOMM=1 || exit 1
  for g in 4 8 16; do python3 -c "
import json; d=json.loads(open('gpurun_out/abe_n8g$g.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}
print('rep$rep g$g', d['value'], 'e2e', e.get('iterations_s'), 'relres==n1', e.get('relres_bitwise_equal_to_n1'))"; done
done
