# grouped record exchange: exchange-path GPU tests, then the emulated N=8 rank and N=1 per
# group size (TKHIP_XCH_GROUP)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_properties.py -x -v -m gpu --timeout 200 --timeout-method thread -k "exchange" > gpurun_out/t_xch.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_xch.log; exit 1; }
tail -1 gpurun_out/t_xch.log
BARGS="--emulate-ranks 8" bash tools/gpu/ab_env.sh n8g1:TKHIP_XCH_GROUP=1 n8g2:TKHIP_XCH_GROUP=2 n8g4:TKHIP_XCH_GROUP=4 n8g8:TKHIP_XCH_GROUP=8 n8g16:TKHIP_XCH_GROUP=16 || exit 1
for g in 1 4 8; do python3 -c "
import json; d=json.loads(open('gpurun_out/abe_n8g$g.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}; print('g$g e2e', e.get('iterations_s'), 'relres==n1', e.get('relres_bitwise_equal_to_n1'))"; done
