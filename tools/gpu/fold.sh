# GPU tests, then C2 (N=1 and emulated N=8 with and without the exchange), C1, C4
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/t_gpu.log | head -20; tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
BARGS="--no-end-to-end" bash tools/gpu/ab_env.sh n1:X=1 || exit 1
BARGS="--emulate-ranks 8" bash tools/gpu/ab_env.sh n8:X=1 n8nocomm:TK_EMULATE_NOCOMM=1 || exit 1
BARGS="--config C1 --no-end-to-end" bash tools/gpu/ab_env.sh c1:X=1 || exit 1
BARGS="--config C4 --no-end-to-end" bash tools/gpu/ab_env.sh c4:X=1 || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/abe_n8.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}; print('n8 e2e', e.get('iterations_s'), 'relres==n1', e.get('relres_bitwise_equal_to_n1'))"
