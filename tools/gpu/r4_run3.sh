# round 4, third box: grouped one-sweep Lanczos (its own test first, short limit), the C2
# TensorLanczos full-size parity test, C2 TensorLanczos with / without groups, native-loop traces
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 150 python -u -m pytest tests/test_gpu_groups.py -x -v --timeout 100 --timeout-method thread > gpurun_out/t_groups.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_groups.log | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k lanczos_all_8 -x -v -s --timeout 500 --timeout-method thread > gpurun_out/t_c2lan.log 2>&1; rc=$?
grep -E "C2 Lanczos|passed|failed|Error" gpurun_out/t_c2lan.log | tail -12
[ $rc -eq 0 ] || exit 1
for G in 1 2 3; do
  TKHIP_FACTOR_GROUPS=$G timeout -k 10 300 python bench.py --no-cpu-baseline --method TensorLanczos --steps 10 --warmup 2 > gpurun_out/lan_g$G.log 2>&1 || { echo "lan G=$G failed"; tail -5 gpurun_out/lan_g$G.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/lan_g$G.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('lanczos G=$G', d['value'], 'frac', d['roofline']['frac'], 'launch_us', d['roofline']['avg_launch_us'], 'e2e', e['iterations_s'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done
bash tools/gpu/r4_e2e.sh 2>&1 | grep -v "C2 Lanczos" 
