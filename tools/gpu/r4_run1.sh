# round 4, first box: GPU suite, then the default C2 line, emulated C2 scaling (N = 2, 4, 8,
# rank 0) and C4's 8-GPU ranks (rank 0 holds 2 factors -- factor groups under the records
# exchange -- rank 7 holds 1), C1 and C4 at N = 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_gpu.log 2>&1
rc=$?; echo "pytest EXIT $rc" >> gpurun_out/t_gpu.log
grep -cE "PASSED" gpurun_out/t_gpu.log; grep -E "FAILED|ERROR" gpurun_out/t_gpu.log | tail -15
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || exit 1
run() {  # name, bench args
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/$nm.log; exit 1; }
  tail -1 gpurun_out/$nm.log > gpurun_out/$nm.json
  python3 -c "
import json; d=json.loads(open('gpurun_out/$nm.json').read()); e=d.get('end_to_end') or {}
print('$nm', d['value'], 'frac', d['roofline']['frac'], 'launch_us', d['roofline']['avg_launch_us'], 'groups', d['roofline'].get('factor_groups'), 'e2e', e.get('iterations_s'), 'relres==n1', e.get('relres_bitwise_equal_to_n1'), {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
}
run c2_n1 --steps 10 --warmup 2
for N in 2 4 8; do run c2_emu$N --steps 6 --warmup 1 --emulate-ranks $N; done
run c4_emu8_r0 --config C4 --steps 10 --warmup 2 --emulate-ranks 8 --emulate-rank 0
run c4_emu8_r7 --config C4 --steps 10 --warmup 2 --emulate-ranks 8 --emulate-rank 7
run c4_n1 --config C4 --steps 10 --warmup 2
run c1_n1 --config C1 --steps 10 --warmup 2
