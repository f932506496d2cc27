# round 4: GPU tests touching the native loop / Gram, then end-to-end A/B (no trace) of the
# tail helpers (TKHIP_SOLVER_TAIL_THREADS 1 vs 3), native orthogonality losses in both
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_groups.py tests/test_gpu_properties.py tests/test_gpu_solution.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t_e2e3.log 2>&1
rc=$?; tail -3 gpurun_out/t_e2e3.log; [ $rc -eq 0 ] || exit 1
ab() {  # name, bench args
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --e2e-reps 5 "$@" > gpurun_out/e2e3_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/e2e3_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e3_$nm.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $nm device', d['value'], 'e2e', e['iterations_s'], 'ratio %.3f' % (e['iterations_s'] / d['value']), 'all', e['iterations_s_all'], 'phases', e['phases_s'])"
}
for rep in a b; do
  for th in 1 3; do
    TKHIP_SOLVER_TAIL_THREADS=$th ab c4_t${th}$rep --config C4 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th ab c1_t${th}$rep --config C1 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th ab c4e8r0_t${th}$rep --config C4 --emulate-ranks 8 --emulate-rank 0 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th ab c4e8r7_t${th}$rep --config C4 --emulate-ranks 8 --emulate-rank 7 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th ab c2e8_t${th}$rep --emulate-ranks 8 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th ab c2_t${th}$rep || exit 1
  done
done
