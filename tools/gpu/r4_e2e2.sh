# round 4: end-to-end A/B of the persistent tail helpers (TKHIP_SOLVER_TAIL_THREADS 1 vs 3),
# two alternations per config, 5 solves each (median reported), native-loop trace of each
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
tr() {  # name, bench args
  local nm=$1; shift
  TKHIP_SOLVER_TRACE=$R/gpurun_out/tr_$nm.csv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --e2e-reps 5 "$@" > gpurun_out/e2e_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/e2e_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e_$nm.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $nm device', d['value'], 'e2e', e['iterations_s'], 'ratio %.3f' % (e['iterations_s'] / d['value']), 'all', e['iterations_s_all'], 'phases', e['phases_s'])
print(1e6/d['value'])" > gpurun_out/e2e_$nm.txt
  head -1 gpurun_out/e2e_$nm.txt
  python3 tools/e2e_trace.py gpurun_out/tr_$nm.csv $(tail -1 gpurun_out/e2e_$nm.txt) > gpurun_out/trs_$nm.txt && sed -n 1,3p gpurun_out/trs_$nm.txt
}
for rep in a b; do
  for th in 1 3; do
    TKHIP_SOLVER_TAIL_THREADS=$th tr c4_t${th}$rep --config C4 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th tr c1_t${th}$rep --config C1 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th tr c4e8r0_t${th}$rep --config C4 --emulate-ranks 8 --emulate-rank 0 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th tr c4e8r7_t${th}$rep --config C4 --emulate-ranks 8 --emulate-rank 7 || exit 1
    TKHIP_SOLVER_TAIL_THREADS=$th tr c2e8_t${th}$rep --emulate-ranks 8 || exit 1
  done
done
