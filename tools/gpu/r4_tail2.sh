# round 4: helpers offered to the last 8 iterations but spinning only for the last 2
# (TKHIP_SOLVER_TAIL_ITERS=8 TKHIP_SOLVER_HOT_ITERS=2) vs the default (2 / 2), end-to-end,
# two alternations, 5 solves per line
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
ab() {  # name, bench args
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --e2e-reps 5 "$@" > gpurun_out/t2_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/t2_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/t2_$nm.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $nm device', d['value'], 'e2e', e['iterations_s'], 'ratio %.3f' % (e['iterations_s'] / d['value']), 'all', e['iterations_s_all'])"
}
for rep in a b; do
  for ti in 2 8; do
    TKHIP_SOLVER_TAIL_ITERS=$ti ab c4_i${ti}$rep --config C4 || exit 1
    TKHIP_SOLVER_TAIL_ITERS=$ti ab c4e8r0_i${ti}$rep --config C4 --emulate-ranks 8 --emulate-rank 0 || exit 1
    TKHIP_SOLVER_TAIL_ITERS=$ti ab c4e8r7_i${ti}$rep --config C4 --emulate-ranks 8 --emulate-rank 7 || exit 1
    TKHIP_SOLVER_TAIL_ITERS=$ti ab c1_i${ti}$rep --config C1 || exit 1
    TKHIP_SOLVER_TAIL_ITERS=$ti ab c2_i${ti}$rep || exit 1
  done
done
