# native-loop traces (TKHIP_SOLVER_TRACE) of the bench's end-to-end solve: C2 at N = 1 and the
# emulated C4 rank 7 (evaluation split on); record cadence vs the device step, evaluation times
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
tr() {  # name, bench args
  local nm=$1; shift
  TKHIP_SOLVER_STATS=1 TKHIP_SOLVER_TRACE=$R/gpurun_out/tr5_$nm.csv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --e2e-reps 3 "$@" > gpurun_out/e2e5_$nm.log 2> gpurun_out/e2e5_$nm.err || { echo "$nm failed"; tail -5 gpurun_out/e2e5_$nm.log gpurun_out/e2e5_$nm.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e5_$nm.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $nm device', d['value'], 'steps-only', e['device_steps_only_iterations_s'], 'e2e', e['iterations_s'], e['iterations_s_all'], 'phases', e['phases_s'])
print(1e6/e['device_steps_only_iterations_s'])" > gpurun_out/e2e5_$nm.txt
  head -1 gpurun_out/e2e5_$nm.txt
  tail -3 gpurun_out/e2e5_$nm.err
  python3 tools/e2e_trace.py gpurun_out/tr5_$nm.csv $(tail -1 gpurun_out/e2e5_$nm.txt)
}
tr c2
tr c4e8r7 --config C4 --emulate-ranks 8 --emulate-rank 7
