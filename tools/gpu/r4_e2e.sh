# round 4: native-loop traces (TKHIP_SOLVER_TRACE) of the bench's end-to-end run: C1, C4, C2 / C4 emulated N=8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
tr() {  # name, bench args
  local nm=$1; shift
  TKHIP_SOLVER_TRACE=$R/gpurun_out/tr_$nm.csv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 "$@" > gpurun_out/e2e_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/e2e_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e_$nm.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $nm device', d['value'], 'e2e', e['iterations_s'], 'phases', e['phases_s'])
print(1e6/d['value'])" > gpurun_out/e2e_$nm.txt
  head -1 gpurun_out/e2e_$nm.txt
  python3 tools/e2e_trace.py gpurun_out/tr_$nm.csv $(tail -1 gpurun_out/e2e_$nm.txt)
}
tr c1 --config C1
tr c4 --config C4
tr c2e8 --emulate-ranks 8
tr c4e8r7 --config C4 --emulate-ranks 8 --emulate-rank 7
tr c2 


TKHIP_SOLVER_TAIL_THREADS=1 tr c4_tail1 --config C4
TKHIP_SOLVER_TAIL_THREADS=1 tr c4e8r7_tail1 --config C4 --emulate-ranks 8 --emulate-rank 7
TKHIP_SOLVER_TAIL_THREADS=1 tr c1_tail1 --config C1
