# round 4: end-to-end A/B of the host worker count (TKHIP_SOLVER_THREADS 8 vs 12) where the
# host is throughput-bound (C4 emulated N=8 ranks 0 / 7) and at C4 / C2 emulated N=8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
ab() {  # name, bench args
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --e2e-reps 5 "$@" > gpurun_out/e2e4_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/e2e4_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e4_$nm.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $nm device', d['value'], 'e2e', e['iterations_s'], 'ratio %.3f' % (e['iterations_s'] / d['value']), 'all', e['iterations_s_all'], 'threads', e['host_threads'])"
}
echo "nproc $(nproc) affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') OMP_NUM_THREADS=$OMP_NUM_THREADS"
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
for rep in a b; do
  for th in 8 12; do
    TKHIP_SOLVER_THREADS=$th ab c4e8r0_p${th}$rep --config C4 --emulate-ranks 8 --emulate-rank 0 || exit 1
    TKHIP_SOLVER_THREADS=$th ab c4e8r7_p${th}$rep --config C4 --emulate-ranks 8 --emulate-rank 7 || exit 1
    TKHIP_SOLVER_THREADS=$th ab c4_p${th}$rep --config C4 || exit 1
    TKHIP_SOLVER_THREADS=$th ab c2e8_p${th}$rep --emulate-ranks 8 || exit 1
  done
done
