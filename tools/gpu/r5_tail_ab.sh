# end-to-end of the emulated C4 N = 8 ranks 7 / 0 with the last iterations split into 3 or 4 helper tasks (TKHIP_SOLVER_TAIL_THREADS)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in a b; do for rk in 7 0; do for tt in 3 4; do
  TKHIP_SOLVER_TAIL_THREADS=$tt timeout -k 10 300 python bench.py --config C4 --emulate-ranks 8 --emulate-rank $rk --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/tail_${rk}_${tt}_$rep.log 2>&1 || { echo "fail $rk $tt"; tail -3 gpurun_out/tail_${rk}_${tt}_$rep.log; exit 1; }
  tail -1 gpurun_out/tail_${rk}_${tt}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d.get('end_to_end') or {}
print('$rep C4 rank $rk tail_threads $tt device', d['value'], 'e2e', e.get('iterations_s'), e.get('vs_device_steps_only'), e.get('iterations_s_all'))"
done; done; done
