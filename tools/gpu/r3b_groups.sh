# factor groups on two streams (default) vs one stream (TKHIP_FACTOR_GROUPS=1): GPU suite, then
# C2 / C1 / C4 bench A/B, two repetitions
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_grp.log 2>&1
rc=$?; tail -3 gpurun_out/t_grp.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/t_grp.log | head; exit 1; }
for rep in 1 2; do for C in C2 C1 C4; do for G in 1 2; do
  TKHIP_FACTOR_GROUPS=$G timeout -k 10 300 python bench.py --config $C --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/grp_${C}_$G.log 2>&1 || { echo "bench $C $G failed"; tail -5 gpurun_out/grp_${C}_$G.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/grp_${C}_$G.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}; print('rep$rep $C groups=$G', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('avg_launch_us'), 'e2e', e.get('iterations_s'))"
done; done; done
