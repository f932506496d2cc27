# round 4: the host's record polls with a pause between reads (default) vs tight (variant
# tools/_build/libtkhip_nopause.so, -DTK_POLL_PAUSE=0): end-to-end at C2 / C4, two alternations,
# and the driver's record cadence (TKHIP_SOLVER_TRACE) of one C2 solve each
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
D=$R/tensorkrylov.jl_amd/tkamd/libtkhip.so; N=$R/tools/_build/libtkhip_nopause.so
ab() {  # name, lib, bench args
  local nm=$1 lib=$2; shift 2
  TKHIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --e2e-reps 5 "$@" > gpurun_out/pl_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/pl_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/pl_$nm.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $nm device', d['value'], 'e2e', e['iterations_s'], 'ratio %.3f' % (e['iterations_s'] / d['value']), 'all', e['iterations_s_all'])"
}
for rep in a b; do
  ab c2_pause$rep $D || exit 1
  ab c2_tight$rep $N || exit 1
  ab c4_pause$rep $D --config C4 || exit 1
  ab c4_tight$rep $N --config C4 || exit 1
done
for v in pause tight; do
  lib=$D; [ $v = tight ] && lib=$N
  TKHIP_LIB=$lib TKHIP_SOLVER_TRACE=$R/gpurun_out/trp_$v.csv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --e2e-reps 1 > gpurun_out/plt_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  dv=$(python3 -c "import json; d=json.loads(open('gpurun_out/plt_$v.log').read().strip().splitlines()[-1]); print(1e6/d['value'])")
  python3 tools/e2e_trace.py gpurun_out/trp_$v.csv $dv > gpurun_out/trps_$v.txt && sed -n 1,4p gpurun_out/trps_$v.txt
done
