# round 4: factor groups at the emulated per-rank shares of C2 (N = 2: 4 factors, N = 4: 2) and
# C4 rank 0 (2 factors): TKHIP_FACTOR_GROUPS 1 / 2 (/ 3 at N = 2), two alternations
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
ab() {  # name, groups, bench args
  local nm=$1 g=$2; shift 2
  TKHIP_FACTOR_GROUPS=$g timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --steps 10 --warmup 2 "$@" > gpurun_out/grp_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/grp_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/grp_$nm.log').read().strip().splitlines()[-1])
print('== $nm G=$g', d['value'], d['roofline']['frac'], d['roofline']['factor_groups'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
}
for rep in a b; do
  for g in 1 2; do
    ab n4_g$g$rep $g --emulate-ranks 4 || exit 1
    ab n2_g$g$rep $g --emulate-ranks 2 || exit 1
    ab c4r0_g$g$rep $g --config C4 --emulate-ranks 8 --emulate-rank 0 || exit 1
  done
  ab n2_g3$rep 3 --emulate-ranks 2 || exit 1
done
