# round 4 A/B: factor groups 2 vs 3 (C1, C4, C2 Arnoldi), then the XCD mapping A/B and the C3
# evidence (probes, PMC)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do for cfg in C1 C4 C2; do for G in 2 3; do
  TKHIP_FACTOR_GROUPS=$G timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --config $cfg --steps 10 --warmup 2 > gpurun_out/g_${cfg}_$G.log 2>&1 || { echo "$cfg G=$G failed"; tail -5 gpurun_out/g_${cfg}_$G.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/g_${cfg}_$G.log').read().strip().splitlines()[-1])
print('rep $rep $cfg G=$G', d['value'], 'frac', d['roofline']['frac'], 'groups', d['roofline']['factor_groups'])"
done; done; done
bash tools/gpu/r4_xmap.sh || exit 1
bash tools/gpu/r4_c3.sh
bash tools/gpu/r4_e2e.sh
