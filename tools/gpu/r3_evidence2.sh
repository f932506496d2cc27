# round-3 evidence, part 2: emulated strong scaling, per-rank N=8 rates, the three methods at C2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu/scale.sh || exit 1
for r in 0 1 5; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end --emulate-ranks 8 --emulate-rank $r > gpurun_out/rk8_$r.log 2>&1 || { echo "rank $r failed"; tail -5 gpurun_out/rk8_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/rk8_$r.log').read().strip().split('\n')[-1]); print('rank $r', d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done
bash tools/gpu/methods.sh
