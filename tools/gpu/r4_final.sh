# round-4 final evidence at HEAD: GPU suite, smoke, bench lines (C2 + CPU baselines, C1, C3, C4),
# rocprofv3 kernel stats of C2, PMC FETCH/WRITE -> pmc_C2_n1.json, MFMA counters, emulated
# strong scaling (C2 N = 1, 2, 4, 8), per-rank N = 8 lines (C2 ranks 0, 1, 5; C4 ranks 0, 7),
# the three methods at C2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu/r3_tests.sh || exit 1
bash tools/gpu/r3_evidence1.sh || exit 1
bash tools/gpu/r3_evidence2.sh || exit 1
for r in 0 7; do
  timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline --emulate-ranks 8 --emulate-rank $r > gpurun_out/c4rk8_$r.log 2>&1 || { echo "C4 rank $r failed"; tail -5 gpurun_out/c4rk8_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c4rk8_$r.log').read().strip().split('\n')[-1]); e=d.get('end_to_end') or {}
print('C4 rank $r', d['value'], d['ms_per_step'], d['roofline']['factor_groups'], 'e2e', e.get('iterations_s'), {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done
