# round 4: GPU suite with the single-column Lanczos layout, then C2 TensorLanczos A/B
# (TKHIP_LANCZOS_SL 1 vs 0, two alternations), rocprof kernel stats of both
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu/r3_tests.sh || exit 1
lb() {  # name, env value
  TKHIP_LANCZOS_SL=$2 timeout -k 10 300 python bench.py --method TensorLanczos --no-cpu-baseline --steps 10 --warmup 2 --e2e-reps 3 "${@:3}" > gpurun_out/lan_$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/lan_$1.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/lan_$1.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $1 SL=$2', d['value'], d['roofline']['frac'], d['roofline'].get('avg_launch_us'), {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']}, 'e2e', e['iterations_s'])"
}
for rep in a b; do
  lb sl1$rep 1 || exit 1
  lb sl0$rep 0 || exit 1
done
lb n8sl1 1 --emulate-ranks 8 || exit 1
lb n8sl0 0 --emulate-ranks 8 || exit 1
for v in 1 0; do
  rm -rf gpurun_out/prof_lan$v
  TKHIP_LANCZOS_SL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lan$v -o run -- python3 bench.py --method TensorLanczos --no-cpu-baseline --no-end-to-end --steps 5 --warmup 1 > gpurun_out/prof_lan$v.log 2>&1 || { echo "prof $v failed"; tail -5 gpurun_out/prof_lan$v.log; exit 1; }
  f=$(find gpurun_out/prof_lan$v -name "*kernel_stats.csv" | head -1); grep -E "k_lan_1w|k_red_lan|k_fin_vy|k_basis_mul|k_gram" $f | cut -d, -f1-4
done
