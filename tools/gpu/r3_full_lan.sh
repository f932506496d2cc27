# full GPU suite, then TensorLanczos C2 N=1 and emulated N=8 rank 0
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu/r3_tests.sh || exit 1
timeout -k 10 300 python bench.py --method TensorLanczos --steps 3 --no-cpu-baseline > gpurun_out/lan_n1.log 2>&1 || { tail -5 gpurun_out/lan_n1.log; exit 1; }
timeout -k 10 300 python bench.py --method TensorLanczos --steps 6 --no-cpu-baseline --no-end-to-end --emulate-ranks 8 --emulate-rank 0 > gpurun_out/lan_rk8_0.log 2>&1 || { tail -5 gpurun_out/lan_rk8_0.log; exit 1; }
for f in lan_n1 lan_rk8_0; do python3 -c "
import json; d=json.loads(open('gpurun_out/$f.log').read().strip().split('\n')[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('end_to_end') or {}).get('iterations_s'), {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"; done
