# Gram on its own stream: gram tests, then N=1 and emulated N=8 rank 0 / rank 1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_solution.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_g.log 2>&1
rc=$?; tail -2 gpurun_out/t_g.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end > gpurun_out/g_n1.log 2>&1 || { tail -5 gpurun_out/g_n1.log; exit 1; }
for r in 0 1; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end --emulate-ranks 8 --emulate-rank $r > gpurun_out/g_rk8_$r.log 2>&1 || { tail -5 gpurun_out/g_rk8_$r.log; exit 1; }
done
for f in g_n1 g_rk8_0 g_rk8_1; do python3 -c "
import json; d=json.loads(open('gpurun_out/$f.log').read().strip().split('\n')[-1]); print('$f', d['value'], d['ms_per_step'], d['orthogonality_gram'].get('avg_us'), {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"; done
