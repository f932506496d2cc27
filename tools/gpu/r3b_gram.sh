# round 3 (second session): k_gram column groups + VALU tail -- parity, A/B against HEAD, rank 0 / 5 at emulated N=8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_gram.log 2>&1
rc=$?; tail -12 gpurun_out/t_gram.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for v in gram_old tree; do
  if [ $v = tree ]; then L=$R/tensorkrylov.jl_amd/tkamd/libtkhip.so; else L=$R/tools/_build/libtkhip_$v.so; fi
  TKHIP_LIB=$L timeout -k 10 120 python tools/gram_bench.py >> gpurun_out/gramab2.log 2>&1 || { echo "variant $v failed"; tail -3 gpurun_out/gramab2.log; exit 1; }
done; done
cat gpurun_out/gramab2.log
for r in 0 5; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end --emulate-ranks 8 --emulate-rank $r > gpurun_out/rk8_$r.log 2>&1 || { echo "rank $r failed"; tail -5 gpurun_out/rk8_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/rk8_$r.log').read().strip().split('\n')[-1]); print('rank $r', d['value'], d['ms_per_step'], d['orthogonality_gram']['avg_us'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done
