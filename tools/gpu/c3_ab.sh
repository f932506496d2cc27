# C3 device rate A/B of variant libraries (interleaved, 2 reps) + per-kernel stats of the last
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do for v in "$@"; do
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 python bench.py --config C3 --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/c3ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/c3ab_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c3ab_$v.log').read().strip().split('\n')[-1]); print('rep$rep $v', d['value'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done; done
