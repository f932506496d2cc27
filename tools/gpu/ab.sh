# A/B: bench C2 with each variant library in tools/_build (args: variant names)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for v in "$@"; do
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
done
for v in "$@"; do python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().split('\n')[-1]); print('$v', d['value'], d['roofline']['achieved'], {k:v['avg_us'] for k,v in d['kernels'].items()})"; done
