# A/B of variant libraries on one method: args METHOD NAMES...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
m=$1; shift
for v in "$@"; do
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end --method $m > gpurun_out/abm_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/abm_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abm_$v.log').read().strip().split('\n')[-1]); print('$v $m', d['value'], d['roofline']['achieved'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
