# A/B of variant libraries (tools/_build/libtkhip_NAME.so): C2 at N=1 and the emulated N=8
# rank (no exchange), device rate only
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for v in "$@"; do
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/ab1_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab1_$v.log; exit 1; }
  TK_EMULATE_NOCOMM=1 TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end --emulate-ranks 8 > gpurun_out/ab8_$v.log 2>&1 || { echo "variant $v n8 failed"; tail -5 gpurun_out/ab8_$v.log; exit 1; }
done
for v in "$@"; do for N in 1 8; do python3 -c "
import json; d=json.loads(open('gpurun_out/ab${N}_$v.log').read().strip().split('\n')[-1]); print('$v N=$N', d['value'], d['roofline']['achieved'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"; done; done
