# A/B of variant libraries (tools/_build/libtkhip_NAME.so) on one box, interleaved:
# C2 N=1, emulated N=8 with and without the exchange, C1 (device rates)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
run() {  # name tag extra-env... -- bench args
  local v=$1 tag=$2; shift 2
  env TKHIP_LIB=$R/tools/_build/libtkhip_$v.so "$@" > gpurun_out/ab4_${v}_$tag.log 2>&1 || { echo "variant $v $tag failed"; tail -5 gpurun_out/ab4_${v}_$tag.log; exit 1; }
}
for rep in 1 2; do for v in "$@"; do
  run $v n1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end
  run $v n8 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end --emulate-ranks 8
  run $v n8nc TK_EMULATE_NOCOMM=1 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end --emulate-ranks 8
  run $v c1 timeout -k 10 300 python bench.py --config C1 --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end
  for t in n1 n8 n8nc c1; do python3 -c "
import json; d=json.loads(open('gpurun_out/ab4_${v}_$t.log').read().strip().split('\n')[-1]); print('rep$rep $v $t', d['value'])"; done
done; done
