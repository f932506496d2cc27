# round 4: k_reduce256 hand-off in the memory-model form (release/acquire add + acquire fence,
# tools/_build/libtkhip_redmm.so, -DTK_RED_MM=1) vs the measured-correct relaxed form (default):
# parity tests of the one-sweep Arnoldi through the variant, then C2 N=1 / emulated N=8 / C1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TKHIP_LIB=$R/tools/_build/libtkhip_redmm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "arnoldi or c2 or c1" > gpurun_out/t_redmm.log 2>&1
rc=$?; tail -2 gpurun_out/t_redmm.log; [ $rc -eq 0 ] || exit 1
ab() {  # name, lib, bench args
  local nm=$1 lib=$2; shift 2
  TKHIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --steps 10 --warmup 2 "$@" > gpurun_out/mm_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/mm_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/mm_$nm.log').read().strip().splitlines()[-1])
print('== $nm', d['value'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
}
D=$R/tensorkrylov.jl_amd/tkamd/libtkhip.so; M=$R/tools/_build/libtkhip_redmm.so
for rep in a b; do
  ab c2_def$rep $D || exit 1
  ab c2_mm$rep $M || exit 1
  ab n8_def$rep $D --emulate-ranks 8 || exit 1
  ab n8_mm$rep $M --emulate-ranks 8 || exit 1
  ab c1_def$rep $D --config C1 || exit 1
  ab c1_mm$rep $M --config C1 || exit 1
done
bash tools/gpu/r4_grpN.sh
