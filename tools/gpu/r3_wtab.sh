# A/B: write-through (sc1) step outputs (tree library, TK_WT=1) vs plain stores (TK_WT=0)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
: > gpurun_out/wtab.log
run() {  # name, lib, args...
  local name=$1 lib=$2; shift 2
  TKHIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end "$@" > gpurun_out/wtab_one.log 2>&1 || { echo "$name failed"; tail -3 gpurun_out/wtab_one.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/wtab_one.log').read().strip().split('\n')[-1]); print('$name', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})" >> gpurun_out/wtab.log
}
for rep in 1 2; do
  for v in wt1 wt0; do
    lib=$R/tensorkrylov.jl_amd/tkamd/libtkhip.so; [ $v = wt0 ] && lib=$R/tools/_build/libtkhip_wt0.so
    run "$v C2" $lib --steps 3 || exit 1
    run "$v C1" $lib --config C1 --steps 4 || exit 1
    run "$v C4" $lib --config C4 --steps 4 || exit 1
    run "$v Lan" $lib --method TensorLanczos --steps 3 || exit 1
    run "$v emu8r0" $lib --steps 6 --emulate-ranks 8 || exit 1
  done
done
cat gpurun_out/wtab.log
