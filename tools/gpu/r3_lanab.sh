# A/B of k_lan_1w rows per thread (TK_LAN_RPT): C2 TensorLanczos N=1 and emulated N=8 rank 0
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
: > gpurun_out/lanab.log
for rep in 1 2; do for v in rpt2 rpt4 rpt8; do
  for e in 0 8; do
    TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 200 python bench.py --method TensorLanczos --steps 3 --no-cpu-baseline --no-end-to-end --emulate-ranks $e > gpurun_out/lanab_one.log 2>&1 || { echo "variant $v failed"; tail -3 gpurun_out/lanab_one.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/lanab_one.log').read().strip().split('\n')[-1]); print('$v emu$e', d['value'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})" >> gpurun_out/lanab.log
  done
done; done
cat gpurun_out/lanab.log
