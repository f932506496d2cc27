# GPU tests, then chained vs unchained one-sweep steps at N=1 and emulated N=8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_gpu.log | head -20; exit 1; }
for N in 1 8; do for C in 1 0; do
  TKHIP_D1_CHAIN=$C timeout -k 10 200 python bench.py --emulate-ranks $N --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/chain_${N}_$C.log 2>&1 || { echo "N=$N C=$C failed"; tail -5 gpurun_out/chain_${N}_$C.log; exit 1; }
  tail -1 gpurun_out/chain_${N}_$C.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$N chain=$C', d['value'], d['roofline']['avg_launch_us'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done; done
