# GPU tests, then the C2 bench at N=1 and the emulated N=8 rank (args: extra env assignments per run, e.g. "X=1" "X=0")
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_gpu.log | head -20; exit 1; }
[ $# -eq 0 ] && set -- "NONE=1"
for N in 1 8; do for E in "$@"; do
  env $E timeout -k 10 200 python bench.py --emulate-ranks $N --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/emu_${N}.log 2>&1 || { echo "N=$N $E failed"; tail -5 gpurun_out/emu_${N}.log; exit 1; }
  tail -1 gpurun_out/emu_${N}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$N $E', d['value'], d['roofline']['avg_launch_us'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done; done
