# Gram on the compute stream vs the side stream: parity, then emulated N=8 ranks 0 and 5 (two repetitions)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_solution.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gram2.log 2>&1
rc=$?; tail -3 gpurun_out/t_gram2.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for cfg in "0 main" "0 side" "5 main"; do set -- $cfg
  TKHIP_GRAM_STREAM=$2 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end --emulate-ranks 8 --emulate-rank $1 > gpurun_out/rk8_$1_$2.log 2>&1 || { echo "rank $1 failed"; tail -5 gpurun_out/rk8_$1_$2.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/rk8_$1_$2.log').read().strip().split('\n')[-1]); print('rep$rep rank $1 $2', d['value'], d['ms_per_step'], d['orthogonality_gram']['avg_us'])"
done; done
