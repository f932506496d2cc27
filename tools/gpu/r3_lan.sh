# TensorLanczos one-sweep at full occupancy: Lanczos/gram parity, then C2 Lanczos N=1 and emulated N=8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_parity.py tests/test_gpu_solution.py tests/test_gpu_configs.py tests/test_gpu_boundary.py -k "anczos or gram or Gram or solution or boundary or exchange or julia or RandSparse or shared or C3" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_lan.log 2>&1
rc=$?; tail -2 gpurun_out/t_lan.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --method TensorLanczos --steps 3 --no-cpu-baseline --no-end-to-end > gpurun_out/lan_n1.log 2>&1 || { tail -5 gpurun_out/lan_n1.log; exit 1; }
timeout -k 10 300 python bench.py --method TensorLanczos --steps 6 --no-cpu-baseline --no-end-to-end --emulate-ranks 8 --emulate-rank 0 > gpurun_out/lan_rk8_0.log 2>&1 || { tail -5 gpurun_out/lan_rk8_0.log; exit 1; }
for f in lan_n1 lan_rk8_0; do python3 -c "
import json; d=json.loads(open('gpurun_out/$f.log').read().strip().split('\n')[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"; done
timeout -k 10 300 python bench.py --config C3 --steps 3 --no-cpu-baseline --no-end-to-end > gpurun_out/c3_n1.log 2>&1 || { tail -5 gpurun_out/c3_n1.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/c3_n1.log').read().strip().split('\n')[-1]); print('c3_n1', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
