# round 3: new tests first (gram, solution, boundary), then the whole GPU suite, then benches
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_solution.py tests/test_gpu_boundary.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_new.log 2>&1
rc=$?; echo "pytest-new EXIT $rc" >> gpurun_out/t_new.log
grep -E "PASSED|FAILED|ERROR" gpurun_out/t_new.log | tail -30; tail -3 gpurun_out/t_new.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1
rc=$?; echo "pytest EXIT $rc" >> gpurun_out/t_gpu.log
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || exit 1
for m in TensorArnoldi TensorLanczos; do for g in rows deferred; do
  TKHIP_GRAM=$g timeout -k 10 300 python bench.py --method $m --no-cpu-baseline --no-end-to-end > gpurun_out/b_${m}_${g}.log 2>&1 || { echo "bench $m $g failed"; tail -5 gpurun_out/b_${m}_${g}.log; exit 1; }
  TKHIP_GRAM=$g timeout -k 10 300 python bench.py --method $m --emulate-ranks 8 --no-cpu-baseline --no-end-to-end > gpurun_out/b8_${m}_${g}.log 2>&1 || { echo "bench8 $m $g failed"; tail -5 gpurun_out/b8_${m}_${g}.log; exit 1; }
done; done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/b*_Tensor*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["roofline"]["frac"], d["roofline"]["avg_launch_us"], d["orthogonality_gram"], d["basis_mul_step"]["avg_us"])
PY
