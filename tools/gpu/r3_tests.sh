# round 3: GPU suite (thread timeouts name a hung test), then emulated N=8 and N=1 benches
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_gpu.log 2>&1
rc=$?; echo "pytest EXIT $rc" >> gpurun_out/t_gpu.log
grep -E "PASSED|FAILED|ERROR" gpurun_out/t_gpu.log | tail -15
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || exit 1
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --emulate-ranks 8 --no-cpu-baseline > gpurun_out/b_emu8.log 2>&1 || { echo "emu8 failed"; tail -5 gpurun_out/b_emu8.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_n1.log 2>&1 || { echo "n1 failed"; tail -5 gpurun_out/b_n1.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/b_emu8.log", "gpurun_out/b_n1.log"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["roofline"]["frac"], (d.get("end_to_end") or {}).get("iterations_s"))
PY
