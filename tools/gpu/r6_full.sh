# round 6: the whole GPU suite, smoke, and the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/t_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print(d['value'],d['roofline']['frac'],d['roofline']['avg_launch_us'],d['end_to_end']['vs_device_steps_only'],d['cpu_baseline']['value'])"
