# C3 SpMV gather-pattern ceiling (tools/gatherprobe.hip over C3's exact SELL index stream)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python tools/c3_sell_dump.py /tmp/c3sell.bin > gpurun_out/c3probe.log 2>&1 || { echo dump failed; cat gpurun_out/c3probe.log; exit 1; }
timeout -k 10 120 tools/_build/gatherprobe /tmp/c3sell.bin >> gpurun_out/c3probe.log 2>&1 || { echo probe failed; cat gpurun_out/c3probe.log; exit 1; }
cat gpurun_out/c3probe.log
timeout -k 10 300 python bench.py --config C3 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_C3.log 2>&1 || { echo "bench C3 failed"; tail -5 gpurun_out/bench_C3.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_C3.log').read().strip().split('\n')[-1]); print('C3', d['value'], d['roofline'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
