# the store-side variants of k_arn_d1's traffic probe, then a kernel trace of the default bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 240 tools/_build/d1probe 1048576 8 50 0 1 2 4 8 6 14 > gpurun_out/d1probe_var.txt 2>&1 || { tail gpurun_out/d1probe_var.txt; exit 1; }
cat gpurun_out/d1probe_var.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o c2 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/prof_c2_bench.json 2> gpurun_out/prof_c2.err || { tail -5 gpurun_out/prof_c2.err; exit 1; }
tail -1 gpurun_out/prof_c2_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
T=$(find gpurun_out/prof_c2 -name "*kernel_trace.csv" | head -1); S=$(find gpurun_out/prof_c2 -name "*kernel_stats.csv" | head -1)
python3 tools/trace_span.py $T && python3 tools/kstats_d1.py $S
