# round-6 evidence, part A: the GPU suite, smoke, bench lines (C2 + CPU baselines, C1, C3, C4),
# rocprofv3 kernel trace + stats of C2 (trace_span.py / kstats_d1.py), PMC FETCH/WRITE -> pmc_C2_n1.json
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu/r5_round.sh || exit 1
cp gpurun_out/t_gpu.log gpurun_out/gpu_tests.log
bash tools/gpu/full.sh || exit 1
cd $R
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write C2 1 50 gpurun_out/pmc_C2_n1.json
T=$(find gpurun_out/prof_c2 -name "*kernel_trace.csv" | head -1); S=$(find gpurun_out/prof_c2 -name "*kernel_stats.csv" | head -1)
python3 tools/trace_span.py $T > gpurun_out/c2_trace_span.txt && python3 tools/kstats_d1.py $S > gpurun_out/c2_kstats_d1.txt
cat gpurun_out/c2_trace_span.txt
