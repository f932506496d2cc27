# round-5 evidence, part A: the GPU suite, smoke, bench lines (C2 + CPU baselines, C1, C3, C4),
# rocprofv3 kernel stats of C2, PMC FETCH/WRITE -> pmc_C2_n1.json
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu/r5_round.sh || exit 1
cp gpurun_out/t_gpu.log gpurun_out/gpu_tests.log
bash tools/gpu/full.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write C2 1 50 gpurun_out/pmc_C2_n1.json
