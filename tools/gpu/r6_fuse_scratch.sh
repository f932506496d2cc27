# fused one-sweep launches without scratch memory (tree) vs HEAD (head): fused tests, then A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_groups.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
CASES="C4:8:0 C1:1" bash tools/gpu/r6_ab.sh head || exit 1
TKHIP_D1_FUSE=1 CASES="C2:1 C2:8:1 C4:8:7 C1:1 C4:1" bash tools/gpu/r6_ab.sh head
