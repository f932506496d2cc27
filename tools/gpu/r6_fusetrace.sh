# block phases of a one-stream k_arn_d1 launch, plain and fused (trace build)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export TKHIP_LIB=tools/_build/libtkhip_trace.so TKHIP_FACTOR_GROUPS=1
timeout -k 10 150 python -u tools/d1_trace.py 8 8 40 > gpurun_out/ftrace_plain.txt 2>&1 || { tail gpurun_out/ftrace_plain.txt; exit 1; }
TKHIP_D1_FUSE=1 timeout -k 10 150 python -u tools/d1_trace.py 8 8 40 > gpurun_out/ftrace_fused.txt 2>&1 || { tail gpurun_out/ftrace_fused.txt; exit 1; }
unset TKHIP_FACTOR_GROUPS
timeout -k 10 150 python -u tools/d1_trace.py 8 8 40 > gpurun_out/ftrace_groups.txt 2>&1 || { tail gpurun_out/ftrace_groups.txt; exit 1; }
grep -v "active blocks\|xcc [0-9]" gpurun_out/ftrace_plain.txt gpurun_out/ftrace_fused.txt gpurun_out/ftrace_groups.txt
