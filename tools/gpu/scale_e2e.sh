# host-only evaluation timing on the box's CPU, then the emulated scaling (scale.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
python tools/host_eval_bench.py > gpurun_out/host_eval.log 2>&1; cat gpurun_out/host_eval.log
lscpu | grep -E "Model name|^CPU\(s\)|Thread|MHz" ; nproc
bash tools/gpu/scale.sh
