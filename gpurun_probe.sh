set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 ./tools/_build/bwprobe 40 > gpurun_out/probe40.log 2>&1 && \
timeout -k 10 120 ./tools/_build/bwprobe 12 > gpurun_out/probe12.log 2>&1
echo "EXIT $?"; cat gpurun_out/probe40.log gpurun_out/probe12.log
