set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for nc in 40 12 6; do timeout -k 10 120 ./tools/_build/bwprobe $nc > gpurun_out/probe$nc.log 2>&1 || exit 1; done
cat gpurun_out/probe40.log gpurun_out/probe12.log gpurun_out/probe6.log
