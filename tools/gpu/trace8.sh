set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace8 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --emulate-ranks 8 > $R/gpurun_out/trace8.log 2>&1
echo "EXIT $?"; ls $R/gpurun_out/trace8
