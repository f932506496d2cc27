# C3 kernel stats only (rocprofv3 --kernel-trace --stats of a short C3 bench)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -o run -- python3 $R/bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/prof_c3.log 2>&1 || { echo "rocprof failed"; exit 1; }
find $R/gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $R/gpurun_out/c3_kernel_stats.csv
