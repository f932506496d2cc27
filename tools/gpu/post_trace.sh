# k_post / k_reduce256 durations at one factor per GPU (emulated N=8), with and without the exchange
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
for M in comm nocomm; do
  E=""; [ $M = nocomm ] && E="TK_EMULATE_NOCOMM=1"
  rm -rf $R/gpurun_out/pt_$M
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pt_$M -o run -- python3 $R/bench.py --emulate-ranks 8 --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/pt_$M.log 2>&1 || { echo "$M failed"; exit 1; }
  echo "== $M"; python3 $R/tools/trace_gaps.py $R/gpurun_out/pt_$M/run_kernel_trace.csv 100
done
