# kernel durations and launch gaps of the emulated 8-rank step, with and without the exchange
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
for v in comm nocomm; do
  rm -rf $R/gpurun_out/emu_$v
  E=0; [ $v = nocomm ] && E=1
  TK_EMULATE_NOCOMM=$E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/emu_$v -o run -- python3 $R/bench.py --emulate-ranks 8 --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/emu_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  echo "== $v"; python3 $R/tools/trace_gaps.py $R/gpurun_out/emu_$v/run_kernel_trace.csv
done
