# per-kernel durations and launch gaps of the emulated N-rank step (one factor per GPU at N=8;
# CFG=C4 RK=7 for another config / rank)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for N in ${@:-8}; do
  timeout -k 10 200 python bench.py --config ${CFG:-C2} --emulate-rank ${RK:-0} --emulate-ranks $N --steps 5 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/emu$N.log 2>&1 || { echo "emu $N failed"; tail -5 gpurun_out/emu$N.log; exit 1; }
  tail -1 gpurun_out/emu$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$N', d['value'], d['roofline']['avg_launch_us'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
cd /tmp && export TMPDIR=/tmp
export TKHIP_RED_MM=0   # (no self-check job in the trace)
for N in ${@:-8}; do
  rm -rf $R/gpurun_out/emu_tr$N
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/emu_tr$N -o run -- python3 $R/bench.py --config ${CFG:-C2} --emulate-rank ${RK:-0} --emulate-ranks $N --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/emu_tr$N.log 2>&1 || { echo "trace $N failed"; exit 1; }
  python3 $R/tools/trace_gaps.py $R/gpurun_out/emu_tr$N/run_kernel_trace.csv
done
