# k_arn_d1 with the 16 low columns of the 48-column tier in LDS (TK_D1_LC): GPU suite, then A/B
# against TK_D1_LC=0 (C2 N=1 and emulated N=8 bench, two repetitions; rocprofv3 per-instance times)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_lc.log 2>&1
rc=$?; tail -3 gpurun_out/t_lc.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for v in lc0 lc16; do for mode in n1 e8; do
  if [ $mode = n1 ]; then EXTRA=""; else EXTRA="--emulate-ranks 8 --emulate-rank 5"; fi
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-end-to-end $EXTRA > gpurun_out/lc_${v}_$mode.log 2>&1 || { echo "bench $v $mode failed"; tail -5 gpurun_out/lc_${v}_$mode.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/lc_${v}_$mode.log').read().strip().split('\n')[-1]); print('rep$rep $v $mode', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels']['sweep_spmv2_dcgs2']['avg_us'])"
done; done; done
cd /tmp && export TMPDIR=/tmp
for v in lc0 lc16; do
  rm -rf $R/gpurun_out/lcprof_$v
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lcprof_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/lcprof_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
  grep -h "k_arn_d1<48\|k_arn_d1<40\|k_arn_d1<56" $R/gpurun_out/lcprof_$v/run_kernel_stats.csv | cut -d, -f1-4
done
