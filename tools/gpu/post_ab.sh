# GPU tests, then k_post duration at one factor (emulated N=8, exchange path) for the in-tree and variant libraries
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_gpu.log | head -20; exit 1; }
cd /tmp && export TMPDIR=/tmp
for v in tree "$@"; do
  L=""; [ "$v" != tree ] && L="TKHIP_LIB=$R/tools/_build/libtkhip_$v.so"
  rm -rf $R/gpurun_out/pab_$v
  env $L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pab_$v -o run -- python3 $R/bench.py --emulate-ranks 8 --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/pab_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  echo "== $v"; python3 $R/tools/trace_gaps.py $R/gpurun_out/pab_$v/run_kernel_trace.csv 100 | grep -E "k_post|k_reduce256"
done
