# GPU tests, per-instance k_arn_d1 stats (in-tree + variants), then C2 N=1 / emulated N=8 per library
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_gpu.log | head -20; exit 1; }
for v in tree "$@"; do for N in 1 8; do
  L=""; [ "$v" != tree ] && L="TKHIP_LIB=$R/tools/_build/libtkhip_$v.so"
  env $L timeout -k 10 200 python bench.py --emulate-ranks $N --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/d1ab_${v}_$N.log 2>&1 || { echo "$v $N failed"; tail -3 gpurun_out/d1ab_${v}_$N.log; exit 1; }
  tail -1 gpurun_out/d1ab_${v}_$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v N=$N', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done; done
