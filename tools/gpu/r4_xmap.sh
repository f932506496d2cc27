# round 4 A/B: k_arn_d1's window -> XCD mapping (contiguous per XCD, the product; interleaved,
# tools/_build/libtkhip_xmap1.so) at C2 N=1 and the emulated one-factor rank (N=8), two reps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do for v in tree xmap1; do for N in 1 8; do
  L=""; [ "$v" != tree ] && L="TKHIP_LIB=$R/tools/_build/libtkhip_$v.so"
  env $L timeout -k 10 200 python bench.py --emulate-ranks $N --steps 6 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/xm_${v}_$N.log 2>&1 || { echo "$v $N failed"; tail -3 gpurun_out/xm_${v}_$N.log; exit 1; }
  tail -1 gpurun_out/xm_${v}_$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep $rep $v N=$N', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done; done; done
