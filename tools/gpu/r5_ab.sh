# A/B without tests: C2 at N=1 and emulated N=8 (rank 0), in-tree library ("tree") and the
# variants tools/_build/libtkhip_NAME.so, interleaved, two repetitions (args: variant names;
# EMU="1 8" by default, CFG=C2)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
EMU=${EMU:-"1 8"}; CFG=${CFG:-C2}
for rep in a b; do for N in $EMU; do for v in tree "$@"; do
  L=""; [ "$v" != tree ] && L="TKHIP_LIB=$R/tools/_build/libtkhip_$v.so"
  env $L timeout -k 10 200 python bench.py --config $CFG --emulate-ranks $N --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end $BARGS > gpurun_out/ab_${v}_${N}_$rep.log 2>&1 || { echo "$v $N failed"; tail -3 gpurun_out/ab_${v}_${N}_$rep.log; exit 1; }
  tail -1 gpurun_out/ab_${v}_${N}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep $CFG N=$N $v', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done; done; done
