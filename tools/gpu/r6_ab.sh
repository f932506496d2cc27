# A/B without tests (round 6): configs x variants, interleaved, REPS repetitions.
# args: variant names (tools/_build/libtkhip_NAME.so; "tree" = the in-tree library is always first)
# CASES: "CFG:EMU[:RANK]" items, e.g. "C2:1 C2:8 C4:8:7 C1:1"; EMU 1 = the plain N = 1 run
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CASES=${CASES:-"C2:1"}; REPS=${REPS:-"a b"}; STEPS=${STEPS:-8}
for rep in $REPS; do for cs in $CASES; do
  IFS=: read CFG N RK <<< "$cs"; RK=${RK:-0}
  EM=""; [ "$N" != 1 ] && EM="--emulate-ranks $N --emulate-rank $RK"
  for v in tree "$@"; do
    # (a variant "VAR=VAL" runs the in-tree library with that environment variable)
    # ("A=1,B=2": several)
    L=""; case "$v" in tree) ;; *=*) L="${v//,/ }" ;; *) L="TKHIP_LIB=$R/tools/_build/libtkhip_$v.so" ;; esac
    vn=${v//=/_}; vn=${vn//,/_}
    log=gpurun_out/ab_${vn}_${CFG}_${N}_${RK}_$rep.log
    env $L timeout -k 10 200 python bench.py --config $CFG $EM --steps $STEPS --warmup 2 --no-cpu-baseline --no-end-to-end $BARGS > $log 2>&1 || { echo "$v $cs failed"; tail -3 $log; exit 1; }
    tail -1 $log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep $cs %-6s' % '$v', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
  done
done; done
