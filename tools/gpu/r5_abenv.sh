# A/B of environment variants on the in-tree library (no tests): each SPEC is NAME:VAR=VAL[,VAR=VAL...]
# (NAME:- for none); runs CFGS (default "C2:1 C2:8") -- CONFIG:EMULATED_RANKS[:RANK] -- interleaved, REPS repetitions
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CFGS=${CFGS:-"C2:1 C2:8"}; REPS=${REPS:-"a b"}
for rep in $REPS; do for cf in $CFGS; do for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "-" ] && envs=""
  IFS=: read cfg N RK <<< "$cf"; RK=${RK:-0}
  env ${envs//,/ } timeout -k 10 200 python bench.py --config $cfg --emulate-ranks $N --emulate-rank $RK --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end $BARGS > gpurun_out/abe_${name}_${cfg}_${N}_${RK}_$rep.log 2>&1 || { echo "$name $cf failed"; tail -3 gpurun_out/abe_${name}_${cfg}_${N}_${RK}_$rep.log; exit 1; }
  tail -1 gpurun_out/abe_${name}_${cfg}_${N}_${RK}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep $cf $name', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done; done; done
