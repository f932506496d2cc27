# A/B over environment settings: each arg is "NAME:VAR=VAL,VAR=VAL" ; bench args via BARGS
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  ( IFS=","; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; IFS=" "
    timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline $BARGS > gpurun_out/abe_$name.log 2>&1 ) || { echo "variant $name failed"; tail -5 gpurun_out/abe_$name.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abe_$name.log').read().strip().split('\n')[-1]); print('$name', d['value'], d['roofline']['achieved'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
