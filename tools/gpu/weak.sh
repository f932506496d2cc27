# the weaker paths: C2 TensorLanczos / LanczosReorth, C1, C3, C4 bench lines + Lanczos kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline "$@"; }
run --method TensorLanczos > gpurun_out/w_lan.log 2>&1 || { tail -5 gpurun_out/w_lan.log; exit 1; }
run --method TensorLanczosReorth > gpurun_out/w_reo.log 2>&1 || { tail -5 gpurun_out/w_reo.log; exit 1; }
for C in C1 C3 C4; do run --config $C > gpurun_out/w_$C.log 2>&1 || { tail -5 gpurun_out/w_$C.log; exit 1; }; done
for f in lan reo C1 C3 C4; do python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/w_$f.log') if l.startswith('{\"metric')][-1]); e=d.get('end_to_end') or {}
print('$f', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()}, 'e2e', e.get('iterations_s'))"; done
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_lan
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lan -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end --method TensorLanczos > $R/gpurun_out/prof_lan.log 2>&1 || exit 1
python3 -c "
import csv
for x in csv.DictReader(open('$R/gpurun_out/prof_lan/run_kernel_stats.csv')): print(x['Name'][:50], x['Calls'], round(float(x['AverageNs'])/1e3,1), round(float(x['TotalDurationNs'])/1e6,3))" | head -20
