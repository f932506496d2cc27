# C2 bench with the fused flush + V*Y (default) and with separate launches, kernel stats of each
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for V in fused sep; do
  if [ $V = sep ]; then export TKHIP_NO_FUSED_FLUSH=1; else unset TKHIP_NO_FUSED_FLUSH; fi
  rm -rf $R/gpurun_out/vy_$V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/vy_$V -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/vy_$V.log 2>&1 || { echo "$V failed"; tail -5 $R/gpurun_out/vy_$V.log; exit 1; }
  echo "== $V"; grep -E "fin_vy|basis_mul|fin_d" $R/gpurun_out/vy_$V/run_kernel_stats.csv | cut -d, -f1-4
  python3 -c "import json; d=json.loads([l for l in open('$R/gpurun_out/vy_$V.log') if l.startswith('{"metric')][-1]); print(d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
