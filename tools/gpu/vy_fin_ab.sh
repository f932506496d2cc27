# k_fin_vy / k_basis_mul durations (rocprofv3 stats) per variant library, C2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
for v in "$@"; do
  rm -rf $R/gpurun_out/vyf_$v
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/vyf_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/vyf_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/vyf_$v/run_kernel_stats.csv')):
    if 'basis_mul' in r['Name'] or 'fin_vy' in r['Name']: print('$v', r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3)"
done
