# k_basis_mul durations (rocprofv3 stats) for the in-tree library and variant libraries (args), C2 and C4
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
for v in tree "$@"; do for C in C2 C4; do
  L=""; [ "$v" != tree ] && L="TKHIP_LIB=$R/tools/_build/libtkhip_$v.so"
  rm -rf $R/gpurun_out/vy_${v}_$C
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/vy_${v}_$C -o run -- python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/vy_${v}_$C.log 2>&1 || { echo "$v $C failed"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/vy_${v}_$C/run_kernel_stats.csv')):
    if 'basis_mul' in r['Name']: print('$v $C', r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3)"
done; done
