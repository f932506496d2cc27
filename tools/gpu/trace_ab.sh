# per-launch k_arn_d1 durations of one C2 sweep for variant libraries (step order)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
for v in "$@"; do
  rm -rf $R/gpurun_out/tr_$v
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_$v -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/tr_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  python3 - $R/gpurun_out/tr_$v/run_kernel_trace.csv $v <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000 for r in rows if 'k_arn_d1' in r['Kernel_Name']]
print(sys.argv[2], ' '.join('%.0f' % x for x in d[:50]))
PY
done
