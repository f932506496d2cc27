# per-instance rocprof stats of the one-sweep Arnoldi kernel for variant libraries
# (args: names built by tools/build_variant.sh), then SQ counters of the first variant
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
for v in "$@"; do
  rm -rf $R/gpurun_out/abprof_$v
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abprof_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/abprof_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
done
cd $R; for v in "$@"; do echo "== $v"; python3 tools/kstats_d1.py gpurun_out/abprof_$v/run_kernel_stats.csv | sort -k2; done
if [ -n "$PMC" ]; then
  cd /tmp
  timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1
  rm -rf $R/gpurun_out/pmc_sq
  TKHIP_LIB=$R/tools/_build/libtkhip_$1.so timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_sq.log 2>&1
  echo "pmc EXIT $?"
fi
