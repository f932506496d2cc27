# per-kernel rocprof stats for variant libraries (args: names)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  rm -rf $R/gpurun_out/abprof_$v
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abprof_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/abprof_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
done
cd $R; for v in "$@"; do echo "== $v"; python3 tools/kstats_bw.py gpurun_out/abprof_$v/run_kernel_stats.csv | sort -k2 | head -20; done
