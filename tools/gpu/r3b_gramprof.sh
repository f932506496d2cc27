# k_gram vs its two reduce launches (rocprofv3 kernel stats of tools/gram_bench.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in gram_old tree; do
  if [ $v = tree ]; then L=$R/tensorkrylov.jl_amd/tkamd/libtkhip.so; else L=$R/tools/_build/libtkhip_$v.so; fi
  TKHIP_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gprof_$v -o run -- python3 $R/tools/gram_bench.py > $R/gpurun_out/gprof_$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/gprof_$v.log; exit 1; }
  grep -h gram $R/gpurun_out/gprof_$v.log
  find $R/gpurun_out/gprof_$v -name '*kernel_stats.csv' -exec grep -h gram {} \;
done
