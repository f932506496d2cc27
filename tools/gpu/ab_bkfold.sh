set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
for v in fold nofold; do
  rm -rf $R/gpurun_out/abm_$v
  F=1; [ $v = nofold ] && F=0
  TKHIP_BK_FOLD=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abm_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/abm_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
done
cd $R; for v in fold nofold; do echo "== $v"; python3 tools/kstats_d1.py gpurun_out/abm_$v/run_kernel_stats.csv | sort -k2; done
