# round 4: per-iteration host evaluation on the box's CPU, AVX2 vs AVX-512 (GEMM + LU solve)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in a b c; do
  for v in 0 1; do
    TKHIP_HOST_AVX512=$v timeout -k 10 300 python tools/host_eval_real.py C4 > gpurun_out/he2_$v$rep.log 2>&1 || { echo "host eval failed"; tail -3 gpurun_out/he2_$v$rep.log; exit 1; }
    echo "avx512=$v $(tail -1 gpurun_out/he2_$v$rep.log)"
  done
done
