# A/B of k_gram variants (tools/gram_bench.py, C2 factor size), two repetitions
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do for v in b512_gq8 b1024_gq8 b1024_gq4 b1024_gq16 b256_gq16; do
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 120 python tools/gram_bench.py >> gpurun_out/gramab.log 2>&1 || { echo "variant $v failed"; tail -3 gpurun_out/gramab.log; exit 1; }
done; done
cat gpurun_out/gramab.log
