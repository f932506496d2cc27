# block timeline of k_arn_d1 with all 8 C2 factors in the launch (N=1): per-XCD spans of factor 0
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TKHIP_LIB=$R/tools/_build/libtkhip_trace.so timeout -k 10 300 python tools/d1_trace.py 8 20 36 48 > gpurun_out/d1_trace_nf8.txt 2>&1 || { tail -5 gpurun_out/d1_trace_nf8.txt; exit 1; }
grep -v "active blocks" gpurun_out/d1_trace_nf8.txt | head -60
