# block timeline of k_arn_d1 at one factor per GPU (N=8 regime) and 4 factors (C1-like)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TKHIP_LIB=$R/tools/_build/libtkhip_trace.so timeout -k 10 300 python tools/d1_trace.py 1 6 20 36 48 > gpurun_out/d1_trace_nf1.txt 2>&1 || { tail -5 gpurun_out/d1_trace_nf1.txt; exit 1; }
grep -v "active blocks" gpurun_out/d1_trace_nf1.txt | head -60
