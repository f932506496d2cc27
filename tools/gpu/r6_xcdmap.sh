# does k_arn_d1's slot -> XCD assumption (block x on XCD x % 8) hold with two concurrent
# factor-group launches?  (trace build: tools/build_variant.sh trace - -DTK_D1_TRACE=1)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export TKHIP_LIB=tools/_build/libtkhip_trace.so
timeout -k 10 150 python -u tools/d1_trace.py 8 8 40 > gpurun_out/xcdmap_groups.txt 2>&1 || { tail gpurun_out/xcdmap_groups.txt; exit 1; }
TKHIP_FACTOR_GROUPS=1 timeout -k 10 150 python -u tools/d1_trace.py 8 8 40 > gpurun_out/xcdmap_onestream.txt 2>&1 || { tail gpurun_out/xcdmap_onestream.txt; exit 1; }
grep -v "active blocks" gpurun_out/xcdmap_groups.txt gpurun_out/xcdmap_onestream.txt
