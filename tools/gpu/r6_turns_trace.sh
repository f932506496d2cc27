# block timelines of factor 0's k_arn_d1 launch: factor groups taking turns vs two streams
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export TKHIP_LIB=tools/_build/libtkhip_trace.so
timeout -k 10 150 python -u tools/d1_trace.py 8 8 40 > gpurun_out/tt_turns.txt 2>&1 || { tail gpurun_out/tt_turns.txt; exit 1; }
TKHIP_D1_TURNS=0 timeout -k 10 150 python -u tools/d1_trace.py 8 8 40 > gpurun_out/tt_streams.txt 2>&1 || { tail gpurun_out/tt_streams.txt; exit 1; }
grep -v "xcc [0-9]" gpurun_out/tt_turns.txt gpurun_out/tt_streams.txt | cut -c1-900
