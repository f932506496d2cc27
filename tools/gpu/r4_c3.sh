# round 4: C3 evidence at HEAD -- shared-matrix parity tests, the bench line, kernel stats,
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) -> gpurun_out/pmc_C3_n1.json, and the
# gather-pattern probe with the 40-B entry layouts (split 32 + 8, packed 40) beside the 64-B one
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
python3 tools/c3_sell_dump.py /tmp/c3_sell.bin > gpurun_out/c3_dump.log 2>&1 || { echo "dump failed"; tail -3 gpurun_out/c3_dump.log; exit 1; }
timeout -k 10 120 tools/_build/gatherprobe /tmp/c3_sell.bin > gpurun_out/c3_gatherprobe.txt 2>&1 || { echo "probe failed"; cat gpurun_out/c3_gatherprobe.txt; exit 1; }
cat gpurun_out/c3_gatherprobe.txt
bash tools/gpu/r3_c3pmc.sh
timeout -k 10 120 tools/_build/syncprobe > gpurun_out/syncprobe.txt 2>&1 || { echo "syncprobe failed"; cat gpurun_out/syncprobe.txt; exit 1; }
cat gpurun_out/syncprobe.txt
