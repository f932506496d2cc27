# round-3 final evidence at HEAD: GPU suite, smoke, C1-C4 bench lines, C2 kernel stats (factor
# groups on, and one stream for comparison), PMC traffic + MFMA counters, emulated scaling,
# per-rank N=8 rates, the three methods at C2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu/r3_tests.sh || exit 1
bash tools/gpu/r3_evidence1.sh || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_c2_1s
TKHIP_FACTOR_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2_1s -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/prof_c2_1s.log 2>&1 || { echo "rocprof 1s failed"; exit 1; }
cd $R
bash tools/gpu/r3_evidence2.sh || exit 1
