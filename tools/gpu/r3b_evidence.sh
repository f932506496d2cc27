# round-3 evidence at HEAD (second session): GPU suite, smoke, C1-C4 bench lines, kernel stats,
# PMC traffic + MFMA counters, emulated scaling, per-rank N=8, the three methods, N=1 block trace
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu/r3_tests.sh || exit 1
bash tools/gpu/r3_evidence1.sh || exit 1
bash tools/gpu/r3_evidence2.sh || exit 1
bash tools/gpu/r3b_trace8.sh || exit 1
