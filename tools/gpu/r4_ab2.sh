# round 4: GPU suite, e2e traces (tail threads A/B), XCD mapping A/B, C3 evidence (probes, PMC)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu/r3_tests.sh || exit 1
bash tools/gpu/r4_e2e.sh || exit 1
bash tools/gpu/r4_xmap.sh || exit 1
bash tools/gpu/r4_c3.sh
