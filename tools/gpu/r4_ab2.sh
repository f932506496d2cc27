# round 4: XCD mapping A/B, C3 evidence (probes, PMC), e2e traces
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu/r4_xmap.sh || exit 1
bash tools/gpu/r4_c3.sh || exit 1
bash tools/gpu/r4_e2e.sh
