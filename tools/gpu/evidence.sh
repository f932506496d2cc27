# round evidence: GPU tests + full.sh (smoke, default bench, C1/C3/C4, rocprof stats, PMC),
# then the emulated strong-scaling curve (scale.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu/round.sh && bash tools/gpu/scale.sh
