set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu/r3b_trace8.sh && bash tools/gpu/r3b_gramprof.sh
