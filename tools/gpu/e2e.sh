set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python tools/e2e_profile.py C2 1 > gpurun_out/e2e_C2.log 2>&1; echo "EXIT $?"
head -60 gpurun_out/e2e_C2.log
