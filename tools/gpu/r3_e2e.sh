set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TKHIP_SOLVER_STATS=1 timeout -k 10 300 python tools/e2e_diag.py > gpurun_out/e2e_diag.log 2>&1; rc=$?; cat gpurun_out/e2e_diag.log; exit $rc
