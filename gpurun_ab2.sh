set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
echo "== C2 emulated rank of 8"; BARGS="--emulate-ranks 8" bash gpurun_ab_env.sh base: nocomm:TK_EMULATE_NOCOMM=1 || exit 1
for v in base nocomm; do grep -o '"host_issue_us_per_iteration": [0-9.]*' gpurun_out/abe_$v.log; done
echo "== C2"; BARGS="" bash gpurun_ab_env.sh c2: ; grep -o '"host_issue_us_per_iteration": [0-9.]*' gpurun_out/abe_c2.log
