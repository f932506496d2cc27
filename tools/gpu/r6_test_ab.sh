# the GPU suite (or a subset: TESTS), then an A/B of the tree against variants ($@) on CASES
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/} -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error|assert" gpurun_out/t_gpu.log | head -30; exit 1; }
if [ $# -gt 0 ]; then CASES="${CASES:-C2:1 C4:8:7 C4:8:0 C1:1 C2:8}" bash tools/gpu/r6_ab.sh "$@"; fi
