# k_arn_d1's memory-traffic ceiling at C2 (tools/d1probe.hip), then the EARLY A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 tools/_build/d1probe > gpurun_out/d1probe_c2.txt 2>&1 || { tail gpurun_out/d1probe_c2.txt; exit 1; }
cat gpurun_out/d1probe_c2.txt
CASES="${CASES:-C2:1 C4:8:7 C4:8:0 C1:1 C2:8}" bash tools/gpu/r6_ab.sh "$@"
