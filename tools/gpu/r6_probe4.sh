# traffic probe: the two factor groups' launches taking turns on one stream (mode 5th column)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 200 tools/_build/d1probe 1048576 8 50 0 > gpurun_out/d1probe_seq.txt 2>&1 || { tail gpurun_out/d1probe_seq.txt; exit 1; }
cat gpurun_out/d1probe_seq.txt
