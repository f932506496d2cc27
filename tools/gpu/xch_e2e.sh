# exchange-path GPU tests, then the emulated N=8/N=2 end-to-end loop with solver stats
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "exchange or pipelined or boundary or golden" > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
bash tools/gpu/e2e_stats.sh 2>&1 | grep -v "^{"
