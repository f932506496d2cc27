# round 4: single-column Lanczos Gram (two rows per lane and load): the layout / Gram / groups
# GPU tests, then kernel stats of C2 TensorLanczos and the bench line
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_groups.py tests/test_gpu_gram.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_sl3.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/t_sl3.log | tail -30; tail -3 gpurun_out/t_sl3.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_lan1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lan1 -o run -- python3 $R/bench.py --method TensorLanczos --no-cpu-baseline --no-end-to-end --steps 5 --warmup 1 > $R/gpurun_out/prof_lan1.log 2>&1 || { echo "prof failed"; tail -5 $R/gpurun_out/prof_lan1.log; exit 1; }
cd $R
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_lan1/run_kernel_stats.csv')):
    if any(x in r['Name'] for x in ('k_lan_1w','k_red_lan','k_fin_vy','k_basis_mul','k_gram')): print(r['Name'][:50], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))"
timeout -k 10 300 python bench.py --method TensorLanczos --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/lan_final.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 gpurun_out/lan_final.log | cut -c1-600
