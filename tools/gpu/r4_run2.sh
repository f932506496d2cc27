# round 4, second box: GPU suite, C2 / C1 / C4 lines (end-to-end after the host-math and
# Gram-ahead changes), emulated C2 N=8 and C4 N=8 ranks, MFMA counters of k_basis_mul + k_gram
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_gpu.log 2>&1
rc=$?; echo "pytest EXIT $rc" >> gpurun_out/t_gpu.log
grep -cE "PASSED" gpurun_out/t_gpu.log; grep -E "FAILED|ERROR" gpurun_out/t_gpu.log | tail -15
tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || exit 1
run() {  # name, bench args
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/$nm.log; exit 1; }
  tail -1 gpurun_out/$nm.log > gpurun_out/$nm.json
  python3 -c "
import json; d=json.loads(open('gpurun_out/$nm.json').read()); e=d.get('end_to_end') or {}
print('$nm', d['value'], 'frac', d['roofline']['frac'], 'launch_us', d['roofline']['avg_launch_us'], 'e2e', e.get('iterations_s'), 'ratio', round(e.get('iterations_s',0)/d['value'],3), 'phases', e.get('phases_s'), 'mfma_us', d['basis_mul_mfma']['avg_us'], d['basis_mul_mfma']['TFLOP_s'])"
}
run c2_n1 --steps 10 --warmup 2
run c1_n1 --config C1 --steps 10 --warmup 2
run c4_n1 --config C4 --steps 10 --warmup 2
run c2_emu8 --steps 6 --warmup 1 --emulate-ranks 8
run c4_emu8_r0 --config C4 --steps 10 --warmup 2 --emulate-ranks 8 --emulate-rank 0
run c4_emu8_r7 --config C4 --steps 10 --warmup 2 --emulate-ranks 8 --emulate-rank 7
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_mfma
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mfma -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_mfma.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/pmc_mfma.log; exit 1; }
python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmc_mfma/run_counter_collection.csv --match k_ | tee $R/gpurun_out/pmc_mfma.txt
