# one rocprofv3 --pmc pass of SQ counters over one C2 sweep (bench.py --pmc-mode), summarized per kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/pmc_sq
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_sq.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/pmc_sq.log; exit 1; }
python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmc_sq/run_counter_collection.csv --match k_arn_d1
