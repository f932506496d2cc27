# round-3 evidence, part 1: smoke, default bench (+CPU baselines), C1/C3/C4, rocprofv3 stats
# of the default bench, PMC FETCH/WRITE, and MFMA counters of k_gram / k_basis_mul
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu/full.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/pmc_list.txt 2>&1
AV=$(grep -o -E "\b(SQ|GRBM)_[A-Z0-9_]+\b" $R/gpurun_out/pmc_list.txt | sort -u)
C=""
for x in SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE; do
  echo "$AV" | grep -qx $x && C="$C $x"
done
echo "counters:$C"
rm -rf $R/gpurun_out/pmc_mfma
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_mfma -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_mfma.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/pmc_mfma.log; exit 1; }
cd $R
python3 tools/pmc_kernels.py gpurun_out/pmc_mfma/run_counter_collection.csv --match k_gram > gpurun_out/pmc_mfma_gram.txt
python3 tools/pmc_kernels.py gpurun_out/pmc_mfma/run_counter_collection.csv --match k_basis_mul > gpurun_out/pmc_mfma_bm.txt
cat gpurun_out/pmc_mfma_gram.txt gpurun_out/pmc_mfma_bm.txt
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write C2 1 50 gpurun_out/pmc_C2_n1.json
