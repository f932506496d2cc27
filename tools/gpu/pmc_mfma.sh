# MFMA counters of the standalone V*Y kernel (k_basis_mul) over one C2 bench pass
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp; mkdir -p $R/gpurun_out
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/pmc_list.txt 2>&1
AV=$(grep -o -E "\b(SQ|GRBM)_[A-Z0-9_]+\b" $R/gpurun_out/pmc_list.txt | sort -u)
echo "$AV" | grep MFMA | tr '\n' ' '; echo
C=""
for x in SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE; do
  echo "$AV" | grep -qx $x && C="$C $x"
done
echo "counters:$C"
rm -rf $R/gpurun_out/pmc_mfma
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_mfma -o run -- python3 $R/bench.py --pmc-mode > $R/gpurun_out/pmc_mfma.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/pmc_mfma.log; exit 1; }
python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmc_mfma/run_counter_collection.csv --match k_basis_mul
