# round 4: rocprofv3 kernel stats of C2 TensorLanczos with single-column / paired tiles, and the
# PMC FETCH / WRITE passes of the single-column sweep (HBM bytes per step)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  rm -rf $R/gpurun_out/prof_lan$v
  TKHIP_LANCZOS_SL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lan$v -o run -- python3 $R/bench.py --method TensorLanczos --no-cpu-baseline --no-end-to-end --steps 5 --warmup 1 > $R/gpurun_out/prof_lan$v.log 2>&1 || { echo "prof $v failed"; tail -5 $R/gpurun_out/prof_lan$v.log; exit 1; }
  grep -E "k_lan_1w|k_red_lan|k_fin_vy|k_basis_mul|k_gram" $R/gpurun_out/prof_lan$v/run_kernel_stats.csv | cut -d, -f1-4
done
rm -rf $R/gpurun_out/pmcl_fetch $R/gpurun_out/pmcl_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcl_fetch -o run -- python3 $R/bench.py --method TensorLanczos --pmc-mode > $R/gpurun_out/pmcl_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcl_write -o run -- python3 $R/bench.py --method TensorLanczos --pmc-mode > $R/gpurun_out/pmcl_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R
python3 tools/pmc_traffic.py gpurun_out/pmcl_fetch gpurun_out/pmcl_write C2 1 50 gpurun_out/pmc_C2_TensorLanczos_n1.json
python3 tools/pmc_kernels.py gpurun_out/pmcl_fetch/run_counter_collection.csv --match k_lan_1w
python3 tools/pmc_kernels.py gpurun_out/pmcl_write/run_counter_collection.csv --match k_lan_1w
