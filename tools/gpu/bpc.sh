# d1 occupancy cap sweep (TKHIP_D1_BPC = blocks per CU via dynamic LDS) at N=1 and emulated N=8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for N in 8 1; do for B in 0 1 2 3 4; do
  TKHIP_D1_BPC=$B timeout -k 10 200 python bench.py --emulate-ranks $N --steps 4 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/bpc$N_$B.log 2>&1 || { echo "N=$N B=$B failed"; tail -5 gpurun_out/bpc$N_$B.log; exit 1; }
  tail -1 gpurun_out/bpc$N_$B.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$N bpc=$B', d['value'], d['roofline']['avg_launch_us'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done; done
