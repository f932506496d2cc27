# emulated N=8 device rate with the RCCL channel count capped (the records all-reduce is ~28 KB
# per group: latency-bound), two repetitions
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  BARGS="--emulate-ranks 8 --no-end-to-end" bash tools/gpu/ab_env.sh n8:TKHIP_XCH_GROUP=4 n8ch1:NCCL_MAX_NCHANNELS=1 n8ch2:NCCL_MAX_NCHANNELS=2 n8nc:TK_EMULATE_NOCOMM=1 || exit 1
done
