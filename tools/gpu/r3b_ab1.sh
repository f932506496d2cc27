# round 3 (second session): k_gram pipelining / block-count A/B, then k_arn_d1 s_setprio A/B (C2 N=1 and emulated N=8 rank 5)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
: > gpurun_out/gramab3.log
for rep in 1 2; do for v in gram_old pipe_gq8 pipe_gq4 pipe_gq4_b256 pipe_gq4_b1024; do
  TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 120 python tools/gram_bench.py >> gpurun_out/gramab3.log 2>&1 || { echo "variant $v failed"; tail -3 gpurun_out/gramab3.log; exit 1; }
done; done
cat gpurun_out/gramab3.log
for rep in 1 2; do for v in pipe_gq8 d1prio1 d1prio3; do
  for mode in n1 e8; do
    if [ $mode = n1 ]; then EXTRA=""; else EXTRA="--emulate-ranks 8 --emulate-rank 5"; fi
    TKHIP_LIB=$R/tools/_build/libtkhip_$v.so timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-end-to-end $EXTRA > gpurun_out/ab1_${v}_$mode.log 2>&1 || { echo "bench $v $mode failed"; tail -5 gpurun_out/ab1_${v}_$mode.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab1_${v}_$mode.log').read().strip().split('\n')[-1]); print('rep$rep $v $mode', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
  done
done; done
