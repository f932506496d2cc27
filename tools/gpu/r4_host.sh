# round 4: host math on the box's CPU (EPYC 9575F): per-iteration evaluation with the AVX-512 vs
# the AVX2 GEMM (tools/host_eval_real.py, real C4 / C1 data), then the end-to-end A/Bs of the
# tail helpers' reach (r4_tail.sh) and of the GEMM kernel at C4 / C4 emulated N=8
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in a b; do
  for v in 0 1; do
    for c in C4 C1; do
      TKHIP_HOST_AVX512=$v timeout -k 10 300 python tools/host_eval_real.py $c > gpurun_out/he_${c}_$v$rep.log 2>&1 || { echo "host eval failed"; tail -3 gpurun_out/he_${c}_$v$rep.log; exit 1; }
      echo "avx512=$v $(tail -1 gpurun_out/he_${c}_$v$rep.log)"
    done
  done
done
ab() {  # name, bench args
  local nm=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --e2e-reps 5 "$@" > gpurun_out/hx_$nm.log 2>&1 || { echo "$nm failed"; tail -5 gpurun_out/hx_$nm.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/hx_$nm.log').read().strip().splitlines()[-1]); e=d['end_to_end']
print('== $nm device', d['value'], 'e2e', e['iterations_s'], 'ratio %.3f' % (e['iterations_s'] / d['value']), 'all', e['iterations_s_all'])"
}
for rep in a b; do
  for v in 0 1; do
    TKHIP_HOST_AVX512=$v ab c4_x$v$rep --config C4 || exit 1
    TKHIP_HOST_AVX512=$v ab c4e8r7_x$v$rep --config C4 --emulate-ranks 8 --emulate-rank 7 || exit 1
  done
done
bash tools/gpu/r4_tail.sh
