# Lanczos parity tests, then C2 TensorLanczos with the in-tree library and variant libraries (args: names)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu -x --timeout 200 -k "anczos" > gpurun_out/t_lan.log 2>&1; rc=$?
tail -2 gpurun_out/t_lan.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/t_lan.log | head -20; exit 1; }
for v in tree "$@"; do
  L=""; [ "$v" != tree ] && L="TKHIP_LIB=$R/tools/_build/libtkhip_$v.so"
  env $L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end --method TensorLanczos > gpurun_out/lan_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/lan_$v.log; exit 1; }
  tail -1 gpurun_out/lan_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items() if v['avg_us']})"
done
