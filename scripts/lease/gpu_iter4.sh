# GPU box: table + golden + parity tests, then local/global benches (cfg2, cfg3, cfg5 sample)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ktab.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_em.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/iter4.log 2>&1; rc=$?
tail -3 gpurun_out/iter4.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/sweep_kt3.jsonl
: > $OUT
for mode in local global; do
  for cfg in 2 3 5; do
    extra=""; [ $cfg = 3 ] && extra="--reads 2000000 --steps 5 --warmup 1"; [ $cfg = 5 ] && extra="--reads 1000000 --steps 3 --warmup 1"
    timeout -k 10 300 python bench.py --config $cfg --mode $mode --no-cpu-baseline --no-pcie $extra > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
    tail -1 gpurun_out/sw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'cfg':$cfg,'mode':'$mode','value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms'],'lf_value':(d['lf_steps'] or {}).get('value')};print(json.dumps(r))" | tee -a $OUT
  done
done
