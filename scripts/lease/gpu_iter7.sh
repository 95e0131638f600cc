# GPU box: parity of the two-deep pipeline, then A/B default vs ktp5 (ilp_kt 1 and 2) on cfg2/3/5 global + cfg2 local
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ktab.py tests/test_gpu_golden.py tests/test_gpu_parity.py \
    tests/test_gpu_em.py tests/test_gpu_fuzz.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/iter7.log 2>&1; rc=$?
tail -3 gpurun_out/iter7.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/ab_2deep.jsonl
: > $OUT
for v in default ktp5; do
  if [ "$v" = default ]; then unset SPEQ_LIB_PATH; else export SPEQ_LIB_PATH=build/variants/$v/libspeq_scan.so; fi
  for ilp in 1 2; do for cm in "2 global" "3 global" "5 global" "2 local"; do
    set -- $cm; cfg=$1; mode=$2
    extra=""; [ $cfg = 3 ] && extra="--reads 2000000 --steps 5 --warmup 1"; [ $cfg = 5 ] && extra="--reads 1000000 --steps 3 --warmup 1"
    timeout -k 10 300 python bench.py --config $cfg --mode $mode --no-cpu-baseline --no-pcie --no-lf-compare --tune ilp_kt=$ilp $extra > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
    tail -1 gpurun_out/sw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'variant':'$v','ilp_kt':$ilp,'cfg':$cfg,'mode':'$mode','value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms'],'U0':d['check']['U'][0]};print(json.dumps(r))" | tee -a $OUT
  done; done
done
