# GPU box: parity of the pipelined table kernel, then A/B: pipeline off/on, occupancy variants; cfg2/3/5, global/local
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ktab.py tests/test_gpu_golden.py tests/test_gpu_parity.py \
    tests/test_gpu_em.py tests/test_gpu_stream.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/iter5.log 2>&1; rc=$?
tail -3 gpurun_out/iter5.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/ab_ktp.jsonl
: > $OUT
run() {  # variant pipeline cfg mode
  local v=$1 pl=$2 cfg=$3 mode=$4
  if [ "$v" = default ]; then unset SPEQ_LIB_PATH; else export SPEQ_LIB_PATH=build/variants/$v/libspeq_scan.so; fi
  extra=""; [ $cfg = 3 ] && extra="--reads 2000000 --steps 5 --warmup 1"; [ $cfg = 5 ] && extra="--reads 1000000 --steps 3 --warmup 1"
  timeout -k 10 300 python bench.py --config $cfg --mode $mode --no-cpu-baseline --no-pcie --no-lf-compare --tune kt_pipeline=$pl $extra > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  tail -1 gpurun_out/sw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'variant':'$v','pipeline':$pl,'cfg':$cfg,'mode':'$mode','value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms'],'U0':d['check']['U'][0]};print(json.dumps(r))" | tee -a $OUT
}
for cfg in 2 3 5; do
  run default 0 $cfg global
  for v in default ktp6; do run $v 1 $cfg global; done
  run ktp6 1 $cfg local
  run default 0 $cfg local
  run default 1 $cfg local
done
