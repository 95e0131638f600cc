# GPU box: A/B of library variants ($VARIANTS plus default) on cfg2/cfg3/cfg5, global mode (ilp_kt $ILP), plus the
# bs2 variant's parity on the table tests when it is listed
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/ab_variants.jsonl
: > $OUT
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset SPEQ_LIB_PATH; else export SPEQ_LIB_PATH=build/variants/$v/libspeq_scan.so; fi
  if [ "$v" = bs2 ]; then
    timeout -k 10 300 python -u -m pytest tests/test_gpu_ktab.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/bs2.log 2>&1 || { tail -5 gpurun_out/bs2.log; exit 1; }
    tail -1 gpurun_out/bs2.log
  fi
  for cfg in 2 3 5; do
    extra=""; [ $cfg = 3 ] && extra="--reads 2000000 --steps 5 --warmup 1"; [ $cfg = 5 ] && extra="--reads 1000000 --steps 3 --warmup 1"
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-pcie --no-lf-compare --tune ilp_kt=${ILP:-1} $extra > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
    tail -1 gpurun_out/sw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'variant':'$v','cfg':$cfg,'value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms'],'table':d['config']['kmer_table']['bytes'],'U0':d['check']['U'][0]};print(json.dumps(r))" | tee -a $OUT
  done
done
