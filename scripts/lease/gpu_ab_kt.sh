# GPU box: A/B of library variants ($VARIANTS, plus default) on the k-mer-table bench, cfg2 and cfg3, ilp_kt 1/2
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/ab_kt.jsonl
: > $OUT
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset SPEQ_LIB_PATH; else export SPEQ_LIB_PATH=build/variants/$v/libspeq_scan.so; fi
  for cfg in 2 3; do
    extra=""; [ $cfg = 3 ] && extra="--reads 2000000 --steps 5 --warmup 1"
    for ilp in 1 2; do
      timeout -k 10 200 python bench.py --config $cfg $extra --no-cpu-baseline --no-pcie --no-lf-compare \
        --tune ilp_kt=$ilp --tune kt_slots=4 $TUNE > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
      tail -1 gpurun_out/ab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'variant':'$v','cfg':$cfg,'ilp_kt':$ilp,'value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms'],'check':d['check']['U'][:3]};print(json.dumps(r))" | tee -a $OUT
    done
  done
done
