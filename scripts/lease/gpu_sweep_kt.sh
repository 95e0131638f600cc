# GPU box: k-mer table launch sweep (ilp_kt x kt_slots x blocks_per_cu) on cfg2 and cfg3; one JSON line per run
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_kt.jsonl
: > $OUT
for cfg in 2 3; do
  extra=""; [ $cfg = 3 ] && extra="--reads 2000000 --steps 5 --warmup 1"
  for ilp in 1 2 4; do for slots in 2 4 8; do for bpc in 0 4; do
    timeout -k 10 200 python bench.py --config $cfg $extra --no-cpu-baseline --no-pcie --no-lf-compare \
      --tune ilp_kt=$ilp --tune kt_slots=$slots --tune blocks_per_cu=$bpc > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
    tail -1 gpurun_out/sw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'cfg':$cfg,'ilp_kt':$ilp,'kt_slots':$slots,'bpc':$bpc,'value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms'],'table_bytes':d['config']['kmer_table']['bytes']};print(json.dumps(r))" | tee -a $OUT
  done; done; done
done
