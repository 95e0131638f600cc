# GPU box: grid_blocks_kt sweep on cfg2/cfg3 (global) after the SGPR-wave-index kernel
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_grid_kt2.jsonl
: > $OUT
for g in 4096 8192 16384 32768; do
  for cfg in 2 3; do
    extra=""; [ $cfg = 3 ] && extra="--reads 2000000 --steps 5 --warmup 1"
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-pcie --no-lf-compare --tune grid_blocks_kt=$g $extra > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
    tail -1 gpurun_out/sw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'grid_blocks_kt':$g,'cfg':$cfg,'value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms']};print(json.dumps(r))" | tee -a $OUT
  done
done
