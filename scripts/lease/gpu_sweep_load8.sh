# GPU box: compact-table load factor (kt_load8, percent) sweep on cfg2, global and local
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_load8.jsonl
: > $OUT
for l in ${LOADS:-12 18 25 35}; do
  for mode in ${MODES:-global local}; do
    timeout -k 10 300 python bench.py --config 2 --mode $mode --no-cpu-baseline --no-pcie --no-lf-compare --tune kt_load8=$l > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
    tail -1 gpurun_out/sw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'kt_load8':$l,'mode':'$mode','value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms'],'table':d['config']['kmer_table']['bytes']};print(json.dumps(r))" | tee -a $OUT
  done
done
