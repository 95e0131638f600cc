# GPU box: k-mer table scans by mode and windows per lane (cfg2, cfg3, cfg5 paired sample); JSON lines
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_kt2.jsonl
: > $OUT
run() {  # cfg mode ilp extra...
  local cfg=$1 mode=$2 ilp=$3; shift 3
  timeout -k 10 300 python bench.py --config $cfg --mode $mode --no-cpu-baseline --no-pcie --tune ilp_kt=$ilp "$@" \
      > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  tail -1 gpurun_out/sw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r={'cfg':$cfg,'mode':'$mode','ilp_kt':$ilp,'value':d['value'],'kernel_ms':d['roofline']['avg_kernel_ms'],'lf_value':(d['lf_steps'] or {}).get('value'),'table':d['config']['kmer_table']};print(json.dumps(r))" | tee -a $OUT
}
for mode in global local; do
  for ilp in 1 2; do
    run 2 $mode $ilp
    run 3 $mode $ilp --reads 2000000 --steps 5 --warmup 1
    run 5 $mode $ilp --reads 1000000 --steps 3 --warmup 1
  done
done
