#!/bin/bash
# Runtime tuning A/B through bench.py (pipelined value, one-stream rate, kernel ms), the list repeated AB_REPEAT times
# (default 2) in turn. Usage: bash scripts/ab_tune_bench.sh "ax_load=35 ax_load=50" [bench args...]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VARS=$1; shift
out=gpurun_out/ab_tune_bench.jsonl
for rep in $(seq 1 ${AB_REPEAT:-2}); do
  for v in $VARS; do
    timeout -k 10 240 python bench.py --no-extra --no-cpu-baseline --no-pcie --no-lf-compare --tune $v \
        --detail gpurun_out/ab_tune_detail.json "$@" > gpurun_out/ab_tune_one.json 2> gpurun_out/ab_tune.err || { echo "tune $v failed"; tail -5 gpurun_out/ab_tune.err; exit 1; }
    python - "$v" "$rep" "$*" >> $out <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_tune_one.json").read().strip().splitlines()[-1])
print(json.dumps({"tune": sys.argv[1], "rep": int(sys.argv[2]), "args": sys.argv[3], "value": round(d["value"] / 1e9, 1),
                  "one_stream": round((d["one_stream"] or {}).get("value", 0) / 1e9, 1),
                  "kernel_ms": round(d["roofline"]["avg_kernel_ms"], 4), "table_bytes": d["config"].get("kmer_table", {}).get("bytes"),
                  "check": d["check"]}))
PY
    tail -1 $out
  done
done
