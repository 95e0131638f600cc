#!/bin/bash
# Interleaved A/B of whole library builds on the GPU box through bench.py (pipelined value, one-stream rate, kernel
# ms, check): build/variants/<name>/libspeq_scan.so per name ("default" = speq_amd/libspeq_scan.so), the list repeated
# AB_REPEAT times (default 2) in turn. Usage: [AB_REPEAT=2] bash scripts/ab_libs.sh "orig bg0 ..." [bench args...]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VARS=$1; shift
out=gpurun_out/ab_libs.jsonl
for rep in $(seq 1 ${AB_REPEAT:-2}); do
  for v in $VARS; do
    if [ "$v" = default ]; then lib=""; else lib="build/variants/$v/libspeq_scan.so"; fi
    SPEQ_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --no-pcie --no-lf-compare \
        --detail gpurun_out/ab_detail_$v.json "$@" > gpurun_out/ab_one.json 2> gpurun_out/ab_libs.err || { echo "variant $v failed"; tail -5 gpurun_out/ab_libs.err; exit 1; }
    python - "$v" "$rep" "$*" >> $out <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
det = json.load(open(f"gpurun_out/ab_detail_{sys.argv[1]}.json"))["head"]["detail"].get("ax_work") or {}
cyc = det.get("cyc_total") or 1
print(json.dumps({"variant": sys.argv[1], "rep": int(sys.argv[2]), "args": sys.argv[3], "value": round(d["value"] / 1e9, 1),
                  "one_stream": round((d["one_stream"] or {}).get("value", 0) / 1e9, 1),
                  "kernel_ms": round(d["roofline"]["avg_kernel_ms"], 4), "ms_per_step": round(d["ms_per_step"], 4),
                  "check": d["check"], "refill_share": round(det.get("cyc_refill", 0) / cyc, 3),
                  "p2_share": round(det.get("cyc_phase2", 0) / cyc, 3),
                  "wave_max_over_mean": round(det.get("cyc_wave_max", 0) / max(1, cyc / max(1, det.get("waves", 1))), 3)}))
PY
    tail -1 $out
  done
done
