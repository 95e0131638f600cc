#!/bin/bash
# Pipelined-launch sweep of the headline (GPU box): grid size of k_scan_ax x streams, one bench process per point,
# compact lines into gpurun_out/pipe_sweep.jsonl. Usage: bash scripts/pipe_sweep.sh "1280 1024 768 640" "2 3" [bench args]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GRIDS=${1:-"1280 1024 768 640"}; STREAMS=${2:-"2"}; shift 2
out=gpurun_out/pipe_sweep.jsonl
for s in $STREAMS; do for g in $GRIDS; do
  timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --no-pcie --no-lf-compare --streams $s \
      --tune grid_blocks_ax=$g --detail gpurun_out/pipe_sweep_detail.json "$@" > gpurun_out/pipe_sweep_one.json 2> gpurun_out/pipe_sweep.err || exit 1
  python - "$g" "$s" >> $out <<'PY'
import json, sys
d = json.loads(open("gpurun_out/pipe_sweep_one.json").read().strip().splitlines()[-1])
print(json.dumps({"grid": int(sys.argv[1]), "streams": int(sys.argv[2]), "value": d["value"], "min": d["value_min"],
                  "max": d["value_max"], "overlap": d["overlap"], "one_stream": (d["one_stream"] or {}).get("value"),
                  "kernel_ms": d["roofline"]["avg_kernel_ms"], "ms_per_step": d["ms_per_step"], "check": d["check"]}))
PY
  tail -1 $out
done; done
