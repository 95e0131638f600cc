#!/bin/bash
# refill sub-section clocks (config 2 k = 21, config 3 k = 31), then A/B of three-chunk-batch staging (su3)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
timeout -k 10 300 python scripts/ax_probe.py --k 21 --err 0.001 --stats > gpurun_out/stats9.jsonl 2>&1 && \
timeout -k 10 300 python scripts/ax_probe.py --config 3 --reads 4000000 --k 31 --err 0.001 --reps 3 --stats >> gpurun_out/stats9.jsonl 2>&1 && \
bash scripts/ab_r04.sh 2 "base su3" "k21|--k 21 --err 0.001" "cfg3|--config 3 --reads 4000000 --k 31 --err 0.001"
