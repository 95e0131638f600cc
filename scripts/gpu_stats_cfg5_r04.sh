#!/bin/bash
# work counters and section clocks of config 5 (paired, k = 31) and config 3 (k = 31)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/ax_probe.py --config 5 --reads 4000000 --paired --k 31 --err 0.001 --reps 3 --stats > gpurun_out/stats_cfg5.jsonl 2>&1 && \
timeout -k 10 300 python scripts/ax_probe.py --config 3 --reads 4000000 --k 31 --err 0.001 --reps 3 --stats >> gpurun_out/stats_cfg5.jsonl 2>&1
