#!/bin/bash
# wave imbalance (longest wave vs mean) from the instrumented twin
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ax_probe.py --k 21 --err 0.001 --reps 2 --stats > gpurun_out/stats_imb.jsonl 2>&1 && \
timeout -k 10 300 python scripts/ax_probe.py --k 70 --err 0.001,0.005 --local --reps 2 --stats >> gpurun_out/stats_imb.jsonl 2>&1 && \
timeout -k 10 300 python scripts/ax_probe.py --config 3 --reads 4000000 --k 31 --err 0.001 --reps 2 --stats >> gpurun_out/stats_imb.jsonl 2>&1
