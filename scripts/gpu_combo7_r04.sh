#!/bin/bash
# round-4 exploration: phase-2 sub-section stats, then an interleaved A/B of staging variants
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
timeout -k 10 300 python scripts/ax_probe.py --k 21,70 --err 0.001,0.005 --stats > gpurun_out/stats7.jsonl 2>&1 && \
timeout -k 10 300 python scripts/ax_probe.py --k 70 --err 0.001,0.005 --local --stats >> gpurun_out/stats7.jsonl 2>&1 && \
bash scripts/ab_r04.sh 2 "base w4su4 w4su4n ref8 ref32" "k21|--k 21,31 --err 0.001" "k70L|--k 70 --err 0.001,0.005 --local" "cfg3|--config 3 --reads 4000000 --k 31 --err 0.001"
