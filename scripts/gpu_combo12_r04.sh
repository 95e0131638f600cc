#!/bin/bash
# A/B: dynamic tail (SPEQ_AX_TAIL percent of the units handed out at run time, SPEQ_AX_GRAB at a time)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
bash scripts/ab_r04.sh 2 "base t10 t25 t50 t25g16" "k21|--k 21 --err 0.001" "k70L|--k 70 --err 0.001,0.005 --local" "cfg3|--config 3 --reads 4000000 --k 31 --err 0.001"
