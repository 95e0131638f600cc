#!/bin/bash
# grid generations (tuning ax_generations: grid = n x the resident blocks, pools 1/n as large)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
bash scripts/ab_r04.sh 2 "base" "g1|--k 21,31 --err 0.001" "g2|--k 21,31 --err 0.001 --tune ax_generations=2" "g3|--k 21,31 --err 0.001 --tune ax_generations=3" "g4|--k 21,31 --err 0.001 --tune ax_generations=4" \
  "L1|--k 70 --err 0.001,0.005 --local" "L2|--k 70 --err 0.001,0.005 --local --tune ax_generations=2" "L3|--k 70 --err 0.001,0.005 --local --tune ax_generations=3" \
  "c1|--config 3 --reads 4000000 --k 31 --err 0.001" "c2|--config 3 --reads 4000000 --k 31 --err 0.001 --tune ax_generations=2" "c3|--config 3 --reads 4000000 --k 31 --err 0.001 --tune ax_generations=3"
