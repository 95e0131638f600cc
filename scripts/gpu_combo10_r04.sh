#!/bin/bash
# A/B: global deferred list of 832 entries (5 blocks per CU up to 212 groups) against 896
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
bash scripts/ab_r04.sh 2 "base d832" "cfg5|--config 5 --reads 4000000 --paired --k 31 --err 0.001 --reps 3" "k21|--k 21 --err 0.001" "cfg3|--config 3 --reads 4000000 --k 31 --err 0.001"
