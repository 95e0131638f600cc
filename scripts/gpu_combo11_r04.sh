#!/bin/bash
# config 5 (structures larger than the MALL): blocks per CU 2 / 3 / 4 (default LDS-limited 4)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
C5="--config 5 --reads 4000000 --paired --k 31 --err 0.001 --reps 3"
bash scripts/ab_r04.sh 2 "base" "cfg5b4|$C5" "cfg5b3|$C5 --tune blocks_per_cu_ax=3" "cfg5b2|$C5 --tune blocks_per_cu_ax=2"
