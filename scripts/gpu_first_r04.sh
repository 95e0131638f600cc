#!/bin/bash
# Round 4, first GPU call: counter calibration, then the round check (tests, smoke, bench, cfg2 profile).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/calibrate_counters.sh > gpurun_out/calib.log 2>&1; tail -1 gpurun_out/calib.log
bash scripts/round_check.sh r04
