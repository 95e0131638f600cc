#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ax_probe.py --k 21,70 --err 0.001,0.005 --stats > gpurun_out/stats6.jsonl 2>&1 && \
timeout -k 10 300 python scripts/ax_probe.py --k 21,70 --err 0.001,0.005 --local --stats >> gpurun_out/stats6.jsonl 2>&1 && \
bash scripts/ab_r04.sh 2 "base pf blk32" "k21|--k 21,31 --err 0.001" "k70L|--k 70 --err 0.001,0.005 --local" "cfg3|--config 3 --reads 4000000 --k 31 --err 0.001"
