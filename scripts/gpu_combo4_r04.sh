#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_r04.sh 2 "base nopf nospec nopfnospec" "k21|--k 21 --err 0.001" "k70|--k 70 --err 0.001,0.005" "k70L|--k 70 --err 0.001,0.005 --local" && \
bash scripts/ab_r04.sh 1 "base nopf" "cfg5|--config 5 --paired --reads 4000000 --k 31 --err 0.001"
