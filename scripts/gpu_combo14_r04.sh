#!/bin/bash
# minimizer-keyed Bloom filter: parity of the anchor-kernel tests with the filter forced on (fmin0), then A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
SPEQ_LIB_PATH=build/variants/fmin0/libspeq_scan.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ax.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_fmin0.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_fmin0.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_r04.sh 2 "base fmin fmin0" "cfg5|--config 5 --reads 4000000 --paired --k 31 --err 0.001 --reps 3" "cfg3|--config 3 --reads 4000000 --k 31 --err 0.001,0.005" "k31|--k 31 --err 0.001"
