#!/bin/bash
# One build -> measure iteration on the GPU box: the k_scan_ax parity tests, then the default bench line (no CPU
# baseline / PCIe / extra lines) into gpurun_out/<tag>.json. Usage: bash scripts/gpu_iter.sh <tag> [bench args...]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_ax.py tests/test_gpu_golden.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG.tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --no-lf-compare --no-extra "$@" > gpurun_out/$TAG.json \
    2> gpurun_out/$TAG.err
rc=$?; echo "bench rc=$rc"; exit $rc
