#!/bin/bash
# One GPU call: GPU tests (stop at the first failure), smoke, the exploration probes, the default bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
bash scripts/gpu_explore_r04.sh && \
timeout -k 10 900 python bench.py --detail gpurun_out/bench_detail.json > gpurun_out/bench_default.log 2>&1 && tail -c 400 gpurun_out/bench_default.log
