#!/bin/bash
# final tree: GPU tests + smoke + a short default bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 900 python bench.py --detail gpurun_out/bench_detail.json > gpurun_out/bench_default.log 2>&1 && tail -c 200 gpurun_out/bench_default.log
