#!/bin/bash
# Round check on the GPU box: GPU tests, smoke, the default bench (cfg2 + local mode + cfg3 k=31 lines), then
# rocprofv3 passes of the cfg2 headline and of cfg3 at its full 10 M reads. Usage: bash scripts/round_check.sh [tag]
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log && \
rm -rf gpurun_out/prof gpurun_out/prof_cfg2 gpurun_out/prof_cfg3 && \
bash scripts/profile.sh 2> gpurun_out/profile_cfg2.err && mv gpurun_out/prof gpurun_out/prof_cfg2 && \
bash scripts/profile.sh --config 3 2> gpurun_out/profile_cfg3.err && mv gpurun_out/prof gpurun_out/prof_cfg3 && echo PROFILES_OK
