#!/bin/bash
# Round check on the GPU box: GPU tests, smoke, the default bench (compact line + detail file), then rocprofv3 passes
# of the cfg2 headline (all counter groups). Usage: bash scripts/round_check.sh [tag]
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 900 python bench.py --detail gpurun_out/bench_detail.json > gpurun_out/bench_default.log 2>&1 && tail -c 600 gpurun_out/bench_default.log && \
rm -rf gpurun_out/prof_cfg2 && OUT=gpurun_out/prof_cfg2 bash scripts/profile.sh 2> gpurun_out/profile_cfg2.err && echo PROFILES_OK
