# full round check: GPU tests, smoke, bench (cfg2 default + cfg3), rocprof passes for both
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 400 python bench.py > gpurun_out/bench_cfg2.log 2>&1 && tail -1 gpurun_out/bench_cfg2.log && \
timeout -k 10 400 python bench.py --config 3 --reads 2000000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2>&1 && tail -1 gpurun_out/bench_cfg3.log && \
rm -rf gpurun_out/prof gpurun_out/prof_cfg2 gpurun_out/prof_cfg3 && \
bash scripts/profile.sh 2> gpurun_out/profile_cfg2.err && mv gpurun_out/prof gpurun_out/prof_cfg2 && \
bash scripts/profile.sh --config 3 --reads 2000000 2> gpurun_out/profile_cfg3.err && mv gpurun_out/prof gpurun_out/prof_cfg3 && echo PROFILES_OK
