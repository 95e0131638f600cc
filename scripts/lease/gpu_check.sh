cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 && echo BENCH_OK
