# GPU box: k-mer table parity tests, then cfg2/cfg3 bench lines (no CPU baseline)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ktab.py tests/test_gpu_golden.py tests/test_gpu_parity.py \
    tests/test_gpu_fuzz.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_ktab.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_ktab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_kt_cfg2.log 2>&1 && tail -1 gpurun_out/bench_kt_cfg2.log && \
timeout -k 10 300 python bench.py --no-cpu-baseline --ilp 1 --no-pcie > gpurun_out/bench_kt_cfg2_ilp1.log 2>&1 && tail -1 gpurun_out/bench_kt_cfg2_ilp1.log && \
timeout -k 10 400 python bench.py --config 3 --reads 2000000 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/bench_kt_cfg3.log 2>&1 && tail -1 gpurun_out/bench_kt_cfg3.log
