# bench + rocprof passes for config 2 (k=21) and config 3 (k=31, first 2M reads)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_cfg2.log 2>&1 && tail -1 gpurun_out/bench_cfg2.log && \
timeout -k 10 400 python bench.py --config 3 --reads 2000000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2>&1 && tail -1 gpurun_out/bench_cfg3.log && \
bash scripts/profile.sh 2> gpurun_out/profile_cfg2.err && mv gpurun_out/prof gpurun_out/prof_cfg2 && \
bash scripts/profile.sh --config 3 --reads 2000000 2> gpurun_out/profile_cfg3.err && mv gpurun_out/prof gpurun_out/prof_cfg3 && echo PROFILES_OK
