cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python scripts/sweep.py --configs 2,3 --reads 1000000 --qs 0,8,10,12 --ref-pass > gpurun_out/sweep1.jsonl 2> gpurun_out/sweep1.err && echo SWEEP_OK && \
bash scripts/profile.sh 2> gpurun_out/profile.err && echo PROF_OK
