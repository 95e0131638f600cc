# GPU box: a subset of the GPU tests (args = test files), verbose, per-test timeout; log in gpurun_out/
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_subset.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_subset.log
exit $rc
