# one iteration: GPU parity tests, then the kernel sweep (args passed to sweep.py)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/sweep.py "$@" > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err; rc=$?
cat gpurun_out/sweep.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if 'kmers_per_s' in d: print(d['config'], d['k'], d['prefix_q'], d.get('pairs'), d.get('lab'), d['mode'], d.get('blocks_per_cu'), d.get('ilp'), d.get('grid_blocks'), round(d['kernel_ms_median'],3), '%.3g' % d['kmers_per_s'], d['counts_match_first'])
    else: print(d)
"
exit $rc
