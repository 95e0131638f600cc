# sweep only (no tests)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python scripts/sweep.py "$@" > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err; rc=$?
python -c "
import sys, json
for l in open('gpurun_out/sweep.jsonl'):
    d = json.loads(l)
    if 'kmers_per_s' in d: print(d['config'], d['k'], d['prefix_q'], d.get('pairs'), d.get('lab'), d['mode'], d.get('blocks_per_cu'), d.get('ilp'), d.get('grid_blocks'), round(d['kernel_ms_median'],3), '%.3g' % d['kmers_per_s'], d['counts_match_first'])
    else: print(d)
"
tail -3 gpurun_out/sweep.err
exit $rc
