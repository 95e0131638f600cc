# A/B: default library vs variants named in $VARIANTS, same sweep args
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in default $VARIANTS; do
  if [ "$v" = default ]; then unset SPEQ_LIB_PATH; else export SPEQ_LIB_PATH=build/variants/$v/libspeq_scan.so; fi
  echo "== $v"
  timeout -k 10 600 python scripts/sweep.py "$@" > gpurun_out/ab_$v.jsonl 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/ab_$v.jsonl'):
    d = json.loads(l)
    if 'kmers_per_s' in d: print(d['config'], d['k'], d['prefix_q'], d.get('pairs'), d.get('lab'), d['mode'], d.get('blocks_per_cu'), d.get('ilp'), round(d['kernel_ms_median'],3), '%.3g' % d['kmers_per_s'], d['counts_match_first'])
"
done
