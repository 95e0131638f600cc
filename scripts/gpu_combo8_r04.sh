#!/bin/bash
# round-4 exploration: deferred-pass margin / refill threshold / staging variants (interleaved A/B), then a
# translation-cache PMC pass on config 2 k = 21
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
bash scripts/ab_r04.sh 2 "base m64 m128 m128r32 w4su4" "k21|--k 21 --err 0.001,0.005" "k70L|--k 70 --err 0.001,0.005 --local" "k70G|--k 70 --err 0.005" "cfg3|--config 3 --reads 4000000 --k 31 --err 0.001" || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum -d gpurun_out/utcl1 -o utcl1 --output-format csv -- python3 scripts/ax_probe.py --k 21 --err 0.001 > gpurun_out/utcl1.log 2>&1
echo utcl1 rc=$?
