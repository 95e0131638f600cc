#!/bin/bash
# `speq scan` (config 3 files, cached .dat) under rocprofv3 --hip-trace --kernel-trace --stats on the GPU box: where
# the CLI's fixed costs go (index load, device open, per-k structures). Output gpurun_out/cli_trace/.
# CLI_NOPROF=1 skips the profiled run. SPEQ_FULL_EXIT=1 on the profiled run: the CLI's quick exit skips atexit handlers, where the profiler writes.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
W=$(mktemp -d /tmp/speq_cli_XXXX)
python - "$W" <<'PY' || exit 1
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from speq_amd import synth
import bench
w = sys.argv[1]
c = synth.CONFIGS[3]
ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
open(os.path.join(w, "refs.fa"), "w").write(ref.fasta_text())
open(os.path.join(w, "groups.txt"), "w").write(ref.groupings_text())
reads = synth.make_reads(ref, int(os.environ.get("CLI_READS", "10000000")))
bench.write_fastq(os.path.join(w, "r1.fq"), reads)
PY
OUT=${CLI_OUT:-$GRAFT_REPO_ROOT/gpurun_out/cli_trace}; mkdir -p $OUT
cd $W
export SPEQ_CLI_TIMING=1 SPEQ_STARTUP_TRACE=1
timeout -k 10 120 $GRAFT_REPO_ROOT/bin/speq index -r refs.fa -g groups.txt -x ref -t 16 > $OUT/index.log 2>&1 || exit 1
timeout -k 10 120 $GRAFT_REPO_ROOT/bin/speq scan -1 r1.fq -x ref -k 31 -t 16 -o o1.txt > $OUT/scan1.log 2>&1 || exit 1
for i in ${CLI_REPS:-1 2 3}; do timeout -k 10 120 python -c "import os, subprocess, sys, time; t = time.time(); r = subprocess.call(sys.argv[1:], env=dict(os.environ, SPEQ_T0=str(time.time_ns()))); print('wall %.3f s' % (time.time() - t), file=sys.stderr); sys.exit(r)" $GRAFT_REPO_ROOT/bin/speq scan -1 r1.fq -x ref -k 31 -t 16 -o o2_$i.txt > $OUT/scan2_$i.log 2>&1 || exit 1; done
[ -n "$CLI_NOPROF" ] || SPEQ_FULL_EXIT=1 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $OUT/prof -o scan --output-format csv -- $GRAFT_REPO_ROOT/bin/speq scan -1 r1.fq -x ref -k 31 -t 16 -o o3.txt > $OUT/scan3.log 2>&1; rc=$?
cd /; rm -rf $W
grep -h "speq: \|speq-trace\|wall" $OUT/scan2_*.log
exit $rc
