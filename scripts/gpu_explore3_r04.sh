#!/bin/bash
# Round 4 exploration 3: deferral-overflow fix (k = 70, 0.5 % errors), k <= 96 instantiation, headline workloads
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/explore3.jsonl
: > $O
tag() { echo "{\"case\": \"$1\"}" >> $O; }
P="timeout -k 10 300 python scripts/ax_probe.py"
tag cfg2 && $P --k 21,31,70 --err 0,0.001,0.005 --stats >> $O 2> gpurun_out/explore3.err && \
tag cfg2_local && $P --k 21,70 --err 0.001,0.005 --local --stats >> $O 2>> gpurun_out/explore3.err && \
tag cfg5 && $P --config 5 --paired --reads 4000000 --k 31 --err 0.001 --stats >> $O 2>> gpurun_out/explore3.err && \
echo explore3-done
