#!/bin/bash
# Round 4 exploration 2: median representatives (default) against the first claimant (rep0) and the cuckoo table (ck)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/explore2.jsonl
: > $O
tag() { echo "{\"case\": \"$1\"}" >> $O; }
P="timeout -k 10 300 python scripts/ax_probe.py"
tag cfg2_med && $P --k 21,31,70 --err 0,0.001,0.005 --stats >> $O 2> gpurun_out/explore2.err && \
tag cfg2_med_local && $P --k 21,70 --err 0.001,0.005 --local --stats >> $O 2>> gpurun_out/explore2.err && \
tag cfg2_rep0 && SPEQ_LIB_PATH=build/variants/rep0/libspeq_scan.so $P --k 21,70 --err 0.001 --stats >> $O 2>> gpurun_out/explore2.err && \
tag cfg2_ck && SPEQ_LIB_PATH=build/variants/ck/libspeq_scan.so $P --k 21,70 --err 0.001 >> $O 2>> gpurun_out/explore2.err && \
tag cfg5_med && $P --config 5 --paired --reads 4000000 --k 31 --err 0.001 --stats >> $O 2>> gpurun_out/explore2.err && \
tag cfg5_rep0 && SPEQ_LIB_PATH=build/variants/rep0/libspeq_scan.so $P --config 5 --paired --reads 4000000 --k 31 --err 0.001 --stats >> $O 2>> gpurun_out/explore2.err && \
tag cfg3_med && $P --config 3 --reads 10000000 --k 31 --err 0.001 --stats >> $O 2>> gpurun_out/explore2.err && \
echo explore2-done
