#!/bin/bash
# Round 4 exploration (GPU box): section-clock breakdown of k_scan_ax (instrumented twin) at configs 2 and 5, error and
# k sensitivity, config 5's per-read cost against its working set (50 / 100 / 200 variants x 5 isolates), and the
# lowest-position representatives (default) against first-claimant ones (build/variants/rep0).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/explore.jsonl
: > $O
tag() { echo "{\"case\": \"$1\"}" >> $O; }
tag cfg2_base && timeout -k 10 240 python scripts/ax_probe.py --k 21,31,70 --err 0,0.001,0.005 --stats >> $O 2> gpurun_out/explore.err && \
tag cfg2_r3 && SPEQ_LIB_PATH=build/variants/r3/libspeq_scan.so timeout -k 10 240 python scripts/ax_probe.py --k 21,70 --err 0.001 >> $O 2>> gpurun_out/explore.err && \
tag cfg2_lin && SPEQ_LIB_PATH=build/variants/lin/libspeq_scan.so timeout -k 10 240 python scripts/ax_probe.py --k 21,70 --err 0.001 >> $O 2>> gpurun_out/explore.err && \
tag cfg2_hw3w4 && SPEQ_LIB_PATH=build/variants/hw3w4/libspeq_scan.so timeout -k 10 240 python scripts/ax_probe.py --k 70 --err 0.001 >> $O 2>> gpurun_out/explore.err && \
tag cfg2_local && timeout -k 10 240 python scripts/ax_probe.py --k 21,70 --err 0.001 --local --stats >> $O 2>> gpurun_out/explore.err && \
tag cfg5_v200_r3 && SPEQ_LIB_PATH=build/variants/r3/libspeq_scan.so timeout -k 10 300 python scripts/ax_probe.py --config 5 --paired --reads 4000000 --k 31 --err 0.001 --stats >> $O 2>> gpurun_out/explore.err && \
tag cfg5_v200_lin && SPEQ_LIB_PATH=build/variants/lin/libspeq_scan.so timeout -k 10 300 python scripts/ax_probe.py --config 5 --paired --reads 4000000 --k 31 --err 0.001 --stats >> $O 2>> gpurun_out/explore.err && \
for v in 200 100 50; do
  tag cfg5_v$v
  timeout -k 10 300 python scripts/ax_probe.py --config 5 --paired --reads 4000000 --variants $v --k 31 --err 0.001 --stats >> $O 2>> gpurun_out/explore.err || exit 1
done
echo explore-done
