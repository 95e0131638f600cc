#!/bin/bash
# k_scan_ax grid-size sweep on the GPU box (tuning grid_blocks_ax): residency / dispatch-tail probe.
# Usage: bash scripts/grid_sweep.sh "<variant ...>" "<grid ...>" [ax_probe args...]; output gpurun_out/grid_sweep.jsonl
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VARS=$1; GRIDS=$2; shift 2
for v in $VARS; do
    if [ "$v" = base ]; then lib=""; else lib="build/variants/$v/libspeq_scan.so"; fi
    for g in $GRIDS; do
        SPEQ_LIB_PATH=$lib timeout -k 10 120 python scripts/ax_probe.py --tune grid_blocks_ax=$g "$@" | \
            sed "s/^{/{\"variant\": \"$v\", \"grid\": $g, /" >> gpurun_out/grid_sweep.jsonl || exit $?
    done
done
