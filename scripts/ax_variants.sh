#!/bin/bash
# A/B of k_scan_ax build variants (make axvariant NAME=...) on the GPU box: scripts/ax_probe.py per variant.
# Usage: bash scripts/ax_variants.sh "base p1 p2 w5" [ax_probe args...]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VARS=$1; shift
for v in $VARS; do
    if [ "$v" = base ]; then lib=""; else lib="build/variants/$v/libspeq_scan.so"; fi
    echo "== $v" >> gpurun_out/ax_variants.jsonl
    SPEQ_LIB_PATH=$lib timeout -k 10 240 python scripts/ax_probe.py "$@" | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/ax_variants.jsonl || exit $?
done
