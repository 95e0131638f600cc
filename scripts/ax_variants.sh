#!/bin/bash
# A/B of k_scan_ax build variants (make axvariant NAME=...) on the GPU box: scripts/ax_probe.py per variant, the
# variant list repeated AX_REPEAT times (default 1) in turn, so that drifts of the box (clocks after idle) fall on
# every variant alike. Usage: [AX_REPEAT=2] bash scripts/ax_variants.sh "base p1 p2 w5" [ax_probe args...]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VARS=$1; shift
for rep in $(seq 1 ${AX_REPEAT:-1}); do
    for v in $VARS; do
        if [ "$v" = base ]; then lib=""; else lib="build/variants/$v/libspeq_scan.so"; fi
        echo "== $v rep $rep" >> gpurun_out/ax_variants.jsonl
        SPEQ_LIB_PATH=$lib timeout -k 10 240 python scripts/ax_probe.py "$@" | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> gpurun_out/ax_variants.jsonl || exit $?
    done
done
