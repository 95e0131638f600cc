#!/bin/bash
# Interleaved A/B of k_scan_ax builds (GPU box): every round runs each variant once per case (box drift +-5 %,
# DESIGN.md §4e); output gpurun_out/ab.jsonl. Usage: bash scripts/ab_r04.sh ROUNDS "base var1 var2" [case ...]
# case = "name|probe args"; base = the product library.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/ab.jsonl
ROUNDS=$1; VARS=$2; shift 2
for r in $(seq 1 $ROUNDS); do
  for c in "$@"; do
    name=${c%%|*}; args=${c#*|}
    for v in $VARS; do
      if [ "$v" = base ]; then lib=""; else lib="build/variants/$v/libspeq_scan.so"; fi
      echo "{\"round\": $r, \"case\": \"$name\", \"variant\": \"$v\"}" >> $O
      SPEQ_LIB_PATH=$lib timeout -k 10 300 python scripts/ax_probe.py $args >> $O 2>> gpurun_out/ab.err || exit 1
    done
  done
done
echo ab-done
