#!/bin/bash
# Calibrates the L2 -> fabric request counters on gfx950 for k_scan_ax's access patterns (tools/microbench/req_size:
# a 16-B/lane stream and 16/64/128-B random gathers over a 2 GiB buffer, known distinct bytes). One rocprofv3 pass per
# counter group (MI355X_MICROARCH.md: FETCH_SIZE alone; the three request counters together).
# Usage (GPU box): bash scripts/calibrate_counters.sh   -> gpurun_out/calib/<pass>/...
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/calib
mkdir -p $OUT
pass() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- ./tools/microbench/req_size > $OUT/$name.log 2>&1
}
pass trace --kernel-trace --stats && \
pass req --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum && \
pass fetch --pmc FETCH_SIZE && \
pass hit --pmc TCC_HIT_sum TCC_MISS_sum
echo "calibrate rc=$?"
