#!/bin/bash
# rocprofv3 passes over the default bench command (run on the GPU box). Kernel trace + stats in one pass, then one
# PMC pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md).
# Output: gpurun_out/prof/<pass>/...; copy the summaries you want judged into profiles/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export SPEQ_BENCH_NO_STATS=1  # no instrumented k_scan_ax launch among the profiled ones
OUT=gpurun_out/prof
mkdir -p $OUT
BENCH="bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-lf-compare --no-extra $*"
run() {  # name, rocprof args...
    local name=$1; shift
    echo "== $name" >&2
    timeout -k 10 420 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $BENCH > $OUT/$name.log 2>&1
}
run trace --kernel-trace --stats && \
run fetch --pmc FETCH_SIZE && \
run write --pmc WRITE_SIZE && \
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum && \
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run sq2 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run ta --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
echo "profile rc=$?" >&2
