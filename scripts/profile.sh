#!/bin/bash
# rocprofv3 passes over one bench workload (run on the GPU box). Kernel trace + stats in one pass, then one PMC pass
# per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md). The "req" pass
# reads the L2's memory-side request counters by size (TCC_EA0_RDREQ = all, TCC_BUBBLE = 128 B, TCC_EA0_RDREQ_32B),
# from which scripts/summarize_profile.py computes the fabric bytes (calibration: scripts/calibrate_counters.sh).
# Usage: PASSES="trace req" OUT=gpurun_out/prof_x bash scripts/profile.sh [bench args...]
#   default PASSES = trace req fetch write tcc sq sq2 ta; OUT default gpurun_out/prof
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export SPEQ_BENCH_NO_STATS=1  # no instrumented k_scan_ax launch among the profiled ones
OUT=${OUT:-gpurun_out/prof}
PASSES=${PASSES:-"trace req fetch write tcc sq sq2 ta"}
mkdir -p $OUT
BENCH="bench.py --steps 5 --warmup 1 --streams 1 --regions 1 --no-cpu-baseline --no-pcie --no-lf-compare --no-extra --detail $OUT/detail.json $*"
run() {  # name, rocprof args...
    local name=$1; shift
    echo "== $name" >&2
    timeout -k 10 420 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $BENCH > $OUT/$name.log 2>&1
}
rc=0
for p in $PASSES; do
    case $p in
        trace) run trace --kernel-trace --stats ;;
        req) run req --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum ;;
        fetch) run fetch --pmc FETCH_SIZE ;;
        write) run write --pmc WRITE_SIZE ;;
        tcc) run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum ;;
        sq) run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE ;;
        sq2) run sq2 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE ;;
        ta) run ta --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum ;;
        *) echo "unknown pass $p" >&2; false ;;
    esac
    rc=$?
    [ $rc -eq 0 ] || break
done
echo "profile rc=$rc" >&2
exit $rc
