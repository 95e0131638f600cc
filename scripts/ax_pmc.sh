#!/bin/bash
# PMC passes (rocprofv3, one counter group per run) over scripts/ax_probe.py for one k_scan_ax build variant.
# Usage (GPU box): bash scripts/ax_pmc.sh <variant|base> [ax_probe args...]; output gpurun_out/axpmc_<variant>/
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
V=$1; shift
if [ "$V" = base ]; then LIB=""; else LIB="build/variants/$V/libspeq_scan.so"; fi
OUT=gpurun_out/axpmc_$V
mkdir -p $OUT
ARGS="$*"
pass() {
    local name=$1; shift
    SPEQ_LIB_PATH=$LIB timeout -k 10 240 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 scripts/ax_probe.py $ARGS > $OUT/$name.log 2>&1
}
pass trace --kernel-trace --stats && \
pass sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
pass sq2 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE && \
pass tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum && \
pass ta --pmc TA_BUSY_avr TA_TA_BUSY_sum
echo "pmc rc=$?"
