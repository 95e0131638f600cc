# GPU box: table tests + golden, cfg2 bench (ilp 1/2), cfg3 bench, then rocprof passes of the cfg2 bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ktab.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_ktab.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_ktab.log; [ $rc -eq 0 ] || exit $rc
for ilp in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie --ilp $ilp > gpurun_out/bench_cfg2_ilp$ilp.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_cfg2_ilp$ilp.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('cfg2 ilp$ilp',d['value']/1e9,d['roofline']['avg_kernel_ms'],d['lf_steps']['value']/1e9)"
done
timeout -k 10 400 python bench.py --config 3 --reads 2000000 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/bench_cfg3.log 2>&1 || exit 1
tail -1 gpurun_out/bench_cfg3.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('cfg3',d['value']/1e9,d['roofline']['avg_kernel_ms'],d['lf_steps']['value']/1e9)"
export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-lf-compare"
P=gpurun_out/prof_kt
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o trace --output-format csv -- python3 $B > $P/trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $P/sq -o sq --output-format csv -- python3 $B > $P/sq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o fetch --output-format csv -- python3 $B > $P/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $P/tcc -o tcc --output-format csv -- python3 $B > $P/tcc.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $P/sq2 -o sq2 --output-format csv -- python3 $B > $P/sq2.log 2>&1
echo "prof rc=$?"
