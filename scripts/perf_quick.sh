#!/bin/bash
# Quick perf pass on the GPU box: bench (cfg2 global + local + cfg3 k=31, no CPU baseline), a k=70 line, and
# rocprofv3 trace + PMC passes of the cfg2 headline. Usage: bash scripts/perf_quick.sh [extra bench args]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcie "$@" > gpurun_out/bench_quick.log 2>&1 && tail -1 gpurun_out/bench_quick.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
f=lambda x: {k: x.get(k) for k in ('value','ms_per_step')} | {'kern_ms': x['roofline']['avg_kernel_ms'], 'frac': round(x['roofline']['frac'],3)}
print('cfg2', f(d)); print('local', f(d['local_mode'])); print('k31', f(d['k31'])); print('prev', d.get('kmer_table_kernel'))" && \
timeout -k 10 200 python bench.py --k 70 --no-extra --no-cpu-baseline --no-pcie "$@" > gpurun_out/bench_k70.log 2>&1 && tail -1 gpurun_out/bench_k70.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('k70', d['value'], d['roofline']['avg_kernel_ms'], 'lf', d['lf_steps']['avg_kernel_ms'] if d['lf_steps'] else None)" && \
rm -rf gpurun_out/prof && bash scripts/profile.sh "$@" 2> gpurun_out/profile.err && echo PROFILE_OK
