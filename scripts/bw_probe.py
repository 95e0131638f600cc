#!/usr/bin/env python3
"""HBM read-rate probe on the bench's read buffers (GPU box): torch reductions over seq/qual, timed with events."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import numpy as np
from speq_amd import synth

ref = synth.make_reference(10, 1, 50_000)
for n in (1_000_000, 4_000_000):
    reads = synth.make_reads(ref, n)
    s = torch.from_numpy(reads.seq).cuda()
    q = torch.from_numpy(reads.qual).cuda()
    s64 = s[: (s.numel() // 8) * 8].view(torch.int64)
    q64 = q[: (q.numel() // 8) * 8].view(torch.int64)
    for name, fn, nbytes in (("sum_seq_i64", lambda: s64.sum(), s64.numel() * 8),
                             ("sum_seq+qual", lambda: (s64.sum(), q64.sum()), 2 * s64.numel() * 8),
                             ("xor_seq_qual", lambda: torch.bitwise_xor(s64, q64), 3 * s64.numel() * 8)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(json.dumps({"reads": n, "op": name, "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}), flush=True)
