#!/usr/bin/env python3
"""What a bench step costs beyond its scan kernel (GPU box): config 2's 1 M reads in HBM, k = 21, 200 back-to-back steps
timed with perf_counter around a synchronize, in four forms — zeroed counters + HIP timing events per launch (bench.py's
step), zeroed counters without events, events without zeroing, the scan alone. Prints one JSON line per form."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (torch first: one HIP runtime per process)
import numpy as np  # noqa: E402

from speq_amd import DeviceIndex, FmIndex, synth  # noqa: E402


def main():
    c = dict(synth.CONFIGS[2])
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True, triple_steps=True,
                        gpu_device=0)
    dev = DeviceIndex(idx, 0)
    reads = synth.make_reads(ref, c["n_reads"], err_rate=0.001)
    d_seq = torch.from_numpy(reads.seq).cuda()
    d_qual = torch.from_numpy(reads.qual).cuda()
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
    k, G = 21, c["n_variants"]
    dev.prepare(k)
    cnt = torch.zeros(G + 2, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    steps = 200
    for name, zero, events in (("zero+events", True, True), ("zero", True, False), ("events", False, True),
                               ("scan", False, False), ("zero+events", True, True)):
        def step():
            if zero:
                cnt.zero_()
            dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k, cnt.data_ptr(), 0,
                            stream=stream)
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        dev.timing(events)
        if events:
            dev.timing_read()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
        kern = dev.timing_read()[0] / steps if events else None
        dev.timing(False)
        print(json.dumps({"form": name, "ms_per_step": round(el, 4), "kernel_ms": kern and round(kern, 4)}), flush=True)


if __name__ == "__main__":
    main()
