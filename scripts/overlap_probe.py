#!/usr/bin/env python3
"""Do consecutive scans overlap when they alternate between HIP streams (GPU box)? Config 2's 1 M reads in HBM,
k = 21 (or --k / --local), 200 back-to-back steps (zeroed counters + scan) on 1, 2 or 3 streams in turn, each
stream with its own counters: the next scan's workgroups can take the CUs the previous one's drain leaves idle.
Prints one JSON line per stream count: ms per step (perf_counter around the loop, synchronized), and whether every
stream's last counters equal the one-stream result."""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reads", type=int, default=0)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--local", action="store_true")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--streams", default="1,2,3,1,2")
    a = ap.parse_args()
    c = dict(synth.CONFIGS[a.config])
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True, triple_steps=True,
                        gpu_device=0)
    dev = DeviceIndex(idx, 0)
    reads = synth.make_reads(ref, a.reads or c["n_reads"], err_rate=0.001)
    d_seq = torch.from_numpy(reads.seq).cuda()
    d_qual = torch.from_numpy(reads.qual).cuda()
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
    G = c["n_variants"]
    dev.prepare(a.k)
    ref_cnt = None
    for form in a.streams.split(","):  # "2": two new streams; "c2": the current stream and one new one
        ns = int(form.lstrip("c"))
        streams = [torch.cuda.Stream() for _ in range(ns)]
        if form.startswith("c"):
            streams[0] = torch.cuda.current_stream()
        cnts = [torch.zeros(G + 2, dtype=torch.int64, device="cuda") for _ in range(ns)]
        ws = [torch.zeros(G, dtype=torch.float64, device="cuda") for _ in range(ns)]

        def step(i):
            s = streams[i % ns]
            with torch.cuda.stream(s):
                cnts[i % ns].zero_()
                if a.local:
                    ws[i % ns].zero_()
                dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, a.k,
                                cnts[i % ns].data_ptr(), ws[i % ns].data_ptr() if a.local else 0, local=a.local,
                                stream=s.cuda_stream)
        torch.cuda.synchronize()
        for i in range(10):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / a.steps * 1e3
        got = [c_.cpu().numpy() for c_ in cnts]
        if ref_cnt is None:
            ref_cnt = got[0]
        equal = all(np.array_equal(g, ref_cnt) for g in got)
        kmers = int(np.maximum(np.diff(reads.offsets).astype(np.int64) - a.k + 1, 0).sum())
        print(json.dumps({"streams": form, "handles": [hex(x.cuda_stream) for x in streams], "k": a.k, "local": a.local, "reads": reads.n, "ms_per_step": round(el, 4),
                          "Gkmers_s": round(kmers / el / 1e6, 1), "counts_equal": equal}), flush=True)


if __name__ == "__main__":
    main()
