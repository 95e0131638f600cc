#!/usr/bin/env python3
"""Kernel-time sweep over index/scan parameters in ONE process (interleaved A/B, cdna_hip_programming.md rule 24).

Prints one JSON line per (config, k, prefix_q, mode) with the median kernel time and k-mers/s.
Usage: python scripts/sweep.py [--configs 2,3] [--reads 1000000] [--qs 0,8,10,12] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3")
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--qs", default="0,8,10,12")
    ap.add_argument("--modes", default="global,local")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--ref-pass", action="store_true")
    ap.add_argument("--bpc", default="auto", help="blocks-per-CU caps to sweep (0 = none; auto = device default)")
    ap.add_argument("--grids", default="auto", help="grid caps to sweep (auto = device default)")
    ap.add_argument("--pairs", default="0,1", help="multi-symbol steps to sweep: 0 single, 1 pairs, 2 pairs + triples")
    ap.add_argument("--labs", default="1", help="label_table values to sweep")
    ap.add_argument("--ilps", default="auto", help="windows per lane to sweep (1, 2; auto = device default)")
    ap.add_argument("--k", type=int, default=0, help="override the config's k")
    ap.add_argument("--sparse", default="-1", help="sparse q-mer table choices (-1 auto, 0 dense, 1 sparse)")
    a = ap.parse_args()
    import torch

    from speq_amd import DeviceIndex, FmIndex, synth
    dev_t = torch.device("cuda:0")
    for cfg in [int(x) for x in a.configs.split(",")]:
        c = synth.CONFIGS[cfg]
        G, k = c["n_variants"], (a.k or c["k"])
        ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
        reads = synth.make_reads(ref, a.reads, paired=c["paired"])
        lens = np.diff(reads.offsets).astype(np.int64)
        kmers = int(np.maximum(lens - k + 1, 0).sum())
        d_seq = torch.from_numpy(reads.seq).to(dev_t)
        d_qual = torch.from_numpy(reads.qual).to(dev_t)
        d_off = torch.from_numpy(reads.offsets.astype(np.int64)).to(dev_t)
        d_counts = torch.zeros(G + 2, dtype=torch.int64, device=dev_t)
        d_w = torch.zeros(G, dtype=torch.float64, device=dev_t)
        stream = torch.cuda.current_stream().cuda_stream
        devs = {}
        for q in [int(x) for x in a.qs.split(",")]:
            for pr in [int(x) for x in a.pairs.split(",")]:
                for lb in [int(x) for x in a.labs.split(",")]:
                    t0 = time.time()
                    idx = FmIndex.build(ref.records, ref.groups, G, prefix_q=q, pair_steps=pr >= 1,
                                        label_table=bool(lb), triple_steps=pr == 2, gpu_device=0)
                    info = idx.info()
                    devs[(q, pr, lb)] = (DeviceIndex(idx), time.time() - t0, info)
        def vals(arg):
            return [-1] if arg == "auto" else [int(x) for x in arg.split(",")]
        times = {(q, m, b, g, il, sp): [] for q in devs for m in a.modes.split(",")
                 for b in vals(a.bpc) for g in vals(a.grids) for il in vals(a.ilps)
                 for sp in [int(x) for x in a.sparse.split(",")]}
        defaults = {q: (d.tuning("blocks_per_cu"), d.tuning("grid_blocks"), d.tuning("ilp"), d.tuning("ilp_local"))
                    for q, (d, _, _) in devs.items()}
        checks = {}
        for r in range(a.rounds):
            for (q, m, b, g, il, sp) in times:
                dev = devs[q][0]
                dev.tune(sparse_prefix=sp)
                db, dg, di, dl = defaults[q]
                dev.tune(blocks_per_cu=db if b < 0 else b, grid_blocks=dg if g < 0 else g,
                         ilp=(dl if m == "local" else di) if il < 0 else il,
                         ilp_local=dl if il < 0 else il)
                d_counts.zero_()
                d_w.zero_()
                dev.timing(True)
                dev.timing_read()
                dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k,
                                d_counts.data_ptr(), d_w.data_ptr(), paired=c["paired"], local=(m == "local"),
                                stream=stream)
                torch.cuda.synchronize()
                ms, n = dev.timing_read()
                times[(q, m, b, g, il, sp)].append(ms)
                checks[(q, m, b, g, il, sp)] = d_counts.cpu().numpy().tolist()
        ref_check = None
        for (q, m, b, g, il, sp), ts in times.items():
            med = statistics.median(ts)
            if ref_check is None:
                ref_check = checks[(q, m, b, g, il, sp)]
            db, dg, di, dl = defaults[q]
            out = {"config": cfg, "k": k, "reads": reads.n, "prefix_q": q[0], "pairs": q[1], "lab": q[2], "mode": m,
                   "blocks_per_cu": db if b < 0 else b, "grid_blocks": dg if g < 0 else g,
                   "ilp": ((dl if m == "local" else di) if il < 0 else il), "kernel_ms_median": med,
                   "kernel_ms_min": min(ts), "kmers_per_s": kmers / (med / 1e3),
                   "algo_GBps": kmers * 2 * k * 64 / (med / 1e3) / 1e9,
                   "index_build_s": round(devs[q][1], 3), "n": int(devs[q][2].n), "n_runs": int(devs[q][2].n_runs),
                   "device_MB": devs[q][2].device_bytes / 1e6, "counts_match_first": checks[(q, m, b, g, il, sp)] == ref_check, "sparse_prefix": sp}
            print(json.dumps(out), flush=True)
        if a.ref_pass:
            for q, (dev, _, info) in devs.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                u, t = dev.count_unique_kmers_per_group(k)
                el = time.perf_counter() - t0
                print(json.dumps({"config": cfg, "ref_pass": True, "prefix_q": q[0], "pairs": q[1], "lab": q[2], "seconds": el,
                                  "windows": int(t.sum()), "windows_per_s": int(t.sum()) / el}), flush=True)


if __name__ == "__main__":
    main()
