#!/usr/bin/env python3
"""Timing probe of the read-scan kernels on config 2 (HBM-resident reads): error rates, k, tuning knobs.

Usage (GPU box): python scripts/ax_probe.py [--k 21] [--tune key=value ...] [--err 0,0.001,0.005]
Prints one JSON line per case (kernel ms from HIP events, k-mers/s)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (torch first: one HIP runtime per process)
import numpy as np  # noqa: E402

from speq_amd import DeviceIndex, FmIndex, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--k", default="21")
    ap.add_argument("--err", default="0,0.001,0.005")
    ap.add_argument("--tune", action="append", default=[])
    ap.add_argument("--local", action="store_true")
    ap.add_argument("--paired", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", type=int, default=0, help="override the config's variant (group) count")
    ap.add_argument("--qual", default="q40", help="quality profile (speq_amd.synth.QUALITY_PROFILES)")
    ap.add_argument("--stats", action="store_true",
                    help="also run the instrumented twin once: work counters + per-section clock shares")
    a = ap.parse_args()
    c = dict(synth.CONFIGS[a.config])
    if a.variants:
        c["n_variants"] = a.variants
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True, triple_steps=True,
                        gpu_device=0)
    dev = DeviceIndex(idx, 0)
    for kv in a.tune:
        key, val = kv.split("=")
        dev.tune(**{key: int(val)})
    G = c["n_variants"]
    for err in [float(x) for x in a.err.split(",")]:
        reads = synth.make_reads(ref, a.reads, err_rate=err, paired=a.paired)
        if a.qual != "q40":
            reads = synth.apply_quality_profile(reads, a.qual)
        d_seq = torch.from_numpy(reads.seq).cuda()
        d_qual = torch.from_numpy(reads.qual).cuda()
        d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
        lens = np.diff(reads.offsets).astype(np.int64)
        for k in [int(x) for x in a.k.split(",")]:
            kmers = int(np.maximum(lens - k + 1, 0).sum())
            info = dev.prepare(k)
            cnt = torch.zeros(G + 2, dtype=torch.int64, device="cuda")
            w = torch.zeros(G, dtype=torch.float64, device="cuda")
            best = None
            for it in range(a.reps + 1):
                cnt.zero_()
                torch.cuda.synchronize()
                dev.timing(True)
                dev.timing_read()
                dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k, cnt.data_ptr(),
                                w.data_ptr(), local=a.local, paired=a.paired)
                torch.cuda.synchronize()
                ms, n = dev.timing_read()
                if it > 0:
                    best = ms if best is None else min(best, ms)
            rec = {"err": err, "k": k, "ms": round(best, 4), "Gkmers_s": round(kmers / best / 1e6, 1),
                   "kernel": dev.tuning("last_kernel"), "T": int(cnt[0]), "amb": int(cnt[1]),
                   "tune": a.tune, "local": a.local, "qual": a.qual, "table_bytes": info["table_bytes"]}
            if a.stats and rec["kernel"] == 3:
                c0 = cnt.cpu().numpy().copy()
                cnt.zero_()
                w.zero_()
                st = dev.scan_device_stats(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k,
                                           cnt.data_ptr(), w.data_ptr(), local=a.local, paired=a.paired)
                rec["stats_equal"] = bool((cnt.cpu().numpy() == c0).all())
                tot = max(1, st["cyc_total"])
                rec["cycle_share"] = {s_: round(st[f"cyc_{s_}"] / tot, 3) for s_ in ("refill", "lookup", "run", "phase2")}
                rec["work"] = {k_: v for k_, v in st.items() if not k_.startswith("cyc_")}
                rec["cyc"] = {k_: v for k_, v in st.items() if k_.startswith("cyc_")}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
