#!/usr/bin/env python3
"""Interleaved A/B of runtime tuning variants on HBM-resident reads (GPU box), one process: every case builds its
index and reads once, then the variants take turns (`--rounds` times, 5 timed launches each, minimum kept), so box
drift falls on every variant alike. Counts must agree across variants.

Usage: python scripts/ab_tune.py --variants "base:;l50:ax_load=50" --cases "2:21:0.001:s:g,3:31:0.001:s:g"
  case = config:k:err:s|p (single-end / paired):g|l (global / local)[:reads]
Prints one JSON line per case: {case, variants: {name: {ms, Gkmers_s}}, counts_equal}."""
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
    ap.add_argument("--variants", required=True, help="name:key=v,key=v;name2:...")
    ap.add_argument("--cases", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    variants = []
    for v in a.variants.split(";"):
        name, _, kv = v.partition(":")
        variants.append((name, dict((x.split("=")[0], int(x.split("=")[1])) for x in kv.split(",") if x)))
    built = {}
    for case in a.cases.split(","):
        f = case.split(":")
        cfg, k, err, paired, local = int(f[0]), int(f[1]), float(f[2]), f[3] == "p", f[4] == "l"
        c = dict(synth.CONFIGS[cfg])
        n = int(f[5]) if len(f) > 5 else (c["n_reads"] if cfg <= 3 else 4_000_000)
        if cfg not in built:
            ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
            idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True,
                                triple_steps=True, gpu_device=0)
            built = {cfg: (ref, idx, DeviceIndex(idx, 0))}
        ref, idx, dev = built[cfg]
        G = c["n_variants"]
        reads = synth.make_reads(ref, n, err_rate=err, paired=paired)
        d_seq = torch.from_numpy(reads.seq).cuda()
        d_qual = torch.from_numpy(reads.qual).cuda()
        d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
        kmers = int(np.maximum(np.diff(reads.offsets).astype(np.int64) - k + 1, 0).sum())
        dev.prepare(k)
        cnt = torch.zeros(G + 2, dtype=torch.int64, device="cuda")
        w = torch.zeros(G, dtype=torch.float64, device="cuda")
        best, counts = {}, {}
        for _ in range(a.rounds):
            for name, tune in variants:
                defaults = {key: dev.tuning(key) for key in tune}
                dev.tune(**tune)
                for it in range(a.reps + 1):
                    cnt.zero_()
                    w.zero_()
                    torch.cuda.synchronize()
                    dev.timing(True)
                    dev.timing_read()
                    dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k, cnt.data_ptr(),
                                    w.data_ptr(), local=local, paired=paired)
                    torch.cuda.synchronize()
                    ms, _ = dev.timing_read()
                    if it > 0:
                        best[name] = min(best.get(name, 1e9), ms)
                counts[name] = (cnt.cpu().numpy().tolist(), float(w.sum().item()))
                dev.tune(**defaults)
        ref_counts = counts[variants[0][0]]
        eq = all(cv[0] == ref_counts[0] and abs(cv[1] - ref_counts[1]) <= 1e-9 * max(1.0, abs(ref_counts[1]))
                 for cv in counts.values())
        print(json.dumps({"case": case, "reads": n, "counts_equal": eq,
                          "variants": {nm: {"ms": round(best[nm], 4), "Gkmers_s": round(kmers / best[nm] / 1e6, 1)}
                                       for nm, _ in variants}}), flush=True)
        if not eq:
            print(json.dumps({"case": case, "counts": counts}), flush=True)
            sys.exit(3)


if __name__ == "__main__":
    main()
