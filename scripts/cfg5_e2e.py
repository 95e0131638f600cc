#!/usr/bin/env python3
"""Config-5 scale check on one GPU (200 variants x 5 isolates x 100 kb, paired 2 x 150 bp, k = 31): GPU index build,
the .dat reference pass, an HBM-resident paired scan, an EM scan + finalize + iterations. One JSON line per stage."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2_000_000)
    a = ap.parse_args()
    import torch
    from speq_amd import DeviceIndex, EmHistogram, FmIndex, em_refine, synth, unique_to_percent
    c = synth.CONFIGS[5]
    k, G = c["k"], c["n_variants"]

    def emit(**d):
        print(json.dumps(d), flush=True)

    t0 = time.perf_counter()
    ref = synth.make_reference(G, c["n_isolates"], c["length"])
    emit(stage="synth_reference", seconds=time.perf_counter() - t0)
    t0 = time.perf_counter()
    idx = FmIndex.build(ref.records, ref.groups, G, prefix_q=12, pair_steps=True, triple_steps=True, label_table="auto",
                        gpu_device=0)
    info = idx.info()
    emit(stage="gpu_index_build", seconds=time.perf_counter() - t0, n=info.n, n_runs=info.n_runs,
         device_gb=info.device_bytes / 1e9, label_table=info.label_table)
    dev = DeviceIndex(idx)
    emit(stage="device_tuning", ilp=dev.tuning("ilp"), blocks_per_cu=dev.tuning("blocks_per_cu"))
    t0 = time.perf_counter()
    u_ref, t_ref = dev.count_unique_kmers_per_group(k)
    dt = time.perf_counter() - t0
    emit(stage="dat_pass", seconds=dt, windows=int(t_ref.sum()), windows_per_s=float(t_ref.sum()) / dt)

    t0 = time.perf_counter()
    reads = synth.make_reads(ref, a.pairs, paired=True)
    emit(stage="synth_reads", seconds=time.perf_counter() - t0, records=reads.n)
    lens = np.diff(reads.offsets).astype(np.int64)
    kmers = int(np.maximum(lens - k + 1, 0).sum())
    dv = torch.device("cuda:0")
    d_seq = torch.from_numpy(reads.seq).to(dv)
    d_qual = torch.from_numpy(reads.qual).to(dv)
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).to(dv)
    d_counts = torch.zeros(G + 2, dtype=torch.int64, device=dv)
    st = torch.cuda.current_stream().cuda_stream
    for ilp in (1, 2):
        dev.tune(ilp=ilp)
        times = []
        for _ in range(4):
            d_counts.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k, d_counts.data_ptr(),
                            paired=True, stream=st)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        best = min(times[1:])
        emit(stage="paired_scan_hbm", ilp=ilp, seconds=best, kmers=kmers, kmers_per_s=kmers / best,
             T=int(d_counts[0]), ambiguous=int(d_counts[1]))
    dev.tune(ilp=1)
    counts = d_counts.cpu().numpy()
    del d_seq, d_qual, d_off

    em = EmHistogram(dev)
    t0 = time.perf_counter()
    r = em.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, paired=True)
    emit(stage="em_scan_host_buffers", seconds=time.perf_counter() - t0, counts_match=bool(r.total == counts[0]))
    t0 = time.perf_counter()
    em.finalize(threads=16)
    n_int, n_ent, n_win = em.info()
    emit(stage="em_finalize", seconds=time.perf_counter() - t0, intervals=n_int, entries=n_ent, windows=n_win)
    ut = r.unique / (0.99 ** k)
    p0 = unique_to_percent(ut, r.total, u_ref, t_ref)
    t0 = time.perf_counter()
    traj = em_refine(lambda p: em.step(p, [c["n_isolates"]] * G, r.unique), ut, r.total, p0, max_iterations=200)
    dt = time.perf_counter() - t0
    emit(stage="em_iterations", iterations=len(traj), seconds=dt, seconds_per_iteration=dt / max(1, len(traj)))


if __name__ == "__main__":
    main()
