#!/usr/bin/env python3
"""bench.py — k-mers scanned/sec of the MI355X SPeQ scan path (BASELINE.json `metric`).

One "step" = one pass of the hot path (exact FM-index backward search of every k-mer window + unique-to-one-group
tally) over this rank's batch of synthetic 150-bp reads already resident in HBM, followed by the RCCL
all-reduce of the G+2 counters (N > 1). Default workload = BASELINE config 2 (10 variants x 50 kb, 1M reads per
GPU, k = 21). Weak scaling: every rank scans its own 1M-read shard of the deterministic read stream.

Launch: python bench.py [--gpus 1 --steps K --warmup W]; for N > 1 the driver uses torch.distributed.run.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
OCC_ENTRY_BYTES = 64   # algorithmic bytes per k-mer = k LF steps x 2 occ loads x 64 B


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", type=int, default=2, help="BASELINE.json config number (1-5)")
    p.add_argument("--reads", type=int, default=0, help="override reads per GPU")
    p.add_argument("--k", type=int, default=0, help="override k")
    p.add_argument("--prefix-q", type=int, default=12)
    p.add_argument("--pair-steps", type=int, default=1)
    p.add_argument("--label-table", default="auto", help="auto|0|1 (auto: only for >= 4 M-symbol indexes)")
    p.add_argument("--mode", choices=["global", "local"], default="global")
    p.add_argument("--ilp", type=int, default=0, help="windows per lane (1|2; 0 = the device default)")
    p.add_argument("--gpu-build", type=int, default=1, help="build the index on the GPU (1) or host SA-IS (0)")
    p.add_argument("--triple-steps", type=int, default=1, help="three-symbol occ planes (1) or not (0)")
    p.add_argument("--kmer-table", type=int, default=1,
                   help="k-mer interval table for k <= 31 (1, default) or LF steps for every window (0)")
    p.add_argument("--tune", action="append", default=[],
                   help="extra launch tuning key=value (speq_device_set_tuning), e.g. ilp_kt=2; repeatable")
    p.add_argument("--no-lf-compare", action="store_true",
                   help="skip timing the LF-step kernel beside the k-mer-table kernel")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample duration")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    return p.parse_args()


def main():
    a = parse_args()
    import torch
    import torch.distributed as dist

    from speq_amd import DeviceIndex, FmIndex, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    torch.cuda.set_device(local_rank)
    dev_t = torch.device(f"cuda:{local_rank}")

    c = dict(synth.CONFIGS[a.config])
    k = a.k or c["k"]
    n_reads = a.reads or (c["n_reads"] if a.config <= 3 else c["n_reads"] // 8)
    paired = c["paired"]
    G = c["n_variants"]

    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    t0 = time.time()
    idx = FmIndex.build(ref.records, ref.groups, G, prefix_q=a.prefix_q, pair_steps=bool(a.pair_steps),
                        label_table="auto" if a.label_table == "auto" else bool(int(a.label_table)),
                        threads=16, gpu_device=local_rank if a.gpu_build else None,
                        triple_steps=bool(a.triple_steps))
    build_s = time.time() - t0
    dev = DeviceIndex(idx, local_rank)
    if a.ilp:
        dev.tune(ilp=a.ilp)
    ilp = dev.tuning("ilp")
    dev.tune(kmer_table=a.kmer_table)
    for kv in a.tune:
        key, val = kv.split("=")
        dev.tune(**{key: int(val)})
    ktab = dev.prepare(k)  # per-k index structure (like the .dat cache): built once, outside the timed region
    # the q-mer table level the scan uses (view_for_k in scan_kernels.hip)
    width = 3 if a.triple_steps else (2 if a.pair_steps else 1)
    q_used = next((a.prefix_q - lv for lv in range(3)
                   if a.prefix_q - lv >= 1 and a.prefix_q - lv <= k and (k - a.prefix_q + lv) % width == 0),
                  a.prefix_q)

    # this rank's shard of the deterministic read stream (pairs never split)
    reads = synth.make_reads(ref, n_reads, start_index=rank * n_reads, paired=paired)
    lens = np.diff(reads.offsets).astype(np.int64)
    kmers_per_step = int(np.maximum(lens - k + 1, 0).sum())
    read_bytes = int(reads.offsets[-1])  # bases per step (qualities: as many again)
    d_seq = torch.from_numpy(reads.seq).to(dev_t)
    d_qual = torch.from_numpy(reads.qual).to(dev_t)
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).to(dev_t)
    d_counts = torch.zeros(G + 2, dtype=torch.int64, device=dev_t)
    d_w = torch.zeros(G, dtype=torch.float64, device=dev_t)
    local = a.mode == "local"
    stream = torch.cuda.current_stream(dev_t).cuda_stream

    def step():
        d_counts.zero_()
        if local:
            d_w.zero_()
        dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k, d_counts.data_ptr(),
                        d_w.data_ptr(), paired=paired, local=local, stream=stream)
        if world > 1:
            dist.all_reduce(d_counts)  # one RCCL all-reduce of the G+2 counters over xGMI
            if local:
                dist.all_reduce(d_w)

    def timed_run(steps, warmup):
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dev.timing(True)
        dev.timing_read()  # reset
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kernel_ms, launches = dev.timing_read()
        dev.timing(False)
        el = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item()), kernel_ms, launches

    elapsed, kernel_ms, launches = timed_run(a.steps, a.warmup)
    counts = d_counts.cpu().numpy()
    if ktab["table_bytes"] and dev.tuning("ilp_kt") <= 2 and dev.tuning("kt_pipeline") == 1:
        kernel_name = "k_scan_kt (software-pipelined k-mer-table scan, speq_amd/csrc/scan_kernels.hip)"
    elif ktab["table_bytes"]:
        kernel_name = "k_scan<..., KT = true> (k-mer-table scan, speq_amd/csrc/scan_kernels.hip)"
    else:
        kernel_name = "k_scan<..., KT = false> (LF-step scan, speq_amd/csrc/scan_kernels.hip)"

    # the LF-step kernel on the same reads (the k-mer table replaces its chain of LF steps; results are identical)
    lf = None
    if a.kmer_table and ktab["table_bytes"] and not a.no_lf_compare:
        dev.tune(kmer_table=0)
        lf_el, lf_ms, lf_n = timed_run(a.steps, 1)
        lf_counts = d_counts.cpu().numpy()
        dev.tune(kmer_table=1)
        if not np.array_equal(lf_counts, counts):
            raise RuntimeError("LF-step scan disagrees with the k-mer-table scan")
        lf = {"value": kmers_per_step * world * a.steps / lf_el, "unit": "k-mers/s",
              "avg_kernel_ms": lf_ms / max(1, lf_n),
              "achieved_GBps": kmers_per_step * 2 * k * OCC_ENTRY_BYTES / (lf_ms / 1e3 / max(1, lf_n)) / 1e9,
              "path": "k_scan<..., KT = false>: q-mer table + three-base LF steps + label-run classification per window"}

    total_kmers = kmers_per_step * world * a.steps
    value = total_kmers / elapsed
    avg_kernel_s = (kernel_ms / 1e3) / max(1, launches)
    algo_bytes_per_launch = kmers_per_step * 2 * k * OCC_ENTRY_BYTES
    achieved_gbs = algo_bytes_per_launch / avg_kernel_s / 1e9

    traffic = None
    traffic_src = None
    prof = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(prof):
        try:
            tj = json.load(open(prof))
            lab = int(idx.info().label_table)
            steps = "_tri1" if a.triple_steps else ""
            kt = "_kt1" if ktab["table_bytes"] else ""
            key = (f"cfg{a.config}_k{k}_q{a.prefix_q}_pairs{a.pair_steps}{steps}_lab{lab}_ilp{ilp}"
                   f"_bpc{dev.tuning('blocks_per_cu')}_{a.mode}_reads{n_reads}{kt}")
            if key in tj:
                traffic = tj[key]["hbm_bytes_per_launch"]
                traffic_src = tj[key]["source"]
        except Exception:
            traffic = None

    # PCIe-inclusive rate (not `value`): the same reads from pageable host memory through the pinned-slot pipeline
    # (speq_scan_reads: memcpy into pinned slots, H2D on a copy stream overlapped with k_scan).
    pcie = None
    if not a.no_pcie:
        seq_b, qual_b = reads.seq.tobytes(), reads.qual.tobytes()
        dev.scan(seq_b, qual_b, reads.offsets[:3], k=k, paired=paired, local=local)  # pipeline warm-up
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            r = dev.scan(seq_b, qual_b, reads.offsets, k=k, paired=paired, local=local)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        if r.total != int(counts[0]) and world == 1:
            raise RuntimeError("host-buffer scan disagrees with the HBM-resident scan")
        pcie = {"value": kmers_per_step / best, "unit": "k-mers/s", "per_gpu": True,
                "path": "speq_scan_reads: pageable host arrays -> pinned slots -> H2D (copy stream) || k_scan",
                "host_GB_per_s": 2 * len(seq_b) / best / 1e9}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(ref, reads, k, G, a.cpu_seconds, local, paired, idx)

    if rank == 0:
        out = {
            "metric": "k-mers scanned/sec (whole node) at k=%d, 150 bp reads" % k,
            "value": value,
            "unit": "k-mers/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 references/reads, SURVEY.md §8(d))",
            "config": {
                "workload": f"BASELINE config {a.config}: {c['n_variants']} variants x {c['n_isolates']} isolates x "
                            f"{c['length']} bp, {n_reads} x 150 bp {'pairs' if paired else 'reads'} per GPU, k={k}",
                "k": k, "reads_per_gpu": n_reads, "paired": paired, "mode": a.mode, "prefix_q": a.prefix_q, "prefix_q_used": q_used, "pair_steps": a.pair_steps, "triple_steps": a.triple_steps, "label_table": int(idx.info().label_table), "ilp": ilp,
                "blocks_per_cu": dev.tuning("blocks_per_cu"), "grid_blocks": dev.tuning("grid_blocks"),
                "ilp_kt": dev.tuning("ilp_kt") or (1 if k <= 23 and dev.tuning("kt_compact") else 2),
                "kt_slots": dev.tuning("kt_slots"),
                "kmers_per_step_per_gpu": kmers_per_step, "parallelism": f"dp{world} (reads sharded, index replicated)",
                "index_build_s": round(build_s, 3), "index_builder": "gpu" if a.gpu_build else "host", "fm_text_len": int(idx.info().n),
                "kmer_table": {"on": bool(ktab["table_bytes"]), "distinct_kmers": ktab["distinct_kmers"],
                               "bytes": ktab["table_bytes"], "build_s": round(ktab["build_ms"] / 1e3, 4)},
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                # measured L2->fabric bytes per launch over this run's launch time: the bandwidth the kernel really
                # draws from Infinity Cache + HBM (an upper bound on HBM bytes), against the same 8 TB/s peak
                "traffic_GBps": (traffic / avg_kernel_s / 1e9) if traffic else None,
                "traffic_frac": (traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
                "kernel": kernel_name,
                "algorithmic_bytes_per_kmer": 2 * k * OCC_ENTRY_BYTES,
                "avg_kernel_ms": avg_kernel_s * 1e3, "launches_timed": launches,
                "traffic_source": traffic_src,
                # the table kernel's own bytes: one 64-B bucket per window plus the read bytes (bases + qualities)
                "table_kernel_model": ({"bytes_per_kmer": round(64 + 2 * read_bytes / max(1, kmers_per_step), 3),
                                        "achieved_GBps": kmers_per_step * (64 + 2 * read_bytes / max(1, kmers_per_step))
                                        / avg_kernel_s / 1e9,
                                        "frac": kmers_per_step * (64 + 2 * read_bytes / max(1, kmers_per_step))
                                        / avg_kernel_s / 1e9 / HBM_PEAK_GBS}
                                       if ktab["table_bytes"] else None),
                "note": "achieved uses SURVEY.md 8(d)'s algorithmic 2*k*64 B per k-mer (k LF steps x 2 uncached "
                        "64-B occ loads), fixed whatever the kernel does; the k-mer-table kernel reads one 64-B bucket "
                        "per window instead (the LF-step kernel ~0.3 of the algorithmic gathers), mostly from "
                        "L2/Infinity Cache, so frac > 1 means HBM does not bound this kernel; traffic = measured "
                        "L2->fabric bytes per launch (DESIGN.md 6)",
            },
            "cpu_baseline": cpu,
            "lf_steps": lf,
            "pcie_inclusive": pcie,
            "check": {"T": int(counts[0]), "ambiguous": int(counts[1]), "U": [int(x) for x in counts[2:]]},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(ref, reads, k, G, target_s, local, paired=False, idx=None):
    """CPU baselines on this host's cores over a bounded sample of the same reads (rank 0, N = 1 only).

    value: oracle/seqan_like.c — the reference's ALGORITHM restated (backward search on a wavelet structure, locate of
    every hit through SA samples every 16 rows, sorted hit lists, first-hit rule), the SURVEY.md 8(d) stand-in for
    the SeqAn3 binary, which cannot be built here (8(c)). "hash_port" beside it: oracle/kmer_oracle.c, a hash-map
    restatement of the same semantics (no FM-index, no locate) — an upper bound for any CPU port."""
    from oracle.oracle import Oracle, SeqanLike
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    t0 = time.perf_counter()
    sl = SeqanLike(ref.records, ref.groups, G)
    sl_build = time.perf_counter() - t0
    orc = Oracle(ref.records, ref.groups, G, k)
    units = reads.n // 2 if paired else reads.n

    def timed(fn, target):
        def run(nu, reps=1):
            nr = 2 * nu if paired else nu
            b = int(reads.offsets[nr])
            t0 = time.perf_counter()
            for _ in range(reps):
                fn(reads.seq[:b], reads.qual[:b], reads.offsets[:nr + 1])
            return time.perf_counter() - t0

        n = min(units, 2_000)
        t = run(n)
        while t < target / 2 and n < units:  # grow the sample first, repeat passes only over the whole shard
            n = int(min(units, n * min(8.0, 1.2 * target / max(t, 1e-3))))
            t = run(n)
        reps = 1
        if t < target / 2:
            reps = max(1, int(target / max(t, 1e-3)))
            t = run(n, reps)
        nr = 2 * n if paired else n
        lens = np.diff(reads.offsets[:nr + 1]).astype(np.int64)
        km = int(np.maximum(lens - k + 1, 0).sum()) * reps
        return km / t, n, reps, km, t

    v, n, reps, km, t = timed(lambda s, q, o: sl.scan(s, q, o, k=k, paired=paired, local=local, threads=threads),
                              target_s)
    hv, hn, hreps, hkm, ht = timed(lambda s, q, o: orc.scan(s, q, o, paired=paired, local=local, threads=threads),
                                   target_s / 3)
    lr = None
    if idx is not None and k <= 32 and not local:  # the build's own algorithm on CPU cores (oracle/fm_cpu.c), global mode
        from oracle.oracle import FmCpu
        fc = FmCpu(idx)
        lv, ln, lreps, lkm, lt = timed(lambda s, q, o: fc.scan(s, q, o, k=k, paired=paired, threads=threads),
                                       target_s / 3)
        lr = {"value": lv, "unit": "k-mers/s", "cores": threads,
              "sample": f"first {ln} x {lreps} passes ({lkm} k-mers, {lt:.1f} s), oracle/fm_cpu.c (this build's "
                        f"label-run FM-index search on host cores, same index arrays as the GPU)"}
    unit = "pairs" if paired else "reads"
    return {"value": v, "unit": "k-mers/s", "cores": threads, "kind": "port",
            "sample": f"first {n} {unit} of the same workload x {reps} passes ({km} k-mers, {t:.1f} s) through "
                      f"oracle/seqan_like.c: the reference algorithm (wavelet backward search + SA-sample-16 locate "
                      f"of every hit + sorted hit list + first-hit rule; index build {sl_build:.1f} s not timed); "
                      f"the SeqAn3 binary cannot be built here (SURVEY.md 8(c))",
            "cpu_model": cpu_model(),
            "label_run_port": lr,
            "hash_port": {"value": hv, "unit": "k-mers/s", "cores": threads,
                          "sample": f"first {hn} {unit} x {hreps} passes ({hkm} k-mers, {ht:.1f} s), "
                                    f"oracle/kmer_oracle.c (hash map k-mer -> group label: no FM-index, no locate)"}}


if __name__ == "__main__":
    main()
