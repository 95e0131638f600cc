#!/usr/bin/env python3
"""bench.py — k-mers scanned/sec of the MI355X SPeQ scan path (BASELINE.json `metric`).

One "step" = one pass of the hot path (exact search of every k-mer window + unique-to-one-group tally) over this
rank's batch of synthetic 150-bp reads already resident in HBM, followed by the RCCL all-reduce of the G+2
counters (N > 1). Default workload = BASELINE config 2 (10 variants x 50 kb, 1M reads per GPU, k = 21, global
mode) -> `value`. The same run also measures, as secondary lines in the same JSON object:
  * "local_mode": config 2 in the reference's default Phred-weighted mode (fixed_accuracy 0, arg_parse.h:23);
  * "k31": BASELINE config 3 (50 variants x 3 isolates, k = 31) at its full 10 M reads per GPU — at N = 8 the
    per-rank shard of config 4 (100 M reads over 8 GPUs, 12.5 M each);
  * "k70_reference_defaults": config 2's reads at the reference CLI's defaults (k = 70, Phred-weighted);
  * "local_varq" (N = 1): config 2, Phred-weighted, with Illumina-like per-base qualities (synth "variable");
  * "cfg5_paired" / "cfg5_paired_local": BASELINE config 5's index (200 variants x 5 isolates), paired 2 x 150 bp,
    k = 31, on a per-GPU sample of the config's pairs (--cfg5-pairs);
  * "fastq_e2e" (N = 1): the drop-in input path, speq_scan_fastq on config 2's reads written as a FASTQ file on
    local disk (file bytes/s and k-mers/s, page cache warm).
Weak scaling: every rank scans its own shard of the deterministic read stream.

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
    p.add_argument("--config", type=int, default=2, help="BASELINE.json config number (1-5) of the headline")
    p.add_argument("--reads", type=int, default=0, help="override reads per GPU")
    p.add_argument("--k", type=int, default=0, help="override k")
    p.add_argument("--prefix-q", type=int, default=12)
    p.add_argument("--pair-steps", type=int, default=1)
    p.add_argument("--label-table", default="auto", help="auto|0|1 (auto: only for >= 4 M-symbol indexes)")
    p.add_argument("--mode", choices=["global", "local"], default="global")
    p.add_argument("--qual", default="q40", help="quality profile of the headline reads (speq_amd.synth.QUALITY_PROFILES)")
    p.add_argument("--ilp", type=int, default=0, help="windows per lane of the LF-step kernel (1|2; 0 = default)")
    p.add_argument("--gpu-build", type=int, default=1, help="build the index on the GPU (1) or host SA-IS (0)")
    p.add_argument("--triple-steps", type=int, default=1, help="three-symbol occ planes (1) or not (0)")
    p.add_argument("--kmer-table", type=int, default=1,
                   help="per-k interval table (1, default) or LF steps for every window (0)")
    p.add_argument("--tune", action="append", default=[],
                   help="extra launch tuning key=value (speq_device_set_tuning), e.g. ilp_kt=2; repeatable")
    p.add_argument("--no-lf-compare", action="store_true",
                   help="skip timing the LF-step kernel beside the table kernel")
    p.add_argument("--no-extra", action="store_true", help="skip the local-mode and k=31 secondary lines")
    p.add_argument("--k31-reads", type=int, default=0, help="reads per GPU of the k=31 line (0 = config 3/4)")
    p.add_argument("--cfg5-pairs", type=int, default=4_000_000, help="pairs per GPU of the config-5 lines (0: skip)")
    p.add_argument("--no-fastq", action="store_true", help="skip the FASTQ end-to-end line")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample duration")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    return p.parse_args()


def host_cpu_info() -> dict:
    """The CPUs this process may use: affinity mask, machine count and the cgroup CPU quota (the GPU box gives
    each job a share of a larger machine: its nproc shows every CPU, the quota says how many it may keep busy)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return {"threads": threads, "affinity_cpus": aff, "nproc": os.cpu_count(), "cgroup_cpu_quota": quota,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "cpu_model": cpu_model(),
            "rule": "threads = min(affinity CPUs, cgroup CPU quota) (all CPUs this job may keep busy)"}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class Ctx:
    def __init__(self, a):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.a = torch, dist, a
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world > 1:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{self.local_rank}"))
        torch.cuda.set_device(self.local_rank)
        self.dev_t = torch.device(f"cuda:{self.local_rank}")
        self.comm = None
        if self.world > 1:
            # the product's own collective (C ABI speq_allreduce_*, ncclAllReduce over xGMI): rank 0's 128-byte
            # RCCL id reaches the other ranks through torch.distributed, which keeps only the barrier and timing
            from speq_amd import Comm
            uid = torch.zeros(Comm.ID_BYTES, dtype=torch.uint8, device=self.dev_t)
            if self.rank == 0:
                uid.copy_(torch.frombuffer(bytearray(Comm.unique_id()), dtype=torch.uint8))
            dist.broadcast(uid, 0)
            self.comm = Comm(self.world, self.rank, bytes(uid.cpu().numpy().tobytes()))

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def allreduce_max(self, x: float) -> float:
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.dev_t)
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def ax_request_bytes(st: dict, k: int, n_reads: int, local: bool) -> dict:
    """Bytes k_scan_ax REQUESTS per launch, from the work counters of its instrumented twin (speq_scan_reads_device_stats,
    same scan, same results): every load the kernel issues, by kind, at the size it issues it (ax_scan.hip):
      read offsets 8 B per read; staging 16 B of bases + 16 B of qualities per 16-base chunk;
      anchor buckets 64 B per lookup (phase 1 and phase 2); run granules 16 B each (counted);
      Bloom-filter words 8 B per deferred window; candidate granules ceil(k/32) + 1 x 16 B per phase-2 verification;
      local mode: single quality bytes."""
    hw = (k + 31) // 32
    parts = {
        "offsets": 8.0 * n_reads,
        "staging": 32.0 * st["chunks"],
        "anchor_buckets": 64.0 * (st["lookup_lanes"] + st["p2_probes"]),
        "run_granules": 16.0 * st["run_granules"],
        "filter": 8.0 * st["deferred"],
        "verify_granules": 16.0 * (hw + 1) * st["p2_verify"],
        "quality_bytes": float(st["qual_bytes"]) if local else 0.0,
    }
    return {"total": sum(parts.values()), "parts": parts}


def kernel_model(dev, k: int, table_on: bool, kmers: int, read_bytes: int, n_reads: int = 0) -> dict:
    """The timed kernel and the bytes IT must move per k-mer window (its own roofline model), for the kernels whose
    loads are a fixed function of the workload. k_scan_ax's are counted instead (ax_request_bytes).

    Table path (k_scan_kt): one 64-B table bucket per window + the read bytes (bases + qualities).
    LF-step path (k_scan): SURVEY.md 8(d)'s 2*k*64 B per window (k LF steps x 2 occ loads)."""
    rb = 2.0 * read_bytes / max(1, kmers)
    if dev.tuning("last_kernel") == 3:
        return {"kernel": "k_scan_ax (anchor-and-extend scan, speq_amd/csrc/ax_scan.hip)", "bytes_per_kmer": None,
                "model": "bytes the kernel requests, counted by its instrumented twin (ax_request_bytes)"}
    if table_on:
        return {"kernel": "k_scan_kt (pipelined k-mer-table scan, speq_amd/csrc/scan_kernels.hip)",
                "bytes_per_kmer": 64.0 + rb,
                "model": "one 64-B table bucket per window + the read's bases and qualities"}
    return {"kernel": "k_scan<..., KT = false> (LF-step scan, speq_amd/csrc/scan_kernels.hip)",
            "bytes_per_kmer": float(2 * k * OCC_ENTRY_BYTES),
            "model": "SURVEY.md 8(d): k LF steps x 2 occ-block loads x 64 B"}


def traffic_lookup(cfg: int, k: int, mode: str, n_reads: int, kernel: str, qual_profile: str = "q40") -> dict | None:
    """Measured fabric bytes per launch of this exact workload and kernel (rocprofv3 PMC passes summarised into
    profiles/traffic.json by scripts/summarize_profile.py --traffic-key), or None."""
    prof = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(prof):
        return None
    try:
        tj = json.load(open(prof))
    except ValueError:
        return None
    key = f"cfg{cfg}_k{k}_{mode}_reads{n_reads}_{kernel}" + ("" if qual_profile == "q40" else f"_{qual_profile}")
    if key not in tj:
        return None
    e = dict(tj[key])
    e["source"] = os.path.normpath(os.path.join("profiles", e["source"]))
    return e


KERNEL_TAG = {0: "lf", 1: "kt", 2: "kt", 3: "ax"}  # speq_device_get_tuning("last_kernel")


def run_workload(ctx: Ctx, cfg_no: int, k: int, n_reads: int, mode: str, steps: int, warmup: int,
                 with_lf: bool, with_pcie: bool, with_cpu: bool, cpu_seconds: float, prepared=None,
                 qual_profile: str = "q40") -> dict:
    """Builds the index of BASELINE config `cfg_no` (or reuses `prepared`), stages this rank's reads in HBM, times
    `steps` scans and returns the measurement (plus the objects for reuse). qual_profile: synth.QUALITY_PROFILES
    (the reads of `prepared` are regenerated with it when they differ)."""
    torch, a = ctx.torch, ctx.a
    from speq_amd import DeviceIndex, FmIndex, synth

    c = dict(synth.CONFIGS[cfg_no])
    paired, G = c["paired"], c["n_variants"]
    if prepared is None:
        ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
        t0 = time.time()
        idx = FmIndex.build(ref.records, ref.groups, G, prefix_q=a.prefix_q, pair_steps=bool(a.pair_steps),
                            label_table="auto" if a.label_table == "auto" else bool(int(a.label_table)),
                            threads=16, gpu_device=ctx.local_rank if a.gpu_build else None,
                            triple_steps=bool(a.triple_steps))
        build_s = time.time() - t0
        dev = DeviceIndex(idx, ctx.local_rank)
        if a.ilp:
            dev.tune(ilp=a.ilp)
        dev.tune(kmer_table=a.kmer_table)
        for kv in a.tune:
            key, val = kv.split("=")
            dev.tune(**{key: int(val)})
        prepared = dict(ref=ref, idx=idx, dev=dev, build_s=build_s, qual_profile=None)
    if prepared.get("qual_profile") != qual_profile:
        reads = synth.make_reads(prepared["ref"], n_reads, start_index=ctx.rank * n_reads, paired=paired)
        reads = synth.apply_quality_profile(reads, qual_profile)
        prepared.update(reads=reads, qual_profile=qual_profile, d_seq=torch.from_numpy(reads.seq).to(ctx.dev_t),
                        d_qual=torch.from_numpy(reads.qual).to(ctx.dev_t),
                        d_off=torch.from_numpy(reads.offsets.astype(np.int64)).to(ctx.dev_t))
    ref, idx, dev, reads = prepared["ref"], prepared["idx"], prepared["dev"], prepared["reads"]
    d_seq, d_qual, d_off = prepared["d_seq"], prepared["d_qual"], prepared["d_off"]
    ktab = dev.prepare(k)  # per-k index structure (like the .dat cache): built once, outside the timed region
    lens = np.diff(reads.offsets).astype(np.int64)
    kmers_per_step = int(np.maximum(lens - k + 1, 0).sum())
    read_bytes = int(reads.offsets[-1])
    d_counts = torch.zeros(G + 2, dtype=torch.int64, device=ctx.dev_t)
    d_w = torch.zeros(G, dtype=torch.float64, device=ctx.dev_t)
    local = mode == "local"
    stream = torch.cuda.current_stream(ctx.dev_t).cuda_stream

    def step():
        d_counts.zero_()
        if local:
            d_w.zero_()
        dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k, d_counts.data_ptr(),
                        d_w.data_ptr(), paired=paired, local=local, stream=stream)
        if ctx.comm is not None:  # one RCCL all-reduce of the G+2 counters over xGMI (speq_allreduce_u64)
            ctx.comm.allreduce_u64(d_counts.data_ptr(), G + 2, stream)
            if local:
                ctx.comm.allreduce_f64(d_w.data_ptr(), G, stream)

    def timed_run(n_steps, n_warm):
        for _ in range(n_warm):
            step()
        torch.cuda.synchronize()
        ctx.barrier()
        torch.cuda.synchronize()
        dev.timing(True)
        dev.timing_read()  # reset
        t0 = time.perf_counter()
        for _ in range(n_steps):
            step()
        torch.cuda.synchronize()
        ctx.barrier()
        elapsed = time.perf_counter() - t0
        kernel_ms, launches = dev.timing_read()
        dev.timing(False)
        return ctx.allreduce_max(elapsed), kernel_ms, launches

    elapsed, kernel_ms, launches = timed_run(steps, warmup)
    counts = d_counts.cpu().numpy()
    weights = d_w.cpu().numpy() if local else None
    table_on = bool(ktab["table_bytes"])
    hot_kernel = dev.tuning("last_kernel")
    km = kernel_model(dev, k, table_on, kmers_per_step, read_bytes, reads.n)

    lf = None
    prev = None
    if with_lf and a.kmer_table and table_on and dev.tuning("last_kernel") == 3:
        # the previous hot path (k-mer-table kernel for k <= 31, else LF steps) on the same reads
        dev.tune(ax_scan=0)
        pv_el, pv_ms, pv_n = timed_run(steps, 1)
        pv_counts = d_counts.cpu().numpy()
        kind = dev.tuning("last_kernel")
        dev.tune(ax_scan=1)
        if not np.array_equal(pv_counts, counts):
            raise RuntimeError("k-mer-table scan disagrees with the anchor-and-extend scan")
        prev = {"value": kmers_per_step * ctx.world * steps / pv_el, "unit": "k-mers/s",
                "avg_kernel_ms": pv_ms / max(1, pv_n),
                "path": {0: "k_scan (LF steps)", 1: "k_scan<KT> (k-mer table)",
                         2: "k_scan_kt (pipelined k-mer-table scan, round-1 hot path)"}.get(kind, str(kind))}
    if with_lf and a.kmer_table and table_on:
        dev.tune(kmer_table=0, ax_scan=0)
        lf_el, lf_ms, lf_n = timed_run(steps, 1)
        lf_counts = d_counts.cpu().numpy()
        dev.tune(kmer_table=1, ax_scan=1)
        if not np.array_equal(lf_counts, counts):
            raise RuntimeError("LF-step scan disagrees with the hot path")
        lf = {"value": kmers_per_step * ctx.world * steps / lf_el, "unit": "k-mers/s",
              "avg_kernel_ms": lf_ms / max(1, lf_n),
              "achieved_GBps": kmers_per_step * 2 * k * OCC_ENTRY_BYTES / (lf_ms / 1e3 / max(1, lf_n)) / 1e9,
              "path": "k_scan<..., KT = false>: q-mer table + three-base LF steps + label-run classification"}

    total_kmers = kmers_per_step * ctx.world * steps
    value = total_kmers / elapsed
    avg_kernel_s = (kernel_ms / 1e3) / max(1, launches)
    ax_stats = None
    if hot_kernel == 3 and not os.environ.get("SPEQ_BENCH_NO_STATS"):
        # one untimed launch of the instrumented twin: the same scan (checked equal), plus its work counters
        d_counts.zero_()
        if local:
            d_w.zero_()
        ax_stats = dev.scan_device_stats(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k,
                                         d_counts.data_ptr(), d_w.data_ptr(), paired=paired, local=local)
        if not np.array_equal(d_counts.cpu().numpy(), counts):
            raise RuntimeError("instrumented anchor-and-extend scan disagrees with the timed scan")
        req = ax_request_bytes(ax_stats, k, reads.n, local)
        own_bytes = req["total"]
        km["bytes_per_kmer"] = own_bytes / kmers_per_step
        km["bytes_parts"] = {key: round(v / kmers_per_step, 4) for key, v in req["parts"].items()}
    elif km["bytes_per_kmer"] is not None:
        own_bytes = kmers_per_step * km["bytes_per_kmer"]
    else:  # SPEQ_BENCH_NO_STATS (profiling passes: no instrumented launch among the profiled kernels)
        own_bytes = 0.0
        km["bytes_per_kmer"] = 0.0
    own_gbs = own_bytes / avg_kernel_s / 1e9
    survey_gbs = kmers_per_step * 2 * k * OCC_ENTRY_BYTES / avg_kernel_s / 1e9
    tr = traffic_lookup(cfg_no, k, mode, n_reads, KERNEL_TAG.get(hot_kernel, "lf"), qual_profile)
    traffic = tr["hbm_bytes_per_launch"] if tr else None
    roofline = {
        "bound": "hbm", "achieved": own_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": own_gbs / HBM_PEAK_GBS,
        "traffic": traffic,
        "kernel": km["kernel"], "bytes_per_kmer": round(km["bytes_per_kmer"], 3), "bytes_model": km["model"],
        "bytes_per_kmer_by_kind": km.get("bytes_parts"), "own_bytes_per_launch": own_bytes,
        "avg_kernel_ms": avg_kernel_s * 1e3, "launches_timed": launches,
        # measured L2->fabric bytes per launch (rocprofv3 PMC, profiles/): what the kernel really draws from
        # Infinity Cache + HBM, over this run's launch time, against the same 8 TB/s; split into reads, writes and
        # the register-spill writes (Scratch_Size x lanes) inside them
        "traffic_fetch": tr.get("fetch_bytes_per_launch") if tr else None,
        "traffic_write": tr.get("write_bytes_per_launch") if tr else None,
        "traffic_scratch_write": tr.get("scratch_write_bytes_per_launch") if tr else None,
        "traffic_GBps": (traffic / avg_kernel_s / 1e9) if traffic else None,
        "traffic_frac": (traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
        "useful_traffic_frac": ((traffic - (tr.get("scratch_write_bytes_per_launch") or 0.0)) / avg_kernel_s / 1e9
                                / HBM_PEAK_GBS) if traffic else None,
        "traffic_source": tr["source"] if tr else None,
        "traffic_rocprof_kernel_ns": tr.get("kernel_steady_state_ns_rocprof") if tr else None,
        # SURVEY.md 8(d)'s fixed model (2*k*64 B per k-mer: k uncached LF steps) — not what this kernel moves
        "survey_model_bytes_per_kmer": 2 * k * OCC_ENTRY_BYTES,
        "survey_model_frac": survey_gbs / HBM_PEAK_GBS,
    }
    if ax_stats is not None:
        roofline["ax_work"] = ax_stats

    pcie = None
    if with_pcie:
        seq_b, qual_b = reads.seq.tobytes(), reads.qual.tobytes()
        dev.scan(seq_b, qual_b, reads.offsets[:3], k=k, paired=paired, local=local)  # pipeline warm-up
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            r = dev.scan(seq_b, qual_b, reads.offsets, k=k, paired=paired, local=local)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        if r.total != int(counts[0]) and ctx.world == 1:
            raise RuntimeError("host-buffer scan disagrees with the HBM-resident scan")
        pcie = {"value": kmers_per_step / best, "unit": "k-mers/s", "per_gpu": True,
                "path": "speq_scan_reads: pageable host arrays -> pinned slots -> H2D (copy stream) || scan",
                "host_GB_per_s": 2 * len(seq_b) / best / 1e9}

    cpu = None
    if with_cpu and ctx.rank == 0 and ctx.world == 1:
        cpu = cpu_baseline(ref, reads, k, G, cpu_seconds, local, paired, idx)

    out = {
        "value": value, "ms_per_step": elapsed / steps * 1e3, "k": k, "mode": mode,
        "workload": f"BASELINE config {cfg_no}: {c['n_variants']} variants x {c['n_isolates']} isolates x "
                    f"{c['length']} bp, {n_reads} x 150 bp {'pairs' if paired else 'reads'} per GPU, k={k}, {mode}"
                    + (f", qualities '{qual_profile}' ({synth.QUALITY_PROFILES[qual_profile]})"
                       if qual_profile != "q40" else ""),
        "reads_per_gpu": n_reads, "kmers_per_step_per_gpu": kmers_per_step, "paired": paired,
        "index_build_s": round(prepared["build_s"], 3), "fm_text_len": int(idx.info().n),
        "kmer_table": {"on": table_on, "distinct_kmers": ktab["distinct_kmers"], "bytes": ktab["table_bytes"],
                       "build_s": round(ktab["build_ms"] / 1e3, 4)},
        "roofline": roofline, "cpu_baseline": cpu, "lf_steps": lf, "kmer_table_kernel": prev, "pcie_inclusive": pcie,
        "check": {"T": int(counts[0]), "ambiguous": int(counts[1]), "U": [int(x) for x in counts[2:]],
                  **({"W_sum": float(weights.sum())} if weights is not None else {})},
    }
    return out, prepared


def main():
    a = parse_args()
    ctx = Ctx(a)
    from speq_amd import synth

    c = dict(synth.CONFIGS[a.config])
    k = a.k or c["k"]
    n_reads = a.reads or (c["n_reads"] if a.config <= 3 else c["n_reads"] // 8)
    head, prep = run_workload(ctx, a.config, k, n_reads, a.mode, a.steps, a.warmup, with_lf=not a.no_lf_compare,
                              with_pcie=not a.no_pcie, with_cpu=not a.no_cpu_baseline, cpu_seconds=a.cpu_seconds,
                              qual_profile=a.qual)
    dev = prep["dev"]
    extra = {}
    if not a.no_extra and a.config == 2 and not a.k and not a.reads and a.qual == "q40":
        other = "local" if a.mode == "global" else "global"
        extra[f"{other}_mode"], _ = run_workload(ctx, 2, k, n_reads, other, a.steps, a.warmup, with_lf=False,
                                                 with_pcie=False, with_cpu=False, cpu_seconds=0, prepared=prep)
        n31 = a.k31_reads or (10_000_000 if ctx.world == 1 else synth.CONFIGS[4]["n_reads"] // 8)
        extra["k31"], p31 = run_workload(ctx, 3, 31, n31, "global", max(3, a.steps // 4), max(1, a.warmup // 2),
                                         with_lf=False, with_pcie=False, with_cpu=not a.no_cpu_baseline,
                                         cpu_seconds=a.cpu_seconds)
        extra["k31"]["note"] = ("config 3 (10 M reads on one GPU); with 8 ranks each scans config 4's 12.5 M-read "
                                "shard of the same index")
        p31["dev"].close()
        # the reference CLI's defaults: k = 70 (include/arg_parse.h:21), Phred-weighted local mode (:23)
        extra["k70_reference_defaults"], _ = run_workload(ctx, 2, 70, n_reads, "local", a.steps, a.warmup,
                                                          with_lf=False, with_pcie=False, with_cpu=False,
                                                          cpu_seconds=0, prepared=prep)
        if ctx.world == 1:
            if not a.no_fastq:  # the drop-in input path before the reads are re-generated below
                extra["fastq_e2e"] = fastq_e2e(ctx, prep, k)
            # the reference's default (Phred-weighted) mode on reads whose qualities vary base by base
            extra["local_varq"], _ = run_workload(ctx, 2, k, n_reads, "local", a.steps, a.warmup, with_lf=False,
                                                  with_pcie=False, with_cpu=False, cpu_seconds=0, prepared=prep,
                                                  qual_profile="variable")
        if a.cfg5_pairs:
            # BASELINE config 5 (the north_star's scaling config): paired, k = 31, on a per-GPU sample of its pairs
            extra["cfg5_paired"], p5 = run_workload(ctx, 5, 31, a.cfg5_pairs, "global", max(3, a.steps // 4),
                                                    max(1, a.warmup // 2), with_lf=False, with_pcie=False,
                                                    with_cpu=False, cpu_seconds=0)
            extra["cfg5_paired"]["note"] = (f"config 5 lists 500 M pairs (a node's job); each GPU scans a "
                                            f"{a.cfg5_pairs}-pair shard of the same deterministic pair stream")
            extra["cfg5_paired_local"], _ = run_workload(ctx, 5, 31, a.cfg5_pairs, "local", max(3, a.steps // 4),
                                                         max(1, a.warmup // 2), with_lf=False, with_pcie=False,
                                                         with_cpu=False, cpu_seconds=0, prepared=p5)
            p5["dev"].close()

    if ctx.rank == 0:
        out = {
            "metric": "k-mers scanned/sec (whole node) at k=%d, 150 bp reads" % k,
            "value": head["value"],
            "unit": "k-mers/s",
            "n_gpus": ctx.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 references/reads, SURVEY.md §8(d))",
            "config": {
                "workload": head["workload"],
                "k": k, "reads_per_gpu": n_reads, "paired": head["paired"], "mode": a.mode,
                "prefix_q": a.prefix_q, "pair_steps": a.pair_steps, "triple_steps": a.triple_steps,
                "label_table": int(prep["idx"].info().label_table),
                "blocks_per_cu": dev.tuning("blocks_per_cu"), "grid_blocks": dev.tuning("grid_blocks"),
                "kmers_per_step_per_gpu": head["kmers_per_step_per_gpu"],
                "parallelism": f"dp{ctx.world} (reads sharded, index replicated)",
                "collective": ("speq_allreduce_u64/_f64 (C ABI; RCCL ncclAllReduce of the G + 2 counters per step)"
                               if ctx.comm is not None else "none (one GPU)"),
                "index_build_s": head["index_build_s"], "index_builder": "gpu" if a.gpu_build else "host",
                "fm_text_len": head["fm_text_len"], "kmer_table": head["kmer_table"],
            },
            "roofline": head["roofline"],
            "cpu_baseline": head["cpu_baseline"],
            "lf_steps": head["lf_steps"],
            "kmer_table_kernel": head["kmer_table_kernel"],
            "pcie_inclusive": head["pcie_inclusive"],
            "check": head["check"],
            **extra,
        }
        print(json.dumps(out), flush=True)
    if ctx.comm is not None:
        ctx.comm.close()
    if ctx.world > 1:
        ctx.dist.destroy_process_group()


def write_fastq(path: str, reads) -> int:
    """Writes equal-length reads as four-line FASTQ records (@r<9-digit index>), vectorised; returns the bytes."""
    lens = np.diff(reads.offsets)
    L = int(lens[0]) if len(lens) else 0
    if not len(lens) or np.any(lens != L):
        raise ValueError("write_fastq: equal-length reads only")
    n = len(lens)
    head = np.frombuffer(b"@r", dtype=np.uint8)
    digits = (np.arange(n, dtype=np.int64)[:, None] // (10 ** np.arange(8, -1, -1))[None, :]) % 10 + ord("0")
    rec = np.empty((n, 2 + 9 + 1 + L + 3 + L + 1), dtype=np.uint8)
    rec[:, 0:2] = head
    rec[:, 2:11] = digits.astype(np.uint8)
    rec[:, 11] = ord("\n")
    rec[:, 12:12 + L] = reads.seq.reshape(n, L)
    rec[:, 12 + L:15 + L] = np.frombuffer(b"\n+\n", dtype=np.uint8)
    rec[:, 15 + L:15 + 2 * L] = reads.qual.reshape(n, L)
    rec[:, 15 + 2 * L] = ord("\n")
    rec.tofile(path)
    return rec.size


def fastq_e2e(ctx: Ctx, prep: dict, k: int) -> dict:
    """The drop-in input path (speq_scan_fastq: reader thread + parser threads -> pinned slots -> H2D || scan) on the
    workload's reads written as one FASTQ file on local disk; best of 3 passes with the page cache warm. Checked
    against the HBM-resident scan of the same reads."""
    import tempfile
    reads, dev = prep["reads"], prep["dev"]
    threads = host_cpu_info()["threads"]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        path = os.path.join(td, "reads.fq")
        nbytes = write_fastq(path, reads)
        ref_res = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k)
        best, res = None, None
        for _ in range(3):
            t0 = time.perf_counter()
            res, st = dev.scan_fastq(path, k=k, threads=threads)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        if (res.total, res.ambiguous, res.unique.tolist()) != (ref_res.total, ref_res.ambiguous,
                                                              ref_res.unique.tolist()):
            raise RuntimeError("FASTQ scan disagrees with the in-memory scan")
    lens = np.diff(reads.offsets).astype(np.int64)
    kmers = int(np.maximum(lens - k + 1, 0).sum())
    return {"value": kmers / best, "unit": "k-mers/s", "file_GB_per_s": nbytes / best / 1e9, "seconds": best,
            "file_bytes": nbytes, "threads": threads, "k": k,
            "path": "speq_scan_fastq: plain FASTQ on local disk (page cache warm), parallel record-aligned cut, "
                    "raw text to pinned slots -> H2D (copy stream) || GPU record parsing + k_scan_ax",
            "workload": f"{reads.n} x 150 bp reads of BASELINE config 2, global mode"}


def cpu_baseline(ref, reads, k, G, target_s, local, paired=False, idx=None):
    """CPU baselines on this host's cores over a bounded sample of the same reads (rank 0, N = 1 only).

    value: oracle/seqan_like.c — the reference's ALGORITHM restated (backward search on a wavelet structure, locate of
    every hit through SA samples every 16 rows, sorted hit lists, first-hit rule), the SURVEY.md 8(d) stand-in for
    the SeqAn3 binary, which cannot be built here (8(c)). "hash_port" beside it: oracle/kmer_oracle.c, a hash-map
    restatement of the same semantics (no FM-index, no locate) — an upper bound for any CPU port."""
    from oracle.oracle import Oracle, SeqanLike
    hw = host_cpu_info()
    threads = hw["threads"]
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
    if idx is not None and k <= 32 and not local:  # the build's own algorithm on CPU cores (oracle/fm_cpu.c)
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
            "host": hw,
            "label_run_port": lr,
            "hash_port": {"value": hv, "unit": "k-mers/s", "cores": threads,
                          "sample": f"first {hn} {unit} x {hreps} passes ({hkm} k-mers, {ht:.1f} s), "
                                    f"oracle/kmer_oracle.c (hash map k-mer -> group label: no FM-index, no locate)"}}


if __name__ == "__main__":
    main()
