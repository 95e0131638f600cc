#!/usr/bin/env python3
"""Streaming / PCIe-inclusive throughput of the scan (SURVEY 8(d) secondary metrics).

  host  : speq_scan_reads on pageable host arrays (memcpy into pinned slots -> H2D on a copy stream -> k_scan)
  fastq : speq_scan_fastq on a FASTQ file in the page cache (reader thread -> parser threads -> pinned slots)
  gz    : the same on a gzip file (zlib inflate on the reader thread)
Prints one JSON line per measurement (and appends them to --out)."""
import argparse
import gzip
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--gz", type=int, default=1)
    ap.add_argument("--split", default="1,0", help="SPEQ_SPLIT_CUT values for the plain-file runs")
    ap.add_argument("--paired", type=int, default=1, help="also time two-file paired streaming")
    ap.add_argument("--lanes", default="", help="stream_lanes values to sweep (default: the device default)")
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process: torch first)
    from speq_amd import DeviceIndex, FmIndex, synth

    c = synth.CONFIGS[a.config]
    k = c["k"]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=11))
    reads = synth.make_reads(ref, a.reads, paired=c["paired"])
    lens = np.diff(reads.offsets).astype(np.int64)
    kmers = int(np.maximum(lens - k + 1, 0).sum())
    out = open(a.out, "a") if a.out else None

    def emit(d):
        d.update({"config": a.config, "reads": reads.n, "kmers": kmers})
        line = json.dumps(d)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
            out.flush()

    seq, qual = reads.seq.tobytes(), reads.qual.tobytes()
    dev.scan(seq, qual, reads.offsets[:1001], k=k)  # warm-up
    for _ in range(3):
        t0 = time.perf_counter()
        r = dev.scan(seq, qual, reads.offsets, k=k, paired=c["paired"])
        dt = time.perf_counter() - t0
    emit({"path": "host (speq_scan_reads, pageable arrays)", "seconds": dt, "kmers_per_s": kmers / dt,
          "GB_per_s_host": 2 * len(seq) / dt / 1e9, "T": r.total})

    path = os.path.join(a.dir, "speq_stream_bench.fq")
    t0 = time.perf_counter()
    with open(path, "wb") as f:
        for i in range(0, reads.n, 100_000):
            parts = []
            for j in range(i, min(reads.n, i + 100_000)):
                s0, s1 = int(reads.offsets[j]), int(reads.offsets[j + 1])
                parts.append(b"@r%d\n%s\n+\n%s\n" % (j, seq[s0:s1], qual[s0:s1]))
            f.write(b"".join(parts))
    size = os.path.getsize(path)
    print(f"# wrote {size / 1e6:.0f} MB FASTQ in {time.perf_counter() - t0:.1f} s", flush=True)
    lane_opts = [int(x) for x in a.lanes.split(",")] if a.lanes else [dev.tuning("stream_lanes")]
    for split_cut, lanes in [(sc, ln) for sc in a.split.split(",") for ln in lane_opts]:
        os.environ["SPEQ_SPLIT_CUT"] = split_cut
        dev.tune(stream_lanes=lanes)
        for th in [int(x) for x in a.threads.split(",")]:
            best = None
            for _ in range(3):
                r2, st = dev.scan_fastq(path, None, k=k, threads=th)
                best = st if best is None or st["seconds"] < best["seconds"] else best
            assert r2.total == r.total and r2.unique.tolist() == r.unique.tolist()
            emit({"path": "fastq (speq_scan_fastq, plain, page cache)", "threads": th,
                  "cut": "parallel" if split_cut != "0" else "sequential", "stream_lanes": lanes, "seconds": best["seconds"],
                  "kmers_per_s": kmers / best["seconds"], "MB_per_s_file": size / best["seconds"] / 1e6,
                  "batches": best["batches"]})
    os.environ.pop("SPEQ_SPLIT_CUT", None)
    if a.paired:  # the same reads as mate pairs in two files (150 + 150 bp), k-mers of both mates
        preads = synth.make_reads(ref, 2 * (a.reads // 2), paired=True)
        plens = np.diff(preads.offsets).astype(np.int64)
        pk = int(np.maximum(plens - k + 1, 0).sum())
        pseq, pqual = preads.seq.tobytes(), preads.qual.tobytes()
        rp = dev.scan(pseq, pqual, preads.offsets, k=k, paired=True)
        paths = [path + ".1", path + ".2"]
        for m, pp in enumerate(paths):
            with open(pp, "wb") as f:
                parts = []
                for j in range(m, preads.n, 2):
                    s0, s1 = int(preads.offsets[j]), int(preads.offsets[j + 1])
                    parts.append(b"@r%d/%d\n%s\n+\n%s\n" % (j // 2, m + 1, pseq[s0:s1], pqual[s0:s1]))
                f.write(b"".join(parts))
        psize = sum(os.path.getsize(pp) for pp in paths)
        th = max(int(x) for x in a.threads.split(","))
        for split_cut in a.split.split(","):
            os.environ["SPEQ_SPLIT_CUT"] = split_cut
            best = None
            for _ in range(3):
                r5, st = dev.scan_fastq(paths[0], paths[1], k=k, threads=th)
                best = st if best is None or st["seconds"] < best["seconds"] else best
            assert r5.total == rp.total and r5.unique.tolist() == rp.unique.tolist()
            d = {"path": "fastq paired (speq_scan_fastq, two plain files, page cache)", "threads": th,
                 "cut": "parallel" if split_cut != "0" else "sequential", "seconds": best["seconds"],
                 "kmers_per_s": pk / best["seconds"], "MB_per_s_file": psize / best["seconds"] / 1e6,
                 "batches": best["batches"]}
            d.update({"config": a.config, "reads": preads.n, "kmers": pk})
            print(json.dumps(d), flush=True)
            if out:
                out.write(json.dumps(d) + "\n")
                out.flush()
        os.environ.pop("SPEQ_SPLIT_CUT", None)
        for pp in paths:
            os.remove(pp)
    if a.gz:
        gpath = path + ".gz"
        with open(path, "rb") as f, gzip.open(gpath, "wb", compresslevel=1) as g:
            while True:
                b = f.read(64 << 20)
                if not b:
                    break
                g.write(b)
        th = max(int(x) for x in a.threads.split(","))
        r3, st = dev.scan_fastq(gpath, None, k=k, threads=th)
        assert r3.total == r.total
        emit({"path": "fastq.gz (speq_scan_fastq, zlib level 1)", "threads": th, "seconds": st["seconds"],
              "kmers_per_s": kmers / st["seconds"], "MB_per_s_file": size / st["seconds"] / 1e6,
              "gz_bytes": os.path.getsize(gpath)})
        os.remove(gpath)
        # BGZF (bgzip's blocked gzip): members inflated in parallel
        import struct
        import zlib
        bpath = path + ".bgz"
        with open(path, "rb") as f, open(bpath, "wb") as g:
            while True:
                chunk = f.read(65280)
                if not chunk:
                    break
                co = zlib.compressobj(1, zlib.DEFLATED, -15)
                comp = co.compress(chunk) + co.flush()
                g.write(struct.pack("<BBBBIBBHBBHH", 0x1f, 0x8b, 8, 4, 0, 0, 0xff, 6, 66, 67, 2, 18 + len(comp) + 7))
                g.write(comp + struct.pack("<II", zlib.crc32(chunk) & 0xffffffff, len(chunk)))
            g.write(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
        for th in sorted({4, max(int(x) for x in a.threads.split(","))}):
            best = None
            for _ in range(2):
                r4, st = dev.scan_fastq(bpath, None, k=k, threads=th)
                best = st if best is None or st["seconds"] < best["seconds"] else best
            assert r4.total == r.total
            emit({"path": "fastq BGZF (speq_scan_fastq, parallel member inflate, zlib level 1)", "threads": th,
                  "seconds": best["seconds"], "kmers_per_s": kmers / best["seconds"],
                  "MB_per_s_file": size / best["seconds"] / 1e6, "bgzf_bytes": os.path.getsize(bpath)})
        os.remove(bpath)
    os.remove(path)


if __name__ == "__main__":
    main()
