#!/usr/bin/env python3
"""Host-buffer scan (speq_scan_reads: host arrays -> packed pinned slots -> H2D || unpack + scan) on config 2's
reads under different pipeline knobs (GPU box). Prints one JSON line per setting (best of 4)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from speq_amd import DeviceIndex, FmIndex, synth  # noqa: E402

SETTINGS = [dict(), dict(SPEQ_HOST_PACK="1"), dict(SPEQ_HOST_PACK="0"),
            dict(SPEQ_HOST_FILLERS="16", SPEQ_HOST_SLOTS="16"), dict(SPEQ_HOST_BATCH_MB="4"),
            dict(SPEQ_HOST_FILLERS="16", SPEQ_HOST_SLOTS="12", SPEQ_HOST_BATCH_MB="6"),
            dict(SPEQ_HOST_FILLERS="8", SPEQ_HOST_SLOTS="12", SPEQ_HOST_BATCH_MB="8"),
            dict(SPEQ_HOST_FILLERS="12", SPEQ_HOST_SLOTS="20", SPEQ_HOST_BATCH_MB="8")]


def main():
    c = synth.CONFIGS[2]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True, triple_steps=True,
                        gpu_device=0)
    dev = DeviceIndex(idx, 0)
    reads = synth.make_reads(ref, c["n_reads"])
    seq_b, qual_b = reads.seq.tobytes(), reads.qual.tobytes()
    kmers = int(np.maximum(np.diff(reads.offsets).astype(np.int64) - 20, 0).sum())
    keys = sorted({k for s in SETTINGS for k in s})
    for st in SETTINGS:
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(st)
        dev.scan(seq_b, qual_b, reads.offsets[:3], k=21)  # pipeline warm-up
        best, r = None, None
        for _ in range(4):
            t0 = time.perf_counter()
            r = dev.scan(seq_b, qual_b, reads.offsets, k=21)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        print(json.dumps({"env": st, "ms": round(best * 1e3, 3), "Gkmers_s": round(kmers / best / 1e9, 2),
                          "host_GB_s": round(2 * len(seq_b) / best / 1e9, 1), "T": r.total}), flush=True)


if __name__ == "__main__":
    main()
