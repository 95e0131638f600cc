"""Parity suite for one build of the anchor-and-extend kernel (run as a child process by tests/test_gpu_ax_knobs.py).

`SPEQ_LIB_PATH=<variant>/libspeq_scan.so python tests/ax_knob_suite.py` scans with that build — a `make axknobs`
variant whose compile-time SPEQ_AX_* knobs are forced away from their defaults — and compares every case with the
CPU oracle (oracle/kmer_oracle.c; test infrastructure) and with the LF-step kernel of the same library: word-boundary
k (single-end and paired, global and Phred-weighted), reads with N / low-quality bases / errors, error-heavy and random
reads (deferred-list overflow), reads longer than a lane's segment, a config-2-sized batch (refills, issue priority,
several deferred passes per wave), HiSeq-style varying qualities (the weight work list) and the EM histogram.
Integer counters bit-exact; W to rtol 1e-10 (re-associated fp64 sums). Prints one JSON line; exits non-zero on any
mismatch."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.oracle import Oracle  # noqa: E402
from speq_amd import DeviceIndex, EmHistogram, FmIndex, synth  # noqa: E402
from speq_amd import _lib  # noqa: E402

CASES = []


def check(dev, orc, seq, qual, off, k, paired=False, local=False, tag=""):
    got = dev.scan(seq.tobytes(), qual.tobytes(), off, k=k, paired=paired, local=local)
    if dev.tuning("last_kernel") != 3:
        raise AssertionError(f"{tag}: k_scan_ax did not take the scan")
    T, amb, U, W = orc.scan(seq, qual, off, paired=paired, local=local)
    if (got.total, got.ambiguous, got.unique.tolist()) != (T, amb, U.tolist()):
        raise AssertionError(f"{tag} k={k} paired={paired} local={local}: {(got.total, got.ambiguous)} != {(T, amb)}")
    if local:
        np.testing.assert_allclose(got.weights, W, rtol=1e-10, atol=0, err_msg=tag)
    CASES.append(f"{tag}:k{k}:{'p' if paired else 's'}{'l' if local else 'g'}")


def main():
    lib = _lib.lib()
    maps = open("/proc/self/maps").read()
    want = os.path.realpath(_lib.LIB_PATH)
    if want not in maps:
        raise AssertionError(f"{want} is not the library this process loaded")
    del lib

    # small collection with N in the references: every k boundary of the word layout, both modes, single / paired
    ref = synth.make_reference(4, 2, 6_000, ref_n_rate=0.002)
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=8, pair_steps=True, triple_steps=True)
    dev = DeviceIndex(idx)
    for paired in (False, True):
        reads = synth.make_reads(ref, 1_500, n_rate=0.003, lowq_rate=0.01, err_rate=0.003, paired=paired,
                                 short_frac=0.0 if paired else 0.05)
        for k in (1, 5, 21, 31, 33, 64, 65, 70, 96, 97, 128):
            orc = Oracle(ref.records, ref.groups, 4, k)
            for local in (False, True):
                check(dev, orc, reads.seq, reads.qual, reads.offsets, k, paired, local, "boundary")

    # error-heavy and random reads: deferred-list overflow, many deferred passes
    rng = np.random.default_rng(5)
    n, L = 2_000, 150
    rnd = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n * L)
    noisy = synth.make_reads(ref, n, err_rate=0.05)
    clean = synth.make_reads(ref, n)
    seq = np.concatenate([rnd, noisy.seq, clean.seq])
    qual = np.full(seq.size, ord("I"), dtype=np.uint8)
    off = np.arange(0, seq.size + 1, L, dtype=np.uint64)
    for k in (11, 21, 45, 70, 100):
        orc = Oracle(ref.records, ref.groups, 4, k)
        for local in (False, True):
            check(dev, orc, seq, qual, off, k, False, local, "errors")

    # reads longer than a lane's staging segment
    reads = synth.make_reads(ref, 300, read_len=400, err_rate=0.002, n_rate=0.001)
    for k in (21, 70):
        check(dev, Oracle(ref.records, ref.groups, 4, k), reads.seq, reads.qual, reads.offsets, k, False, k == 21,
              "long")

    # HiSeq-style varying qualities (Phred-weighted: the weight work list), single-end and paired
    for paired in (False, True):
        reads = synth.make_reads(ref, 2_000, err_rate=0.002, paired=paired)
        reads = synth.apply_quality_profile(reads, "variable")
        for k in (21, 70):
            check(dev, Oracle(ref.records, ref.groups, 4, k), reads.seq, reads.qual, reads.offsets, k, paired, True,
                  "varq")

    # EM histogram: anchor kernel == LF steps (same library)
    reads = synth.make_reads(ref, 4_000, n_rate=0.001, lowq_rate=0.005, err_rate=0.004)
    rows = []
    for tune in (dict(ax_scan=1), dict(ax_scan=0, kmer_table=0)):
        d2 = DeviceIndex(idx)
        d2.tune(**tune)
        em = EmHistogram(d2)
        r = em.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=31, local=True)
        em.finalize()
        rows.append((r.total, r.ambiguous, r.unique.tolist(), em.info(),
                     em.step(np.linspace(5.0, 30.0, 4), [3] * 4, r.unique).tolist()))
        d2.close()
    if rows[0] != rows[1]:
        raise AssertionError(f"EM histogram: anchor kernel {rows[0][:4]} != LF steps {rows[1][:4]}")
    CASES.append("em:k31")
    dev.close()

    # a config-2-sized batch (200 k reads per launch: several refills and deferred passes per wave, full grid)
    c = synth.CONFIGS[2]
    ref2 = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx2 = FmIndex.build(ref2.records, ref2.groups, c["n_variants"], prefix_q=10, pair_steps=True, triple_steps=True)
    dev2 = DeviceIndex(idx2)
    reads = synth.make_reads(ref2, 200_000, err_rate=0.002)
    for k in (21, 70):
        orc = Oracle(ref2.records, ref2.groups, c["n_variants"], k)
        for local in (False, True):
            check(dev2, orc, reads.seq, reads.qual, reads.offsets, k, False, local, "cfg2")
    dev2.close()
    print(json.dumps({"lib": want, "cases": len(CASES), "ok": True}), flush=True)


if __name__ == "__main__":
    main()
