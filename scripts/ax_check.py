#!/usr/bin/env python3
"""Quick GPU check of the anchor-and-extend scan (k_scan_ax) against the previous kernels and the CPU oracle.

Usage (GPU box): python scripts/ax_check.py [--timing]
Prints one line per case; exits non-zero on the first mismatch.
"""
import sys
import os
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401  (one HIP runtime per process: torch first)
import numpy as np

from oracle.oracle import Oracle
from speq_amd import DeviceIndex, FmIndex, synth


def compare(name, a, b, weights=True):
    ok = a.total == b.total and a.ambiguous == b.ambiguous and np.array_equal(a.unique, b.unique)
    if ok and weights and a.weights is not None and b.weights is not None:
        ok = np.allclose(a.weights, b.weights, rtol=1e-10, atol=0)
    print(f"{'ok  ' if ok else 'FAIL'} {name}: T {a.total}/{b.total} amb {a.ambiguous}/{b.ambiguous} "
          f"U {a.unique[:6].tolist()} / {b.unique[:6].tolist()}", flush=True)
    if not ok:
        d = np.nonzero(a.unique != b.unique)[0]
        print("   differing groups", d[:20].tolist(), (a.unique[d] - b.unique[d].astype(np.int64))[:20].tolist())
        if a.weights is not None and b.weights is not None:
            print("   W", a.weights[:5], b.weights[:5])
        sys.exit(1)


def main():
    timing = "--timing" in sys.argv
    cases = [
        dict(v=3, i=1, L=10_000, reads=5000, ks=[11, 15, 21, 31, 33, 40, 70, 100], nr=0.004, lq=0.01, ref_n=0.0005),
        dict(v=6, i=2, L=4000, reads=3000, ks=[21, 31, 64, 65, 128], nr=0.0, lq=0.0, ref_n=0.0),
    ]
    for c in cases:
        ref = synth.make_reference(c["v"], c["i"], c["L"], ref_n_rate=c["ref_n"])
        idx = FmIndex.build(ref.records, ref.groups, c["v"], prefix_q=10, pair_steps=True, triple_steps=True)
        dev = DeviceIndex(idx, 0)
        for paired in (False, True):
            reads = synth.make_reads(ref, c["reads"], n_rate=c["nr"], lowq_rate=c["lq"], short_frac=0.03,
                                     paired=paired)
            sb, qb = reads.seq.tobytes(), reads.qual.tobytes()
            for k in c["ks"]:
                orc = Oracle(ref.records, ref.groups, c["v"], k)
                for local in (False, True):
                    dev.tune(ax_scan=1)
                    got = dev.scan(sb, qb, reads.offsets, k=k, paired=paired, local=local)
                    T, amb, U, Wt = orc.scan(reads.seq, reads.qual, reads.offsets, paired=paired, local=local)
                    from speq_amd.api import ScanResult
                    exp = ScanResult(T, amb, U, Wt if local else None)
                    compare(f"v{c['v']} k={k} paired={paired} local={local} vs oracle", got, exp)
                    dev.tune(ax_scan=0)
                    old = dev.scan(sb, qb, reads.offsets, k=k, paired=paired, local=local)
                    dev.tune(ax_scan=1)
                    compare(f"v{c['v']} k={k} paired={paired} local={local} vs old kernels", got, old)
        dev.close()
    if timing:
        cfg = synth.CONFIGS[2]
        ref = synth.make_reference(cfg["n_variants"], cfg["n_isolates"], cfg["length"])
        idx = FmIndex.build(ref.records, ref.groups, cfg["n_variants"], prefix_q=12, pair_steps=True,
                            triple_steps=True, gpu_device=0)
        dev = DeviceIndex(idx, 0)
        reads = synth.make_reads(ref, 1_000_000)
        import torch as T
        d_seq = T.from_numpy(reads.seq).cuda()
        d_qual = T.from_numpy(reads.qual).cuda()
        d_off = T.from_numpy(reads.offsets.astype(np.int64)).cuda()
        G = cfg["n_variants"]
        for ax in (1, 0):
            dev.tune(ax_scan=ax)
            print("prepare", dev.prepare(21), flush=True)
            cnt = T.zeros(G + 2, dtype=T.int64, device="cuda")
            w = T.zeros(G, dtype=T.float64, device="cuda")
            for local in (False, True):
                for it in range(3):
                    cnt.zero_()
                    w.zero_()
                    T.cuda.synchronize()
                    dev.timing(True)
                    dev.timing_read()
                    dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, 21, cnt.data_ptr(),
                                    w.data_ptr(), local=local)
                    T.cuda.synchronize()
                    ms, n = dev.timing_read()
                print(f"cfg2 ax={ax} local={local}: {ms:.3f} ms  {130e6 / ms / 1e6:.1f} G k-mers/s  "
                      f"T={int(cnt[0])} amb={int(cnt[1])} U0={int(cnt[2])} W0={float(w[0]):.6f}", flush=True)
    print("AX_CHECK_OK")


if __name__ == "__main__":
    main()
