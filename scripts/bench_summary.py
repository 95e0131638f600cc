#!/usr/bin/env python3
"""One-screen summary of bench.py JSON lines (the headline and its secondary lines): python scripts/bench_summary.py f"""
import json
import sys


def line(tag, d):
    r = d.get("roofline") or {}
    print(f"{tag:28s} {d['value'] / 1e9:8.1f} G k-mers/s  kernel {r.get('avg_kernel_ms', 0):.4f} ms  "
          f"own {r.get('bytes_per_kmer')} B/k-mer  frac {r.get('frac', 0):.3f}")
    if r.get("bytes_per_kmer_by_kind"):
        print("    bytes/k-mer:", r["bytes_per_kmer_by_kind"])
    if r.get("ax_work"):
        print("    work:", r["ax_work"])


for path in sys.argv[1:]:
    for ln in open(path):
        ln = ln.strip()
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        line("headline", d)
        for key, v in d.items():
            if isinstance(v, dict) and "value" in v and "roofline" in v:
                line(key, v)
