#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/<case>/ with a PURE-PYTHON brute force.

Independent of both the C oracle (hash map) and the product (FM-index): every window is matched against every
indexed text with str.find, the hit list is sorted by (text_id, pos) as SeqAn 3.0.x returns it (upstream,
believed) and the reference's loops are replayed literally:

  texts [fwd_r, revcomp(fwd_r)]                         /root/reference/src/fm_indexer.cpp:25-33
  filter min(Q) > cutoff && no N                         /root/reference/src/fm_scanner.cpp:162
  which_hit first-hit loop                               /root/reference/src/fm_scanner.cpp:165-177
  which_group / is_ambiguous (single: keep first)        /root/reference/src/fm_scanner.cpp:178-191
  paired local: which_group = last seen                  /root/reference/src/fm_scanner.cpp:941-957
  qavg = fold(a / (1 - 1/10^(b/10)))                     /root/reference/src/fm_scanner.cpp:454
  .dat pass hits_per_scaffold / is_unique                /root/reference/src/fm_scanner.cpp:1503-1539
  unique_to_percent                                      /root/reference/src/fm_scanner.cpp:1455-1474

Parity against SeqAn3 itself is UNPINNED (the reference cannot be built here); these vectors
pin our restatement of it. Run: python tests/golden/make_golden.py  (rewrites the fixtures deterministically).
"""
from __future__ import annotations

import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from speq_amd import synth  # noqa: E402  (numpy-only generator; no library load)

COMP = {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N"}


def dna5(s: str) -> str:
    out = []
    for ch in s:
        c = ch.upper()
        out.append("T" if c == "U" else (c if c in "ACGT" else "N"))
    return "".join(out)


def revcomp(s: str) -> str:
    return "".join(COMP[c] for c in reversed(s))


def phred(ch: str) -> int:
    return min(41, max(0, ord(ch) - 33))


def texts_of(records):
    t = []
    for r in records:
        f = dna5(r)
        t += [f, revcomp(f)]
    return t


def hits(texts, kmer):
    out = []
    for tid, t in enumerate(texts):
        p = t.find(kmer)
        while p >= 0:
            out.append((tid, p))
            p = t.find(kmer, p + 1)
    return sorted(out)


def which_hit(texts, dgs, kmer):
    w = -1
    for tid, _ in hits(texts, kmer):
        if w == -1:
            w = dgs[tid]
        elif w != dgs[tid]:
            w = -2
            break
    return w


def scan(texts, dgs, G, reads, quals, k, cutoff, local, paired):
    U = [0] * G
    W = [0.0] * G
    T = amb = 0
    units = [(2 * i, 2 * i + 1) for i in range(len(reads) // 2)] if paired else [(i,) for i in range(len(reads))]
    for unit in units:
        which_group, is_amb = -1, False
        for r in unit:
            s, q = dna5(reads[r]), [phred(c) for c in quals[r]]
            for j in range(len(s) - k + 1):
                km, qm = s[j:j + k], q[j:j + k]
                if not (min(qm) > cutoff and "N" not in km):
                    continue
                T += 1
                wh = which_hit(texts, dgs, km)
                if wh < 0:
                    continue
                U[wh] += 1
                if local:
                    acc = 1.0
                    for b in qm:
                        acc = acc / (1.0 - 1.0 / math.pow(10.0, b / 10.0))
                    W[wh] += acc
                if paired and local:
                    if which_group >= 0 and which_group != wh:
                        is_amb = True
                    which_group = wh
                else:
                    if which_group >= 0 and which_group != wh:
                        is_amb = True
                    else:
                        which_group = wh
        amb += int(is_amb)
    return T, amb, U, W


def em_pass(texts, dgs, G, reads, quals, k, cutoff, local, pp, percent, counts):
    """One EM estimator pass, literally (/root/reference/src/fm_scanner.cpp:1087-1125 global, :1175-1219 local)."""
    nxt = [0.0] * G
    for s_raw, q_raw in zip(reads, quals):
        s, q = dna5(s_raw), [phred(c) for c in q_raw]
        for j in range(len(s) - k + 1):
            km, qm = s[j:j + k], q[j:j + k]
            if not (min(qm) > cutoff and "N" not in km):
                continue
            if local:
                x = 1.0
                for b in qm:
                    x = x / (1.0 - 1.0 / math.pow(10.0, b / 10.0))
                y = 1.0
                for b in qm:
                    y = y * (1.0 - 1.0 / math.pow(10.0, b / 10.0))
                f = x - (1.0 - y)
            else:
                f = 1.0 / pp - (1 - pp)
            h = [0.0] * G
            for tid, _ in hits(texts, km):
                h[dgs[tid]] += f
            a = [h[i] * percent[i] / counts[i] for i in range(G)]
            norm = 0.0
            for x in a:
                norm += x
            if norm > 0.0:
                for i in range(G):
                    nxt[i] += a[i] / norm
    return nxt


def em_loop(step, unique_totals, total, percent, precision=1e-6, max_iter=200):
    """The refinement loop of /root/reference/src/fm_scanner.cpp:248-279."""
    out = []
    diff = [1.0] * len(percent)
    while max(diff) > precision and len(out) < max_iter:
        nxt = step(percent)
        new = unique_to_percent(unique_totals, total, unique_totals, nxt)
        diff = [abs(x - y) for x, y in zip(new, percent)]
        percent = new
        out.append({"percent": new, "next_tkpg": nxt})
    return out


def ref_unique(records, texts, dgs, group_scaffolds, G, k):
    u, t = [0] * G, [0] * G
    for r, (g, rec) in enumerate(zip(group_scaffolds, records)):
        f = dna5(rec)
        for s in (f, revcomp(f)):
            for j in range(len(s) - k + 1):
                per = [0] * len(dgs)
                for tid, _ in hits(texts, s[j:j + k]):
                    per[tid] += 1
                is_unique = all(not per[h] or g == dgs[h] for h in range(len(per)))
                t[g] += 1
                u[g] += int(is_unique)
    return u, t


def unique_to_percent(ur, total, uref, tref):
    out = []
    for i in range(len(uref)):
        if tref[i] > 0:
            pu = uref[i] / tref[i]
            out.append(100.0 * ur[i] / float(total) / pu if total else float("nan"))
        else:
            out.append(0.0)
    return out


def write_case(name, records, groups_text, group_scaffolds, n_groups, reads1, quals1, reads2, quals2, ks, cutoff,
               fixed_accuracy, group_counts):
    d = os.path.join(HERE, name)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "refs.fa"), "w") as f:
        for i, r in enumerate(records):
            f.write(f">rec{i}\n")
            for p in range(0, len(r), 70):
                f.write(r[p:p + 70] + "\n")
    with open(os.path.join(d, "groups.txt"), "w") as f:
        f.write(groups_text)
    for fn, rs, qs in (("reads_1.fq", reads1, quals1), ("reads_2.fq", reads2, quals2)):
        if rs is None:
            continue
        with open(os.path.join(d, fn), "w") as f:
            for i, (s, q) in enumerate(zip(rs, qs)):
                f.write(f"@r{i}\n{s}\n+\n{q}\n")
    texts = texts_of(records)
    dgs = [g for g in group_scaffolds for _ in (0, 1)]
    paired = reads2 is not None
    if paired:
        reads = [x for pair in zip(reads1, reads2) for x in pair]
        quals = [x for pair in zip(quals1, quals2) for x in pair]
    else:
        reads, quals = reads1, quals1
    exp = {"n_groups": n_groups, "group_scaffolds": group_scaffolds, "group_counts": group_counts, "paired": paired,
           "phred_cutoff": cutoff, "fixed_accuracy": fixed_accuracy, "by_k": {}}
    for k in ks:
        e = {}
        u_ref, t_ref = ref_unique(records, texts, dgs, group_scaffolds, n_groups, k)
        e["u_ref"], e["tot_ref"] = u_ref, t_ref
        for local in (False, True):
            T, amb, U, W = scan(texts, dgs, n_groups, reads, quals, k, cutoff, local, paired)
            if local:
                ut = W
            else:
                pp = math.pow(fixed_accuracy, k)
                ut = [u / pp for u in U]
            pct = unique_to_percent(ut, T, u_ref, t_ref)
            pp = math.pow(fixed_accuracy, k)
            em = em_loop(lambda p: em_pass(texts, dgs, n_groups, reads, quals, k, cutoff, local, pp, p, group_counts),
                         ut, T, pct) if k == ks[0] else None
            e["local" if local else "global"] = {"T": T, "ambiguous": amb, "U": U, "W": W if local else None,
                                                  "unique_totals": ut, "percent": pct, "em": em}
        exp["by_k"][str(k)] = e
    with open(os.path.join(d, "expected.json"), "w") as f:
        json.dump(exp, f, indent=1)
    print(name, {k: (v["global"]["T"], v["global"]["U"], v["u_ref"]) for k, v in exp["by_k"].items()},
          "em iterations", [len(exp["by_k"][str(ks[0])][m]["em"]) for m in ("global", "local")])


def reads_lists(reads):
    rs, qs = [], []
    for i in range(reads.n):
        a, b = int(reads.offsets[i]), int(reads.offsets[i + 1])
        rs.append(reads.seq[a:b].tobytes().decode())
        qs.append(reads.qual[a:b].tobytes().decode())
    return rs, qs


def main():
    # case 1: three variants, N in references and reads, low-Q bases, reads shorter than k
    ref = synth.make_reference(3, 1, 600, ref_n_rate=0.004)
    recs = [r.decode() for r in ref.records]
    recs[1] = recs[1][:300] + recs[1][300:].lower()   # lowercase input is dna5-converted
    rd = synth.make_reads(ref, 80, read_len=60, n_rate=0.01, lowq_rate=0.02, short_frac=0.1)
    rs, qs = reads_lists(rd)
    write_case("tiny_single", recs, ref.groupings_text(), [0, 1, 2], 3, rs, qs, None, None, [11, 7, 16], 30, 0.99,
               [1, 1, 1])

    # case 2: paired mates over 2 variants x 2 isolates
    ref2 = synth.make_reference(2, 2, 500)
    rp = synth.make_reads(ref2, 30, read_len=50, fragment=120, paired=True, n_rate=0.005, lowq_rate=0.02)
    rs, qs = reads_lists(rp)
    write_case("tiny_paired", [r.decode() for r in ref2.records], ref2.groupings_text(), [0, 0, 1, 1], 2,
               rs[0::2], qs[0::2], rs[1::2], qs[1::2], [13, 9], 30, 0.995, [2, 2])

    # case 3: scattered groupings written with ranges, singletons, comments and a bad token
    ref3 = synth.make_reference(5, 1, 300)
    groups_text = ("# scattered assignment\n"
                   "beta(2): 1, 4   # two records\n"
                   "alpha(1): 0-0, x7\n"
                   "gamma(3): 2-3\n"
                   "ignored line without a colon\n")
    rd3 = synth.make_reads(ref3, 40, read_len=40, lowq_rate=0.01)
    rs, qs = reads_lists(rd3)
    write_case("scattered_groups", [r.decode() for r in ref3.records], groups_text, [1, 0, 2, 2, 0], 3, rs, qs,
               None, None, [12, 8], 20, 0.98, [2, 1, 3])


if __name__ == "__main__":
    main()
