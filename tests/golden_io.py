"""Test helper: loads a tests/golden/<case>/ fixture (plain FASTA/FASTQ parsing, no product code)."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["tiny_single", "tiny_paired", "scattered_groups"]


def read_fasta(path):
    recs, cur = [], None
    for line in open(path):
        line = line.rstrip("\n")
        if line.startswith(">"):
            if cur is not None:
                recs.append(cur)
            cur = ""
        elif cur is not None:
            cur += line.strip()
    if cur is not None:
        recs.append(cur)
    return [r.encode() for r in recs]


def read_fastq(path):
    lines = open(path).read().split("\n")
    seqs, quals = [], []
    for i in range(0, len(lines) - 3, 4):
        seqs.append(lines[i + 1].encode())
        quals.append(lines[i + 3].encode())
    return seqs, quals


class Case:
    def __init__(self, name):
        d = os.path.join(GOLDEN, name)
        self.name, self.dir = name, d
        self.records = read_fasta(os.path.join(d, "refs.fa"))
        self.exp = json.load(open(os.path.join(d, "expected.json")))
        self.groups = self.exp["group_scaffolds"]
        self.G = self.exp["n_groups"]
        self.paired = self.exp["paired"]
        s1, q1 = read_fastq(os.path.join(d, "reads_1.fq"))
        if self.paired:
            s2, q2 = read_fastq(os.path.join(d, "reads_2.fq"))
            seqs = [x for p in zip(s1, s2) for x in p]
            quals = [x for p in zip(q1, q2) for x in p]
        else:
            seqs, quals = s1, q1
        self.seq = b"".join(seqs)
        self.qual = b"".join(quals)
        self.offsets = np.zeros(len(seqs) + 1, dtype=np.uint64)
        self.offsets[1:] = np.cumsum([len(s) for s in seqs])
        self.ks = [int(k) for k in self.exp["by_k"]]
        self.cutoff = self.exp["phred_cutoff"]
