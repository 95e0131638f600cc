"""CPU: the SeqAn-like stand-in (oracle/seqan_like.c: wavelet-matrix backward search + SA-sample locate + sorted
hit lists + first-hit rule) against the committed golden vectors, the pure-Python brute force and the hash-map
oracle. Three independent restatements of the reference's per-window semantics must agree bit-exactly."""
import os
import sys

import numpy as np
import pytest

from golden_io import CASES, Case
from oracle.oracle import Oracle, SeqanLike
from speq_amd import synth

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as bf  # noqa: E402


@pytest.mark.parametrize("name", CASES)
def test_seqan_like_matches_golden(name):
    c = Case(name)
    sl = SeqanLike(c.records, c.groups, c.G)
    for k in c.ks:
        for mode in ("global", "local"):
            g = c.exp["by_k"][str(k)][mode]
            T, amb, U, W = sl.scan(c.seq, c.qual, c.offsets, k=k, phred_cutoff=c.cutoff, paired=c.paired,
                                   local=mode == "local")
            assert (T, amb, U.tolist()) == (g["T"], g["ambiguous"], g["U"])
            if mode == "local":
                np.testing.assert_allclose(W, g["W"], rtol=1e-12)


@pytest.mark.parametrize("seed", range(3))
def test_seqan_like_counts_equal_substring_search(seed):
    rng = np.random.default_rng(seed)
    ref = synth.make_reference(3, 2, 400, ref_n_rate=0.01)
    recs = [r.decode() for r in ref.records]
    texts = bf.texts_of(recs)
    dgs = [g for g in ref.groups for _ in (0, 1)]
    sl = SeqanLike(ref.records, ref.groups, 3)
    assert sl.n == sum(len(t) + 1 for t in texts) + 1
    for _ in range(200):
        t = texts[int(rng.integers(len(texts)))]
        k = int(rng.integers(1, 25))
        p = int(rng.integers(0, len(t) - k + 1))
        km = t[p:p + k]
        if rng.random() < 0.2:  # mutate: often absent
            km = km[:k // 2] + "ACGT"[int(rng.integers(4))] + km[k // 2 + 1:]
        assert sl.count(km.encode()) == len(bf.hits(texts, km))
        assert sl.which(km.encode()) == bf.which_hit(texts, dgs, km)


@pytest.mark.parametrize("paired", [False, True])
def test_seqan_like_equals_hash_oracle(paired):
    ref = synth.make_reference(4, 2, 3_000, ref_n_rate=0.002)
    reads = synth.make_reads(ref, 1_500, read_len=120, paired=paired, n_rate=0.003, lowq_rate=0.01, short_frac=0.0)
    sl = SeqanLike(ref.records, ref.groups, 4)
    for k in (9, 21, 31):
        orc = Oracle(ref.records, ref.groups, 4, k)
        for local in (False, True):
            a = sl.scan(reads.seq, reads.qual, reads.offsets, k=k, paired=paired, local=local, threads=4)
            b = orc.scan(reads.seq, reads.qual, reads.offsets, paired=paired, local=local, threads=4)
            assert a[:2] == b[:2] and a[2].tolist() == b[2].tolist()
            if local:
                np.testing.assert_allclose(a[3], b[3], rtol=1e-12)


@pytest.mark.parametrize("steps", [1, 2, 3])
@pytest.mark.parametrize("paired", [False, True])
def test_label_run_cpu_path_equals_hash_oracle(steps, paired):
    """oracle/fm_cpu.c (the build's label-run algorithm on CPU cores, the bench's second CPU column) over our own
    index arrays agrees with the hash-map oracle."""
    from oracle.oracle import FmCpu
    from speq_amd import FmIndex
    ref = synth.make_reference(4, 2, 4_000, ref_n_rate=0.002)
    reads = synth.make_reads(ref, 1_500, read_len=110, paired=paired, n_rate=0.003, lowq_rate=0.01)
    for q in (0, 7):
        idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=q, pair_steps=steps >= 2, triple_steps=steps == 3)
        fc = FmCpu(idx)
        for k in (9, 21, 32):
            orc = Oracle(ref.records, ref.groups, 4, k)
            a = fc.scan(reads.seq, reads.qual, reads.offsets, k=k, paired=paired, threads=4)
            b = orc.scan(reads.seq, reads.qual, reads.offsets, paired=paired, threads=4)
            assert a[:2] == b[:2] and a[2].tolist() == b[2].tolist(), (q, k)


def test_seqan_like_from_product_suffix_array_is_the_same_structure():
    """bench.py's config-5 CPU baseline hands the product index's suffix array to the stand-in (its own doubling sort
    takes minutes at 200 M symbols): a suffix array is unique, so the structure — SA samples and scan results — must
    be identical to the stand-in's own build."""
    from speq_amd import FmIndex
    ref = synth.make_reference(4, 2, 3000, ref_n_rate=0.002)
    own = SeqanLike(ref.records, ref.groups, 4)
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=4)
    given = SeqanLike(ref.records, ref.groups, 4, sa=idx.array("sa", np.uint32))
    assert own.n == given.n
    assert all(own.sample(j) == given.sample(j) for j in range(own.n // 16 + 1))
    reads = synth.make_reads(ref, 300, err_rate=0.01, n_rate=0.005, lowq_rate=0.01)
    for k in (15, 31):
        a = own.scan(reads.seq, reads.qual, reads.offsets, k=k)
        b = given.scan(reads.seq, reads.qual, reads.offsets, k=k)
        assert (a[0], a[1], a[2].tolist()) == (b[0], b[1], b[2].tolist())
    with pytest.raises(ValueError):
        SeqanLike(ref.records, ref.groups, 4, sa=idx.array("sa", np.uint32)[:-1])
