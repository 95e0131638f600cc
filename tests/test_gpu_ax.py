"""GPU: the anchor-and-extend read scan (k_scan_ax) against the CPU oracle and the other kernels.

The scan classifies a window from the class of the text position its bases were compared equal with, and finds a
window absent only after its anchor-table chain ended without a verified match; these tests aim at the places where
that could go wrong: windows that match the 2-bit text across a separator or an N (class SENT, deferred), reads
with many errors or no match at all (deferred-list overflow), low-complexity references (poly-A/T: long chains of
equal fingerprints and hash buckets), every anchor-table load factor, reads longer than a lane's staging segment,
k at the word boundaries of the compare (32/33, 64/65, 96/97, 127/128), and EM histograms.
Integer counters bit-exact; W to rtol 1e-10 (re-associated fp64 sums)."""
import numpy as np
import pytest

from oracle.oracle import Oracle
from speq_amd import DeviceIndex, EmHistogram, FmIndex, synth

pytestmark = pytest.mark.gpu

COMP = bytes.maketrans(b"ACGTN", b"TGCAN")


def distinct_kmers(records, k):
    seen = set()
    for r in records:
        r = r.upper()
        for s in (r, r.translate(COMP)[::-1]):
            for i in range(len(s) - k + 1):
                w = s[i:i + k]
                if b"N" not in w:
                    seen.add(w)
    return len(seen)


def check(dev, orc, seq, qual, off, k, paired=False, local=False, cutoff=30):
    got = dev.scan(seq.tobytes(), qual.tobytes(), off, k=k, paired=paired, local=local, phred_cutoff=cutoff)
    T, amb, U, W = orc.scan(seq, qual, off, paired=paired, local=local, phred_cutoff=cutoff)
    assert (got.total, got.ambiguous, got.unique.tolist()) == (T, amb, U.tolist()), (k, paired, local)
    if local:
        np.testing.assert_allclose(got.weights, W, rtol=1e-10, atol=0)
    return got


@pytest.fixture(scope="module")
def small():
    ref = synth.make_reference(4, 2, 6_000, ref_n_rate=0.002)
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=8, pair_steps=True, triple_steps=True)
    return ref, idx


@pytest.mark.parametrize("k", [1, 2, 7, 16, 21, 31, 40, 70, 128])
def test_distinct_kmers_and_last_kernel(small, k):
    ref, idx = small
    dev = DeviceIndex(idx)
    info = dev.prepare(k)
    assert info["distinct_kmers"] == distinct_kmers(ref.records, k)
    reads = synth.make_reads(ref, 300)
    dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k)
    assert dev.tuning("last_kernel") == 3  # k_scan_ax


@pytest.mark.parametrize("k", [1, 5, 31, 32, 33, 64, 65, 96, 97, 127, 128])
@pytest.mark.parametrize("paired", [False, True])
def test_word_boundary_k_vs_oracle(small, k, paired):
    ref, idx = small
    dev = DeviceIndex(idx)
    reads = synth.make_reads(ref, 1_500, n_rate=0.003, lowq_rate=0.01, err_rate=0.003, paired=paired,
                             short_frac=0.0 if paired else 0.05)
    orc = Oracle(ref.records, ref.groups, 4, k)
    for local in (False, True):
        check(dev, orc, reads.seq, reads.qual, reads.offsets, k, paired=paired, local=local)


def test_k_above_128_falls_back(small):
    ref, idx = small
    dev = DeviceIndex(idx)
    reads = synth.make_reads(ref, 300, read_len=250)
    check(dev, Oracle(ref.records, ref.groups, 4, 129), reads.seq, reads.qual, reads.offsets, 129)
    assert dev.tuning("last_kernel") == 0  # LF steps


@pytest.mark.parametrize("read_len", [191, 192, 193, 250, 400, 1000])
def test_long_reads_span_segments(small, read_len):
    ref, idx = small
    dev = DeviceIndex(idx)
    reads = synth.make_reads(ref, 400, read_len=read_len, err_rate=0.002, n_rate=0.001)
    for k in (21, 70, 128):
        orc = Oracle(ref.records, ref.groups, 4, k)
        check(dev, orc, reads.seq, reads.qual, reads.offsets, k, local=k == 21)


@pytest.mark.parametrize("ax_load", [10, 35, 90])
def test_table_load_factor(small, ax_load):
    ref, idx = small
    dev = DeviceIndex(idx)
    dev.tune(ax_load=ax_load)
    reads = synth.make_reads(ref, 2_000, err_rate=0.005)
    for k in (11, 21, 31, 55):
        check(dev, Oracle(ref.records, ref.groups, 4, k), reads.seq, reads.qual, reads.offsets, k)


def test_random_and_error_heavy_reads_overflow_the_deferred_list(small):
    """Random reads: every anchor is absent, so each lane defers k - 1 windows per lookup and the wave's list
    overflows (the lane then keeps its windows); reads with 5 % errors defer most of their windows too."""
    ref, idx = small
    dev = DeviceIndex(idx)
    rng = np.random.default_rng(5)
    n, L = 3_000, 150
    rnd = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n * L)
    noisy = synth.make_reads(ref, n, err_rate=0.05)
    clean = synth.make_reads(ref, n)
    seq = np.concatenate([rnd, noisy.seq, clean.seq])
    qual = np.full(seq.size, ord("I"), dtype=np.uint8)
    off = np.arange(0, seq.size + 1, L, dtype=np.uint64)
    for k in (11, 21, 31, 45, 70, 100):
        for local in (False, True):
            check(dev, Oracle(ref.records, ref.groups, 4, k), seq, qual, off, k, local=local)


def test_errors_in_first_windows_near_text_starts():
    """k > 64, reads with one to three errors in their first 90 bases: absent windows with no known mismatch (every
    window after them deferred), absent windows after absent windows, and deferred windows at the end of a read;
    reads from the first bases of short records whose k-mers the other records share put anchors near text starts
    (runs that must stop at a text end). Round 3 tried speculative left runs on exactly these reads (DESIGN.md §4e,
    commit dee1ce1); the test stays as a guard of the deferral paths."""
    ref = synth.make_reference(6, 3, 400)
    idx = FmIndex.build(ref.records, ref.groups, 6, prefix_q=8, pair_steps=True, triple_steps=True)
    dev = DeviceIndex(idx)
    rng = np.random.default_rng(11)
    comp = np.frombuffer(bytes.maketrans(b"ACGT", b"TGCA"), dtype=np.uint8)
    parts = []
    for i in range(6_000):
        rec = np.frombuffer(ref.records[int(rng.integers(len(ref.records)))], dtype=np.uint8)
        L = int(rng.choice([150, 150, 100, 75]))
        s0 = int(rng.integers(0, 8)) if i % 2 else int(rng.integers(0, rec.size - L + 1))
        r = rec[s0:s0 + L].copy()
        if i % 3 == 0:
            r = comp[r[::-1]]
        for _ in range(int(rng.integers(1, 4))):
            pos = int(rng.integers(0, min(90, L)))
            r[pos] = np.frombuffer(b"ACGT", dtype=np.uint8)[(np.searchsorted(np.frombuffer(b"ACGT", dtype=np.uint8),
                                                                            r[pos]) + 1 + int(rng.integers(3))) % 4]
        parts.append(r)
    seq = np.concatenate(parts)
    off = np.concatenate([[0], np.cumsum([p.size for p in parts])]).astype(np.uint64)
    qual = np.full(seq.size, ord("I"), dtype=np.uint8)
    qual[rng.random(seq.size) < 0.01] = ord("#")  # a few low-quality bases: invalid windows between anchors
    for k in (65, 70, 97, 128):
        for local in (False, True):
            check(dev, Oracle(ref.records, ref.groups, 6, k), seq, qual, off, k, local=local)


@pytest.mark.parametrize("k", [11, 21, 23, 31])
def test_low_complexity_references(k):
    """Poly-A / poly-T runs and short tandem repeats in the references and in the reads: one k-mer with thousands of
    occurrences, reads that match the 2-bit text across separators (coded as A) and Ns, and (for the k-mer table)
    the all-T key; compared with the k-mer table at two load factors, LF steps and the oracle."""
    rng = np.random.default_rng(k)
    recs = []
    for r in range(6):
        parts = [bytes(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=300))]
        parts.append(b"A" * int(rng.integers(40, 120)))
        parts.append(b"CAG" * int(rng.integers(10, 40)))
        parts.append(bytes(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=200)))
        parts.append(b"T" * int(rng.integers(40, 120)))
        parts.append(b"N" * int(rng.integers(0, 3)))
        parts.append(bytes(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=250)))
        recs.append(b"".join(parts))
    groups = [r % 3 for r in range(6)]
    idx = FmIndex.build(recs, groups, 3, prefix_q=6, pair_steps=True, triple_steps=True)
    reads = []
    for _ in range(3_000):
        r = recs[int(rng.integers(0, 6))]
        p = int(rng.integers(0, len(r) - 100))
        s = r[p:p + 100]
        if rng.random() < 0.5:
            s = s.translate(COMP)[::-1]
        reads.append(s)
    reads += [b"A" * 100, b"T" * 100, b"CAG" * 33 + b"C", b"A" * 60 + b"C" * 40]
    seq = np.frombuffer(b"".join(reads), dtype=np.uint8).copy()
    qual = np.full(seq.size, ord("I"), dtype=np.uint8)
    off = np.zeros(len(reads) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(x) for x in reads])
    orc = Oracle(recs, groups, 3, k)
    for tune in (dict(ax_scan=1), dict(ax_scan=1, ax_load=90), dict(ax_scan=0, kt_load8=35),
                 dict(ax_scan=0, kt_load8=90), dict(ax_scan=0, kt_compact=0), dict(ax_scan=0, kmer_table=0)):
        dev = DeviceIndex(idx)
        dev.tune(**tune)
        check(dev, orc, seq, qual, off, k)
        check(dev, orc, seq, qual, off, k, local=True)


@pytest.mark.parametrize("paired", [False, True])
def test_em_histogram_equals_other_kernels(paired):
    ref = synth.make_reference(5, 3, 8_000, ref_n_rate=0.0005)
    idx = FmIndex.build(ref.records, ref.groups, 5, prefix_q=9, pair_steps=True, triple_steps=True)
    reads = synth.make_reads(ref, 15_000, paired=paired, n_rate=0.001, lowq_rate=0.005, err_rate=0.004)
    res = {}
    for name, tune in (("ax", dict(ax_scan=1)), ("kt", dict(ax_scan=0)), ("lf", dict(ax_scan=0, kmer_table=0))):
        dev = DeviceIndex(idx)
        dev.tune(**tune)
        for k in (21, 31, 50):
            em = EmHistogram(dev)
            r = em.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, paired=paired, local=True)
            em.finalize()
            p = np.linspace(5.0, 30.0, 5)
            res[(name, k)] = (r.total, r.ambiguous, r.unique.tolist(), r.weights, em.info(),
                              em.step(p, [3] * 5, r.unique))
    for k in (21, 31, 50):
        for other in ("kt", "lf"):
            a, b = res[("ax", k)], res[(other, k)]
            assert a[:3] == b[:3], (k, other)
            np.testing.assert_allclose(a[3], b[3], rtol=1e-12)
            assert a[4] == b[4]
            np.testing.assert_array_equal(a[5], b[5])


def test_device_buffers_and_grid_knobs(small):
    """The HBM-resident entry point with tiny grids (many batches per wave) and occupancy caps."""
    import torch
    ref, idx = small
    reads = synth.make_reads(ref, 5_000, err_rate=0.002)
    d_seq = torch.from_numpy(reads.seq).cuda()
    d_qual = torch.from_numpy(reads.qual).cuda()
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
    orc = Oracle(ref.records, ref.groups, 4, 21)
    T, amb, U, _ = orc.scan(reads.seq, reads.qual, reads.offsets)
    dev = DeviceIndex(idx)
    for grid, bpc in ((1, 0), (3, 2), (65535, 0), (100, 1)):
        dev.tune(grid_blocks_ax=grid, blocks_per_cu_ax=bpc)
        cnt = torch.zeros(6, dtype=torch.int64, device="cuda")
        dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, 21, cnt.data_ptr())
        torch.cuda.synchronize()
        c = cnt.cpu().numpy()
        assert (int(c[0]), int(c[1]), c[2:].tolist()) == (T, amb, U.tolist()), (grid, bpc)


def test_grid_generations_give_identical_counts(small):
    """Tuning ax_generations (grid = n x the resident blocks, blocks dispatched as slots free up) and the one-block-per-
    CU cap change only which wave scans which reads: the counts of every setting equal the default's."""
    import torch
    ref, idx = small
    reads = synth.make_reads(ref, 150_000, err_rate=0.002)
    d_seq = torch.from_numpy(reads.seq).cuda()
    d_qual = torch.from_numpy(reads.qual).cuda()
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
    dev = DeviceIndex(idx)
    got = []
    for bpc, gens in ((0, 1), (1, 1), (1, 2), (1, 3), (0, 4)):
        dev.tune(blocks_per_cu_ax=bpc, ax_generations=gens)
        assert dev.tuning("ax_generations") == gens
        cnt = torch.zeros(6, dtype=torch.int64, device="cuda")
        dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, 31, cnt.data_ptr())
        torch.cuda.synchronize()
        got.append(cnt.cpu().numpy().tolist())
    assert all(g == got[0] for g in got), got
    with pytest.raises(Exception):
        dev.tune(ax_generations=0)


@pytest.mark.parametrize("k", [12, 21, 24, 25, 31, 32, 33, 40, 70, 97, 128])  # weight8's batch edges
@pytest.mark.parametrize("paired", [False, True])
def test_varying_quality_weights_within_the_documented_bound(k, paired):
    """Phred-weighted scans of reads whose qualities vary base by base (the anchor kernel's non-uniform path: k
    reciprocal products, or the shared-middle 8-window blocks) against the reference's left-to-right divisions
    (fm_scanner.cpp:454, restated in oracle/kmer_oracle.c) at the bound DESIGN.md §4e documents rather than 1e-10:
    each window within 3k·2^-53 (relative), and each group's sum of n_g windows within another (n_g + 1)·2^-53 for
    the different summation order, so |W_gpu - W_ref| <= (3k + 2 n_g + 2)·2^-53 · W_ref. Few hundred reads keep n_g
    small enough for the bound to see a single mis-weighted window (one wrong quality byte moves W by ~1e-5)."""
    ref = synth.make_reference(24, 1, 4_000)
    idx = FmIndex.build(ref.records, ref.groups, 24, prefix_q=8, pair_steps=True, triple_steps=True)
    dev = DeviceIndex(idx)
    orc = Oracle(ref.records, ref.groups, 24, k)
    reads = synth.make_reads(ref, 200, err_rate=0.002, paired=paired)
    rng = np.random.default_rng(k + 7 * paired)
    # qualities 31..41 changing at almost every base, 1 % at Q20 (below the cutoff 30: they split runs)
    q = rng.integers(31, 42, size=len(reads.qual)).astype(np.uint8)
    q[rng.random(len(q)) < 0.01] = 20
    qual = (q + 33).astype(np.uint8)
    got = dev.scan(reads.seq.tobytes(), qual.tobytes(), reads.offsets, k=k, paired=paired, local=True)
    T, amb, U, W = orc.scan(reads.seq, qual, reads.offsets, paired=paired, local=True)
    assert (got.total, got.ambiguous, got.unique.tolist()) == (T, amb, U.tolist())
    assert dev.tuning("last_kernel") == 3
    u = 2.0 ** -53
    for g in range(24):
        tol = (3 * k + 2 * int(U[g]) + 2) * u * W[g]
        assert abs(got.weights[g] - W[g]) <= tol, (g, got.weights[g], W[g], tol)
    assert int(U.sum()) > (2000 if k <= 70 else 200)  # enough windows counted for the bound to mean something


@pytest.mark.parametrize("k", [1, 3, 5, 7, 8, 9, 10])
def test_varying_quality_weights_short_k(k):
    """The same bound for k < 12, where windows are unique only if the groups share no k-mer: group 0's texts are
    A/T only and group 1's C/G only (both alphabets closed under reverse complement), so every window of a read is
    unique to its group. k < 8 weighs windows one by one (k reciprocal products in order), k = 8 is weight8 without a
    middle product, 9-10 with one partial batch."""
    rng = np.random.default_rng(100 + k)
    recs = [bytes(rng.choice(np.frombuffer(a, dtype=np.uint8), size=1_500)) for a in (b"AT", b"AT", b"CG", b"CG")]
    groups = [0, 0, 1, 1]
    idx = FmIndex.build(recs, groups, 2, prefix_q=6, pair_steps=True, triple_steps=True)
    dev = DeviceIndex(idx)
    orc = Oracle(recs, groups, 2, k)
    seqs = []
    for _ in range(150):
        r = recs[int(rng.integers(0, 4))]
        a = int(rng.integers(0, len(r) - 150))
        x = r[a:a + 150]
        seqs.append(x.translate(COMP)[::-1] if rng.random() < 0.5 else x)
    seq = np.frombuffer(b"".join(seqs), dtype=np.uint8)
    off = np.arange(0, 150 * len(seqs) + 1, 150, dtype=np.uint64)
    q = rng.integers(31, 42, size=len(seq)).astype(np.uint8)
    q[rng.random(len(q)) < 0.01] = 20
    qual = (q + 33).astype(np.uint8)
    got = dev.scan(seq.tobytes(), qual.tobytes(), off, k=k, local=True)
    T, amb, U, W = orc.scan(seq, qual, off, local=True)
    assert (got.total, got.ambiguous, got.unique.tolist()) == (T, amb, U.tolist())
    assert dev.tuning("last_kernel") == 3
    u = 2.0 ** -53
    for g in range(2):
        tol = (3 * k + 2 * int(U[g]) + 2) * u * W[g]
        assert abs(got.weights[g] - W[g]) <= tol, (g, got.weights[g], W[g], tol)
    assert int(U.sum()) > 10_000


def test_suffix_sort_failure_leaves_a_working_replica(small, monkeypatch):
    """The median representatives come from a suffix array that build_ax sorts into a buffer of its own and frees
    after k_ax_classify (a failed sort used to leave a published, unsorted array that later builds read).
    With the sort failing (injected after its buffer was allocated) the first claimant represents each k-mer: same
    counts as the oracle; a later k on the same replica (sort succeeding) too."""
    ref, idx = small
    reads = synth.make_reads(ref, 3_000, err_rate=0.003, n_rate=0.001)
    monkeypatch.setenv("SPEQ_INJECT_SA_SORT_FAILURE", "1")
    dev = DeviceIndex(idx)
    for k in (21, 70):
        for local in (False, True):
            check(dev, Oracle(ref.records, ref.groups, 4, k), reads.seq, reads.qual, reads.offsets, k, local=local)
        assert dev.tuning("last_kernel") == 3
    monkeypatch.delenv("SPEQ_INJECT_SA_SORT_FAILURE")
    for k in (31, 64):
        check(dev, Oracle(ref.records, ref.groups, 4, k), reads.seq, reads.qual, reads.offsets, k)
        assert dev.tuning("last_kernel") == 3
