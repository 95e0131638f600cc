"""GPU: the k-mer interval table gives exactly what LF-step search gives: counters, Phred weights
(same per-window arithmetic, rtol 1e-12 for the different summation order), EM histograms and the .dat pass; its
key set is the set of distinct N-free k-mers of the reference texts (fwd and rc of every record); k-mers absent
from the reference are found absent; k > 31 has no table."""
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


@pytest.fixture(scope="module")
def small():
    ref = synth.make_reference(3, 2, 5_000, ref_n_rate=0.002)
    idx = FmIndex.build(ref.records, ref.groups, 3, prefix_q=8, pair_steps=True, triple_steps=True)
    return ref, idx


@pytest.mark.parametrize("k", [1, 2, 7, 16, 21, 31])
def test_key_set_is_the_distinct_reference_kmers(small, k):
    ref, idx = small
    dev = DeviceIndex(idx)
    dev.tune(ax_scan=0)  # the k-mer table (the anchor-and-extend structures: tests/test_gpu_ax.py)
    info = dev.prepare(k)
    assert info["distinct_kmers"] == distinct_kmers(ref.records, k)
    # 16-B slots at load <= 1/2, or (k <= 23) 8-B slots at load kt_load8 (35 % by default, ~23 B per k-mer):
    # >= 16 B per distinct k-mer either way
    assert info["table_bytes"] >= 16 * info["distinct_kmers"]


def test_no_table_above_31_or_when_off(small):
    _, idx = small
    dev = DeviceIndex(idx)
    dev.tune(ax_scan=0)
    assert dev.prepare(32)["table_bytes"] == 0
    dev.tune(kmer_table=0)
    assert dev.prepare(21)["table_bytes"] == 0
    assert dev.tuning("kmer_table") == 0


@pytest.mark.parametrize("paired", [False, True])
@pytest.mark.parametrize("local", [False, True])
def test_table_equals_lf_steps_with_em(paired, local):
    ref = synth.make_reference(6, 3, 12_000, ref_n_rate=0.0005)
    idx = FmIndex.build(ref.records, ref.groups, 6, prefix_q=10, pair_steps=True, triple_steps=True)
    reads = synth.make_reads(ref, 30_000, paired=paired, n_rate=0.001, lowq_rate=0.005, err_rate=0.004)
    res = {}
    for kt in (1, 0):
        dev = DeviceIndex(idx)
        dev.tune(kmer_table=kt, ax_scan=0)
        for k in (31, 21, 15):  # several tables on one replica, built in turn
            em = EmHistogram(dev)
            r = em.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, paired=paired, local=local)
            em.finalize()
            p = np.linspace(5.0, 30.0, 6)
            res[(kt, k)] = (r, em.info(), em.step(p, [3] * 6, r.unique))
            u = dev.count_unique_kmers_per_group(k)
            res[(kt, k, "dat")] = (u[0].tolist(), u[1].tolist())
    for k in (31, 21, 15):
        a, b = res[(1, k)], res[(0, k)]
        assert (a[0].total, a[0].ambiguous, a[0].unique.tolist()) == (b[0].total, b[0].ambiguous, b[0].unique.tolist())
        if local:
            np.testing.assert_allclose(a[0].weights, b[0].weights, rtol=1e-12)
        assert a[1] == b[1]
        np.testing.assert_array_equal(a[2], b[2])
        assert res[(1, k, "dat")] == res[(0, k, "dat")]


def test_absent_kmers_and_oracle():
    ref = synth.make_reference(4, 1, 8_000)
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=6, pair_steps=True, triple_steps=True)
    dev = DeviceIndex(idx)
    dev.tune(ax_scan=0)
    rng = np.random.default_rng(7)
    n, L = 2_000, 120
    seq = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n * L)  # random reads: absent 21-mers
    mixed = synth.make_reads(ref, n, read_len=L)
    seq = np.concatenate([seq, mixed.seq])
    qual = np.full(seq.size, ord("I"), dtype=np.uint8)
    off = np.arange(0, seq.size + 1, L, dtype=np.uint64)
    for k in (11, 21, 31):
        r = dev.scan(seq.tobytes(), qual.tobytes(), off, k=k)
        T, amb, U, _ = Oracle(ref.records, ref.groups, 4, k).scan(seq, qual, off)
        assert (r.total, r.ambiguous, r.unique.tolist()) == (T, amb, U.tolist())
        assert r.total == 2 * n * (L - k + 1)


@pytest.mark.parametrize("ilp_kt", [0, 1, 2, 4])
@pytest.mark.parametrize("kt_slots", [2, 5, 16])
def test_launch_knobs_keep_results(small, ilp_kt, kt_slots):
    ref, idx = small
    reads = synth.make_reads(ref, 4_000, n_rate=0.002, lowq_rate=0.01, short_frac=0.05)
    dev = DeviceIndex(idx)
    dev.tune(ilp_kt=ilp_kt, kt_slots=kt_slots, ax_scan=0)
    for k in (13, 21, 31):
        r = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k)
        T, amb, U, _ = Oracle(ref.records, ref.groups, 3, k).scan(reads.seq, reads.qual, reads.offsets)
        assert (r.total, r.ambiguous, r.unique.tolist()) == (T, amb, U.tolist())


def test_phred_weight_of_one_window_is_bit_exact(small):
    """A read of exactly k bases that occurs in one group: W[g] is that window's weight, the reference's
    left-to-right divisions w = w / (1 - 1/10^(q/10)) (fm_scanner.cpp:454). The k-mer-table kernel divides the same
    way (bit-exact); the anchor kernel takes one-quality windows from its quotient table (bit-exact) and multiplies
    the k reciprocals of any other window: |w - w_ref| <= 3 k 2^-53 w."""
    ref, idx = small
    rng = np.random.default_rng(11)
    devs = [DeviceIndex(idx), DeviceIndex(idx)]
    devs[1].tune(ax_scan=0)  # both read-scan kernels
    k = 31
    checked = 0
    tol = 3 * k * 2.0 ** -53
    for _ in range(150):
        r = int(rng.integers(0, len(ref.records)))
        rec = ref.records[r]
        p = int(rng.integers(0, len(rec) - k))
        seq = rec[p:p + k].upper()
        if b"N" in seq:
            continue
        # varied qualities, or one quality for the whole window (weight from the per-block uniform-q table)
        q = rng.integers(31, 42, size=k) if checked % 2 else np.full(k, int(rng.integers(31, 42)))
        qual = bytes((q + 33).astype(np.uint8))
        for dev, exact in zip(devs, (checked % 2 == 0, True)):
            res = dev.scan(seq, qual, np.array([0, k], dtype=np.uint64), k=k, local=True)
            if res.unique.sum() != 1:
                break  # the window is shared by several groups
            w = 1.0
            for x in q:
                w = w / (1.0 - 1.0 / (10.0 ** (float(x) / 10.0)))
            g = int(np.argmax(res.unique))
            if exact:
                assert res.weights[g] == w, (res.weights[g], w)
            else:
                assert abs(res.weights[g] - w) <= tol * w, (res.weights[g], w)
        else:
            checked += 1
    assert checked > 50


@pytest.mark.parametrize("paired", [False, True])
def test_compact_table_equals_wide_table(paired):
    """k <= 23 uses the compact 8-B-slot table by default; it must give what the 16-B-slot table and LF steps give
    (counters, Phred weights, EM rows and steps); k = 24 falls back to the wide table."""
    ref = synth.make_reference(5, 3, 10_000, ref_n_rate=0.0005)
    idx = FmIndex.build(ref.records, ref.groups, 5, prefix_q=9, pair_steps=True, triple_steps=True)
    reads = synth.make_reads(ref, 20_000, paired=paired, n_rate=0.001, lowq_rate=0.005, err_rate=0.004)
    res = {}
    for mode in ("compact", "wide", "lf"):
        dev = DeviceIndex(idx)
        dev.tune(kt_compact=int(mode == "compact"), kmer_table=int(mode != "lf"), kt_load8=50, ax_scan=0)
        for k in (11, 21, 23, 24):
            info = dev.prepare(k)
            em = EmHistogram(dev)
            r = em.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, paired=paired, local=True)
            em.finalize()
            p = np.linspace(5.0, 30.0, 5)
            res[(mode, k)] = (r.total, r.ambiguous, r.unique.tolist(), r.weights, em.info(),
                              em.step(p, [2] * 5, r.unique), info["table_bytes"])
    for k in (11, 21, 23, 24):
        for other in ("wide", "lf"):
            a, b = res[("compact", k)], res[(other, k)]
            assert a[:3] == b[:3], (k, other)
            np.testing.assert_allclose(a[3], b[3], rtol=1e-12)
            assert a[4] == b[4]
            np.testing.assert_array_equal(a[5], b[5])
    # at kt_load8 = 50 % the compact table (16 B per k-mer + 8 B per multi-group k-mer) is smaller than the wide one (>= 32 B
    # per k-mer) for k <= 23; k = 24 uses the wide table either way
    for k in (11, 21, 23):
        assert res[("compact", k)][6] < res[("wide", k)][6]
    assert res[("compact", 24)][6] == res[("wide", 24)][6]


@pytest.mark.parametrize("load8", [35, 90])
def test_compact_table_poly_t_and_full_buckets(load8):
    """The compact lookup relies on slots filling a bucket in order and on the all-T k-mer being the only key whose
    bits can look like an empty slot's: poly-T (and poly-A) runs in the reference and in the reads, present and absent,
    at the default load and at 90 % (many full buckets: lookups continue into the next bucket). Compact, wide and LF
    steps must agree (k = 11, 21, 23)."""
    rng = np.random.default_rng(5)
    base = synth.make_reference(3, 2, 6_000)
    recs = []
    for i, r in enumerate(base.records):
        r = bytearray(r)
        if i % 2 == 0:  # poly-T / poly-A runs of 40 inside every other record (the rc texts get the complement)
            for p in rng.integers(0, len(r) - 50, 4):
                r[p:p + 40] = (b"T" if p % 2 else b"A") * 40
        recs.append(bytes(r))
    groups = list(base.groups)
    idx = FmIndex.build(recs, groups, 3, prefix_q=8, pair_steps=True, triple_steps=True)
    reads = synth.make_reads(base, 6_000, n_rate=0.001)
    extra = [b"T" * 60, b"A" * 60, b"T" * 30 + b"ACGT" * 8, b"G" * 50, b"TTTTTTTTTTTTTTTTTTTTTTTC" * 3]
    seqs = [reads.seq[int(reads.offsets[i]):int(reads.offsets[i + 1])].tobytes() for i in range(reads.n)] + extra
    off = np.zeros(len(seqs) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in seqs])
    seq = b"".join(seqs)
    qual = b"I" * len(seq)
    res = {}
    for mode in ("compact", "wide", "lf"):
        dev = DeviceIndex(idx)
        dev.tune(kt_compact=int(mode == "compact"), kmer_table=int(mode != "lf"), kt_load8=load8, ax_scan=0)
        for k in (11, 21, 23):
            r = dev.scan(seq, qual, off, k=k, local=True)
            res[(mode, k)] = (r.total, r.ambiguous, r.unique.tolist(), r.weights)
        dev.close()
    for k in (11, 21, 23):
        for other in ("wide", "lf"):
            a, b = res[("compact", k)], res[(other, k)]
            assert a[:3] == b[:3], (k, other)
            np.testing.assert_allclose(a[3], b[3], rtol=1e-12)
        T, amb, U, W = Oracle(recs, groups, 3, k).scan(np.frombuffer(seq, np.uint8), np.frombuffer(qual, np.uint8),
                                                       off, local=True)
        assert res[("compact", k)][:3] == (T, amb, U.tolist())
