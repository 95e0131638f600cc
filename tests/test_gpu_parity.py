"""GPU parity: the HIP scan path (through the C ABI) against the CPU oracle on the same seeded inputs.

Integer counters (T, ambiguous, U[g], U_ref[g], Tot_ref[g]) must be bit-exact. Phred-weighted W[g] is fp64: per
window it is computed with the same left-to-right divisions as the reference (fm_scanner.cpp:454), but windows
are summed in a different order, so W is compared with rtol = 1e-10 (worst-case re-association error ~N eps).
"""
import numpy as np
import pytest

from oracle.oracle import Oracle
from speq_amd import DeviceIndex, FmIndex, synth

pytestmark = pytest.mark.gpu
W_RTOL = 1e-10  # fp64 sums of up to ~1e8 windows in a different order (worst case ~N * eps)


# kernel variants: anchor-and-extend (the default), the k-mer-table kernel, LF steps (one and two windows per lane)
VARIANTS = [dict(ax_scan=1, kmer_table=1, ilp=1), dict(ax_scan=0, kmer_table=1, ilp=1),
            dict(ax_scan=0, kmer_table=0, ilp=1), dict(ax_scan=0, kmer_table=0, ilp=2)]


def _check(dev, orc, reads, k, cutoff=30, paired=False, local=False, ilps=(1, 2)):
    """Every kernel variant (anchor-and-extend; k-mer interval table; LF steps with 1 and 2 windows per lane) must
    give the oracle's counts."""
    for v in VARIANTS:
        if v["ilp"] not in ilps:
            continue
        dev.tune(ilp=v["ilp"], ilp_local=v["ilp"], kmer_table=v["kmer_table"], ax_scan=v["ax_scan"])
        got = _check_one(dev, orc, reads, k, cutoff, paired, local)
    dev.tune(ilp=1, ilp_local=1, kmer_table=1, ax_scan=1)
    return got


def _check_one(dev, orc, reads, k, cutoff, paired, local):
    got = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, phred_cutoff=cutoff,
                   paired=paired, local=local)
    T, amb, U, W = orc.scan(reads.seq, reads.qual, reads.offsets, phred_cutoff=cutoff, paired=paired, local=local)
    assert got.total == T
    assert got.ambiguous == amb
    assert np.array_equal(got.unique, U), (got.unique, U)
    if local:
        np.testing.assert_allclose(got.weights, W, rtol=W_RTOL, atol=0)
    return got


@pytest.fixture(scope="module")
def cfg1():
    ref = synth.make_reference(3, 1, 10_000)
    reads = synth.make_reads(ref, 10_000)
    return ref, reads


@pytest.mark.parametrize("q", [0, 10])
@pytest.mark.parametrize("local", [False, True])
@pytest.mark.parametrize("steps", [1, 2, 3])
def test_config1_single(cfg1, q, local, steps):
    ref, reads = cfg1
    idx = FmIndex.build(ref.records, ref.groups, 3, prefix_q=q, pair_steps=steps >= 2, label_table=steps == 2,
                        triple_steps=steps == 3)
    dev = DeviceIndex(idx)
    orc = Oracle(ref.records, ref.groups, 3, 21)
    got = _check(dev, orc, reads, 21, local=local)
    assert got.total == 10_000 * 130  # all-Q40, no N: every window passes
    u, t = dev.count_unique_kmers_per_group(21)
    ou, ot = orc.ref_unique()
    assert np.array_equal(u, ou) and np.array_equal(t, ot)


@pytest.fixture(scope="module")
def edge():
    ref = synth.make_reference(4, 2, 3_000, ref_n_rate=0.003)
    reads = synth.make_reads(ref, 3_000, n_rate=0.005, lowq_rate=0.02, short_frac=0.05)
    return ref, reads


@pytest.mark.parametrize("k", [1, 2, 5, 16, 21, 31, 32, 33, 70, 150, 151])
@pytest.mark.parametrize("steps", [1, 2, 3])
def test_edge_reads_all_k(edge, k, steps):
    ref, reads = edge
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=6, pair_steps=steps >= 2, label_table=steps != 2,
                        triple_steps=steps == 3)
    dev = DeviceIndex(idx)
    orc = Oracle(ref.records, ref.groups, 4, k)
    _check(dev, orc, reads, k)
    _check(dev, orc, reads, k, local=True)
    _check(dev, orc, reads, k, cutoff=5)
    u, t = dev.count_unique_kmers_per_group(k)
    ou, ot = orc.ref_unique()
    assert np.array_equal(u, ou) and np.array_equal(t, ot), (k, u, ou, t, ot)


@pytest.mark.parametrize("steps", [1, 2, 3])
def test_prefix_levels_agree(edge, steps):
    """Every q-mer table level (q, q-1, q-2; auto picks by k) gives the oracle's counts."""
    ref, reads = edge
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=9, pair_steps=steps >= 2, triple_steps=steps == 3,
                        label_table=True)
    dev = DeviceIndex(idx)
    for k in (5, 7, 8, 9, 10, 11, 21, 31, 70):
        orc = Oracle(ref.records, ref.groups, 4, k)
        for lvl, sparse in ((-1, 0), (0, 0), (0, 1), (1, 1), (2, 0), (2, 1), (-1, 1), (-1, -1)):
            dev.tune(prefix_level=lvl, sparse_prefix=sparse)
            assert dev.tuning("prefix_level") == lvl and dev.tuning("sparse_prefix") == sparse
            _check_one(dev, orc, reads, k, 30, False, False)
            u, t = dev.count_unique_kmers_per_group(k)
            ou, ot = orc.ref_unique()
            assert np.array_equal(u, ou) and np.array_equal(t, ot), (k, lvl)
    dev.tune(prefix_level=-1, sparse_prefix=0)


@pytest.mark.parametrize("local", [False, True])
def test_paired(edge, local):
    ref, _ = edge
    reads = synth.make_reads(ref, 2_000, paired=True, n_rate=0.003, lowq_rate=0.01)
    for tri in (False, True):
        idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=8, pair_steps=True, label_table=True,
                            triple_steps=tri)
        dev = DeviceIndex(idx)
        for k in (21, 31, 64):
            orc = Oracle(ref.records, ref.groups, 4, k)
            _check(dev, orc, reads, k, paired=True, local=local)


def test_empty_and_short_inputs(edge):
    ref, _ = edge
    idx = FmIndex.build(ref.records, ref.groups, 4)
    dev = DeviceIndex(idx)
    got = dev.scan(b"", b"", np.zeros(1, np.uint64), k=21)
    assert got.total == 0 and got.ambiguous == 0 and not got.unique.any()
    seq = b"ACGT" * 5
    off = np.array([0, 4, 4, 20], dtype=np.uint64)  # 3 reads: 4 bp, empty, 16 bp (< k)
    got = dev.scan(seq, b"I" * 20, off, k=21)
    assert got.total == 0 and not got.unique.any()


def test_many_groups_global_atomics():
    """G > 2048 takes the global-atomic tally path of the kernel."""
    G = 2500
    ref = synth.make_reference(G, 1, 300)
    reads = synth.make_reads(ref, 4_000, read_len=100)
    idx = FmIndex.build(ref.records, ref.groups, G, prefix_q=5, pair_steps=True, label_table=True)
    dev = DeviceIndex(idx)
    orc = Oracle(ref.records, ref.groups, G, 25)
    _check(dev, orc, reads, 25)
    _check(dev, orc, reads, 25, local=True)
    u, t = dev.count_unique_kmers_per_group(25)
    ou, ot = orc.ref_unique()
    assert np.array_equal(u, ou) and np.array_equal(t, ot)


@pytest.mark.parametrize("k", [21, 45, 70])
def test_two_byte_classes_lds_tally(k):
    """254 <= G <= 2048: two-byte anchor classes with the LDS tally (the kernel built for 3 waves/SIMD there)."""
    G = 300
    ref = synth.make_reference(G, 1, 400)
    reads = synth.make_reads(ref, 4_000)
    idx = FmIndex.build(ref.records, ref.groups, G, prefix_q=6, pair_steps=True, label_table=True)
    dev = DeviceIndex(idx)
    orc = Oracle(ref.records, ref.groups, G, k)
    _check(dev, orc, reads, k)
    _check(dev, orc, reads, k, local=True)


def test_irregular_groupings():
    """Records assigned to groups out of order, one group spanning scattered records, single group."""
    ref = synth.make_reference(6, 1, 4_000)
    reads = synth.make_reads(ref, 2_000)
    for groups, G in (([2, 0, 1, 2, 0, 1], 3), ([0] * 6, 1), ([5, 4, 3, 2, 1, 0], 6)):
        idx = FmIndex.build(ref.records, groups, G, prefix_q=7, pair_steps=True, label_table=True)
        dev = DeviceIndex(idx)
        orc = Oracle(ref.records, groups, G, 19)
        _check(dev, orc, reads, 19)
        u, t = dev.count_unique_kmers_per_group(19)
        ou, ot = orc.ref_unique()
        assert np.array_equal(u, ou) and np.array_equal(t, ot)


def test_device_buffers_match_host_path(cfg1):
    """The hot-path entry (speq_scan_reads_device on HBM-resident torch tensors) equals the host path."""
    torch = pytest.importorskip("torch")
    ref, reads = cfg1
    idx = FmIndex.build(ref.records, ref.groups, 3, prefix_q=10)
    dev = DeviceIndex(idx)
    host = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21, local=True)
    cuda = torch.device("cuda:0")
    d_seq = torch.from_numpy(reads.seq).to(cuda)
    d_qual = torch.from_numpy(reads.qual).to(cuda)
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).to(cuda)
    d_counts = torch.zeros(3 + 2, dtype=torch.int64, device=cuda)
    d_w = torch.zeros(3, dtype=torch.float64, device=cuda)
    stream = torch.cuda.current_stream().cuda_stream  # 0 = the null stream: torch's ops and ours are ordered
    for _ in range(3):  # zero -> scan, repeated: the counters must hold ONE pass (stream ordering regression)
        d_counts.zero_()
        d_w.zero_()
        dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, 21, d_counts.data_ptr(),
                        d_w.data_ptr(), local=True, stream=stream)
    torch.cuda.synchronize()
    c = d_counts.cpu().numpy().astype(np.uint64)
    assert c[0] == host.total and c[1] == host.ambiguous and np.array_equal(c[2:], host.unique)
    np.testing.assert_allclose(d_w.cpu().numpy(), host.weights, rtol=W_RTOL)


def test_config2_full_size_vs_oracle():
    """BASELINE config 2 at full size (10 x 50 kb, 1M x 150 bp, k = 21): bit-exact vs the oracle, plus
    size-independent properties (shard additivity, read-order invariance, run-to-run determinism)."""
    c = synth.CONFIGS[2]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    reads = synth.make_reads(ref, c["n_reads"])
    G, k = c["n_variants"], c["k"]
    idx = FmIndex.build(ref.records, ref.groups, G, prefix_q=11, pair_steps=True, label_table=True)
    dev = DeviceIndex(idx)
    orc = Oracle(ref.records, ref.groups, G, k)
    full = _check(dev, orc, reads, k)
    assert full.total == c["n_reads"] * (150 - k + 1)
    again = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k)
    assert again.total == full.total and np.array_equal(again.unique, full.unique)
    # shards: [0, h) + [h, n) == whole
    h = reads.n // 3
    parts = []
    for lo, hi in ((0, h), (h, reads.n)):
        a, b = int(reads.offsets[lo]), int(reads.offsets[hi])
        parts.append(dev.scan(reads.seq[a:b].tobytes(), reads.qual[a:b].tobytes(),
                              reads.offsets[lo:hi + 1] - reads.offsets[lo], k=k))
    assert sum(p.total for p in parts) == full.total
    assert sum(p.ambiguous for p in parts) == full.ambiguous
    assert np.array_equal(parts[0].unique + parts[1].unique, full.unique)
    # read order
    perm = np.random.default_rng(7).permutation(reads.n)[:200_000]
    segs = [reads.seq[int(reads.offsets[i]):int(reads.offsets[i + 1])] for i in perm]
    qs = [reads.qual[int(reads.offsets[i]):int(reads.offsets[i + 1])] for i in perm]
    off = np.zeros(len(perm) + 1, np.uint64)
    off[1:] = np.cumsum([len(s) for s in segs])
    sub = synth.Reads(np.concatenate(segs), np.concatenate(qs), off, reads.variant[perm])
    _check(dev, orc, sub, k)
    u, t = dev.count_unique_kmers_per_group(k)
    ou, ot = orc.ref_unique()
    assert np.array_equal(u, ou) and np.array_equal(t, ot)
    # three-symbol planes, built on the GPU: same counts
    dev3 = DeviceIndex(FmIndex.build(ref.records, ref.groups, G, prefix_q=11, pair_steps=True, triple_steps=True,
                                     label_table=True, gpu_device=0))
    _check(dev3, orc, reads, k)


def test_label_table_saturation_gpu():
    """Single-group runs longer than 65535 SA positions: wide intervals take the rank fallback of classify()."""
    ref = synth.make_reference(2, 2, 120_000)
    reads = synth.make_reads(ref, 3_000, read_len=40)
    for groups, G in (([0, 0, 0, 0], 1), ([0, 0, 0, 1], 2)):
        idx = FmIndex.build(ref.records, groups, G, prefix_q=0, pair_steps=True, label_table=True)
        dev = DeviceIndex(idx)
        for k in (1, 3, 12):
            orc = Oracle(ref.records, groups, G, k)
            _check(dev, orc, reads, k)


@pytest.mark.parametrize("k", [21, 31, 70])
def test_long_and_mixed_length_reads(k):
    """Reads far longer than one wave pass (64 * NWIN windows) mixed with short ones: the flattened window cursor
    must carry a read across passes and units."""
    ref = synth.make_reference(3, 2, 40_000)
    long_reads = synth.make_reads(ref, 300, read_len=12_000, n_rate=0.0005, lowq_rate=0.002)
    short = synth.make_reads(ref, 2_000, read_len=100, short_frac=0.2, start_index=999)
    segs, quals = [], []
    for rd in (long_reads, short):
        for i in range(rd.n):
            a, b = int(rd.offsets[i]), int(rd.offsets[i + 1])
            segs.append(rd.seq[a:b])
            quals.append(rd.qual[a:b])
    order = np.random.default_rng(k).permutation(len(segs))
    segs = [segs[i] for i in order]
    quals = [quals[i] for i in order]
    off = np.zeros(len(segs) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in segs])
    reads = synth.Reads(np.concatenate(segs), np.concatenate(quals), off, np.zeros(len(segs), np.int32))
    for tri in (False, True):
        idx = FmIndex.build(ref.records, ref.groups, 3, prefix_q=10, pair_steps=True, triple_steps=tri,
                            label_table=True)
        dev = DeviceIndex(idx)
        orc = Oracle(ref.records, ref.groups, 3, k)
        _check(dev, orc, reads, k)
        _check(dev, orc, reads, k, local=True)


def test_config3_index_vs_oracle():
    """BASELINE config 3's index (50 variants x 3 isolates x 33 kb, k = 31) with every default the bench uses (GPU
    build, three-symbol planes, q = 12 tables, label table, 4 blocks/CU): all 10 M reads of the config bit-exact vs
    the oracle (default kernel), and the .dat pass. Oracle: ~0.4 GB table, ~10 s of 16 host threads."""
    c = synth.CONFIGS[3]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    reads = synth.make_reads(ref, c["n_reads"], n_rate=0.0005, lowq_rate=0.001)
    G, k = c["n_variants"], c["k"]
    idx = FmIndex.build(ref.records, ref.groups, G, prefix_q=12, pair_steps=True, triple_steps=True,
                        label_table="auto", gpu_device=0)
    assert idx.info().label_table == 1 and idx.info().triple_steps == 1
    dev = DeviceIndex(idx)
    assert dev.tuning("blocks_per_cu") == 4
    orc = Oracle(ref.records, ref.groups, G, k)
    got = _check_one(dev, orc, reads, k, 30, False, False)
    assert got.total > 0.9 * c["n_reads"] * (150 - k + 1)
    u, t = dev.count_unique_kmers_per_group(k)
    ou, ot = orc.ref_unique()
    assert np.array_equal(u, ou) and np.array_equal(t, ot)


@pytest.mark.parametrize("paired", [False, True])
def test_logical_shards_sum_to_unsharded(paired):
    """S in {1, 2, 4, 8} logical shards of the bench's deterministic read stream (rank r scans
    make_reads(start_index = r * n)), run one after another on one GPU, sum to the unsharded scan of all S * n reads
    (the quantity the RCCL all-reduce forms across ranks)."""
    ref = synth.make_reference(6, 2, 20_000)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 6, prefix_q=10, pair_steps=True, triple_steps=True,
                                    label_table=True, gpu_device=0))
    n = 4_000
    whole = synth.make_reads(ref, 8 * n, paired=paired)
    full = dev.scan(whole.seq.tobytes(), whole.qual.tobytes(), whole.offsets, k=21, paired=paired, local=True)
    for S in (1, 2, 4, 8):
        per = 8 * n // S
        tot, amb, U, W = 0, 0, np.zeros(6, np.uint64), np.zeros(6)
        for r in range(S):
            sh = synth.make_reads(ref, per, start_index=r * per, paired=paired)
            g = dev.scan(sh.seq.tobytes(), sh.qual.tobytes(), sh.offsets, k=21, paired=paired, local=True)
            tot, amb, U, W = tot + g.total, amb + g.ambiguous, U + g.unique, W + g.weights
        assert (tot, amb, U.tolist()) == (full.total, full.ambiguous, full.unique.tolist()), S
        np.testing.assert_allclose(W, full.weights, rtol=1e-12)
