"""GPU: the staged anchor-and-extend scan (k_scan_axq, tuning ax_stager = 1) against the CPU oracle.

A stager wave per workgroup stages pieces (read segments of at most 160 bases, mates) into the consumer waves' ready
rings; units of several pieces (mate pairs, long reads) are finished by whichever lanes scan their pieces, through a
per-unit ring record of the first group / another group seen / pieces left. These tests aim at that: paired scans
(ambiguity across two lanes), reads of 161-1000 bases (up to seven pieces per unit, units split over stager passes),
reads shorter than k (empty pieces), error-heavy reads (deferred-list overflow), tiny grids (pools of thousands of
units: many passes, ring wrap-around), EM histograms and the instrumented twin. Integer counters bit-exact."""
import numpy as np
import pytest

from oracle.oracle import Oracle
from speq_amd import DeviceIndex, EmHistogram, FmIndex, synth

pytestmark = pytest.mark.gpu


def check(dev, orc, seq, qual, off, k, paired=False):
    got = dev.scan(seq.tobytes(), qual.tobytes(), off, k=k, paired=paired)
    T, amb, U, _ = orc.scan(seq, qual, off, paired=paired)
    assert (got.total, got.ambiguous, got.unique.tolist()) == (T, amb, U.tolist()), (k, paired)
    assert dev.tuning("last_kernel") == 3
    return got


@pytest.fixture(scope="module")
def small():
    ref = synth.make_reference(4, 2, 6_000, ref_n_rate=0.002)
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=8, pair_steps=True, triple_steps=True)
    return ref, idx


def staged(idx, **tune):
    dev = DeviceIndex(idx)
    dev.tune(ax_stager=1, **tune)
    assert dev.tuning("ax_stager") == 1
    return dev


@pytest.mark.parametrize("k", [1, 5, 21, 31, 33, 64, 65, 97, 128])
@pytest.mark.parametrize("paired", [False, True])
def test_word_boundary_k(small, k, paired):
    ref, idx = small
    dev = staged(idx)
    reads = synth.make_reads(ref, 1_500, n_rate=0.003, lowq_rate=0.01, err_rate=0.003, paired=paired,
                             short_frac=0.0 if paired else 0.05)
    check(dev, Oracle(ref.records, ref.groups, 4, k), reads.seq, reads.qual, reads.offsets, k, paired)


@pytest.mark.parametrize("read_len", [159, 160, 161, 250, 400, 1000])
@pytest.mark.parametrize("paired", [False, True])
def test_multi_piece_units(small, read_len, paired):
    ref, idx = small
    dev = staged(idx)
    reads = synth.make_reads(ref, 300, read_len=read_len, err_rate=0.002, n_rate=0.001, paired=paired,
                             fragment=2 * read_len + 50)
    for k in (21, 70, 128):
        check(dev, Oracle(ref.records, ref.groups, 4, k), reads.seq, reads.qual, reads.offsets, k, paired)


def test_mixed_lengths_and_short_reads(small):
    """Reads of 5-700 bases in one batch: single-piece units, units of up to five pieces and reads with no window."""
    ref, idx = small
    rng = np.random.default_rng(3)
    parts = []
    for _ in range(3_000):
        rec = ref.records[int(rng.integers(len(ref.records)))]
        L = int(rng.choice([5, 20, 90, 150, 161, 320, 700]))
        s0 = int(rng.integers(0, len(rec) - L))
        parts.append(np.frombuffer(rec[s0:s0 + L], dtype=np.uint8))
    seq = np.concatenate(parts)
    off = np.concatenate([[0], np.cumsum([p.size for p in parts])]).astype(np.uint64)
    qual = np.full(seq.size, ord("I"), dtype=np.uint8)
    qual[rng.random(seq.size) < 0.005] = ord("#")
    dev = staged(idx)
    for k in (21, 45):
        check(dev, Oracle(ref.records, ref.groups, 4, k), seq, qual, off, k)
        check(dev, Oracle(ref.records, ref.groups, 4, k), seq, qual, off[: 2 * 1_500 + 1], k, paired=True)


def test_error_heavy_and_random_reads(small):
    ref, idx = small
    rng = np.random.default_rng(5)
    n, L = 3_000, 150
    rnd = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n * L)
    noisy = synth.make_reads(ref, n, err_rate=0.05)
    clean = synth.make_reads(ref, n)
    seq = np.concatenate([rnd, noisy.seq, clean.seq])
    qual = np.full(seq.size, ord("I"), dtype=np.uint8)
    off = np.arange(0, seq.size + 1, L, dtype=np.uint64)
    dev = staged(idx)
    for k in (11, 21, 31, 45, 70, 100):
        check(dev, Oracle(ref.records, ref.groups, 4, k), seq, qual, off, k)


@pytest.mark.parametrize("grid", [1, 2, 7, 65535])
def test_small_grids_many_passes(small, grid):
    """One to seven workgroups: each stager stages thousands of units over many passes (ring records reused many
    times), paired and single-end."""
    ref, idx = small
    dev = staged(idx, grid_blocks_ax=grid)
    for paired in (False, True):
        reads = synth.make_reads(ref, 20_000, err_rate=0.003, paired=paired)
        check(dev, Oracle(ref.records, ref.groups, 4, 31), reads.seq, reads.qual, reads.offsets, 31, paired)


@pytest.mark.parametrize("paired", [False, True])
def test_em_histogram_equals_unstaged(paired):
    ref = synth.make_reference(5, 3, 8_000, ref_n_rate=0.0005)
    idx = FmIndex.build(ref.records, ref.groups, 5, prefix_q=9, pair_steps=True, triple_steps=True)
    reads = synth.make_reads(ref, 15_000, paired=paired, n_rate=0.001, lowq_rate=0.005, err_rate=0.004)
    res = []
    for stager in (0, 1):
        dev = DeviceIndex(idx)
        dev.tune(ax_stager=stager)
        em = EmHistogram(dev)
        r = em.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=31, paired=paired)
        em.finalize()
        res.append((r.total, r.ambiguous, r.unique.tolist(), em.info(),
                    em.step(np.linspace(5.0, 30.0, 5), [3] * 5, r.unique).tolist()))
    assert res[0] == res[1]


def test_config2_size_and_stats_twin():
    """Config 2's index and 300 k reads: the staged scan, its instrumented twin and the unstaged kernel agree with
    the oracle; the twin's staged chunk count equals the reads' chunk count."""
    c = synth.CONFIGS[2]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=10, pair_steps=True, triple_steps=True)
    reads = synth.make_reads(ref, 300_000, err_rate=0.002)
    orc = Oracle(ref.records, ref.groups, c["n_variants"], 21)
    dev = staged(idx)
    check(dev, orc, reads.seq, reads.qual, reads.offsets, 21)
    import torch
    d_seq = torch.from_numpy(reads.seq).cuda()
    d_qual = torch.from_numpy(reads.qual).cuda()
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
    cnt = torch.zeros(c["n_variants"] + 2, dtype=torch.int64, device="cuda")
    st = dev.scan_device_stats(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, 21, cnt.data_ptr())
    T, amb, U, _ = orc.scan(reads.seq, reads.qual, reads.offsets)
    c_ = cnt.cpu().numpy()
    assert (int(c_[0]), int(c_[1]), c_[2:].tolist()) == (T, amb, U.tolist())
    starts = reads.offsets[:-1].astype(np.int64)
    ends = reads.offsets[1:].astype(np.int64)
    assert st["chunks"] == int(((ends + 15) // 16 - starts // 16).sum())
    assert st["segments"] == reads.n
