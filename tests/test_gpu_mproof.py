"""GPU: m-mer absence proofs in the anchor-and-extend scan (k_scan_ax lane state 4).

When a window's anchor lookup finds nothing and the read's mismatch e against the previous run is known, the windows
that share e are proven absent by a few m-mer probes (an m-mer holding e whose bits are missing from the m-mer
filter lies inside each window it covers) instead of being deferred one by one to the Bloom-filter pass. A window
is dropped only on such a proof, so counts, ambiguity, weights and EM histograms must equal the oracle's and the
scan without proofs (tuning ax_mproof = 0) bit for bit, while the instrumented twin defers fewer windows.
These tests aim at the proof's edges: k near the smallest that takes proofs (k = m + 11: 24 on these 96 k-symbol
texts, m = 13; smaller k runs without them), error-dense reads (several
mismatches per read, deferred-list overflow), mismatches near read and segment ends, N in reads and references,
mismatches that are SNPs of another variant (the m-mer occurs: its windows stay deferred), paired and local scans."""
import numpy as np
import pytest

from oracle.oracle import Oracle
from speq_amd import DeviceIndex, EmHistogram, FmIndex, synth

pytestmark = pytest.mark.gpu


def scan(dev, reads, k, paired=False, local=False, mproof=1):
    dev.tune(ax_mproof=mproof)
    got = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, paired=paired, local=local)
    assert dev.tuning("last_kernel") == 3
    return got


def same(a, b, local):
    assert (a.total, a.ambiguous, a.unique.tolist()) == (b.total, b.ambiguous, b.unique.tolist())
    if local:
        np.testing.assert_allclose(a.weights, b.weights, rtol=1e-12, atol=0)


@pytest.fixture(scope="module")
def small():
    ref = synth.make_reference(4, 2, 6_000, ref_n_rate=0.002)
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=8, pair_steps=True, triple_steps=True)
    return ref, idx


@pytest.mark.parametrize("k", [21, 23, 24, 25, 31, 33, 45, 64, 70, 97, 128])
@pytest.mark.parametrize("err", [0.003, 0.03])
def test_proofs_match_oracle_and_no_proofs(small, k, err):
    ref, idx = small
    dev = DeviceIndex(idx)
    reads = synth.make_reads(ref, 2_000, err_rate=err, n_rate=0.002, lowq_rate=0.01, short_frac=0.05)
    orc = Oracle(ref.records, ref.groups, 4, k)
    T, amb, U, _ = orc.scan(reads.seq, reads.qual, reads.offsets)
    on = scan(dev, reads, k)
    assert (on.total, on.ambiguous, on.unique.tolist()) == (T, amb, U.tolist()), k
    same(on, scan(dev, reads, k, mproof=0), False)


@pytest.mark.parametrize("k", [21, 31, 70])
@pytest.mark.parametrize("paired", [False, True])
def test_proofs_local_and_paired(small, k, paired):
    ref, idx = small
    dev = DeviceIndex(idx)
    reads = synth.make_reads(ref, 1_500, err_rate=0.01, paired=paired, n_rate=0.001)
    orc = Oracle(ref.records, ref.groups, 4, k)
    for local in (False, True):
        T, amb, U, W = orc.scan(reads.seq, reads.qual, reads.offsets, paired=paired, local=local)
        on = scan(dev, reads, k, paired=paired, local=local)
        assert (on.total, on.ambiguous, on.unique.tolist()) == (T, amb, U.tolist()), (k, paired, local)
        if local:
            np.testing.assert_allclose(on.weights, W, rtol=1e-10, atol=0)
        same(on, scan(dev, reads, k, paired=paired, local=local, mproof=0), local)


@pytest.mark.parametrize("read_len", [60, 191, 193, 400])
def test_proofs_near_read_and_segment_ends(small, read_len):
    """Short reads (the probes' m-mers reach the read's last bases) and reads longer than a lane's 192-base segment
    (mismatches near the segment boundary)."""
    ref, idx = small
    dev = DeviceIndex(idx)
    reads = synth.make_reads(ref, 800, read_len=read_len, err_rate=0.02)
    for k in (24, 31, 58):
        if k > read_len:
            continue
        T, amb, U, _ = Oracle(ref.records, ref.groups, 4, k).scan(reads.seq, reads.qual, reads.offsets)
        on = scan(dev, reads, k)
        assert (on.total, on.ambiguous, on.unique.tolist()) == (T, amb, U.tolist()), (k, read_len)


def test_snp_mismatches_keep_their_windows():
    """Many variants that differ by SNPs: a run breaks at another variant's allele, whose m-mers occur in the texts;
    those windows must still be looked up (deferred), not dropped."""
    ref = synth.make_reference(24, 1, 3_000)
    idx = FmIndex.build(ref.records, ref.groups, 24, prefix_q=8, pair_steps=True, triple_steps=True)
    dev = DeviceIndex(idx)
    reads = synth.make_reads(ref, 3_000, err_rate=0.004)
    for k in (21, 31, 70):
        T, amb, U, _ = Oracle(ref.records, ref.groups, 24, k).scan(reads.seq, reads.qual, reads.offsets)
        on = scan(dev, reads, k)
        assert (on.total, on.ambiguous, on.unique.tolist()) == (T, amb, U.tolist()), k
        assert int(U.sum()) > 0


@pytest.mark.parametrize("paired", [False, True])
def test_em_histogram_equal_with_and_without_proofs(paired):
    ref = synth.make_reference(5, 3, 8_000, ref_n_rate=0.0005)
    idx = FmIndex.build(ref.records, ref.groups, 5, prefix_q=9, pair_steps=True, triple_steps=True)
    reads = synth.make_reads(ref, 6_000, paired=paired, n_rate=0.001, lowq_rate=0.005, err_rate=0.01)
    res = []
    for mproof in (1, 0):
        dev = DeviceIndex(idx)
        dev.tune(ax_mproof=mproof)
        em = EmHistogram(dev)
        r = em.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=31, paired=paired)
        em.finalize()
        res.append((r.total, r.ambiguous, r.unique.tolist(), em.info(),
                    em.step(np.linspace(5.0, 30.0, 5), [3] * 5, r.unique).tolist()))
    assert res[0] == res[1]


def test_config2_fewer_deferred_windows():
    """Config 2's index, 200 k reads at 0.5 % errors: the instrumented twin defers fewer windows with the proofs
    (k = 31, 70; k = 21 takes none at m = 14), and both scans (and the ordinary kernel) agree with the oracle."""
    import torch

    c = synth.CONFIGS[2]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=10, pair_steps=True, triple_steps=True)
    reads = synth.make_reads(ref, 200_000, err_rate=0.005)
    G = c["n_variants"]
    d_seq = torch.from_numpy(reads.seq).cuda()
    d_qual = torch.from_numpy(reads.qual).cuda()
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
    dev = DeviceIndex(idx)
    for k in (31, 70):
        T, amb, U, _ = Oracle(ref.records, ref.groups, G, k).scan(reads.seq, reads.qual, reads.offsets)
        deferred = {}
        for mproof in (1, 0):
            dev.tune(ax_mproof=mproof)
            cnt = torch.zeros(G + 2, dtype=torch.int64, device="cuda")
            st = dev.scan_device_stats(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, k,
                                       cnt.data_ptr())
            c_ = cnt.cpu().numpy()
            assert (int(c_[0]), int(c_[1]), c_[2:].tolist()) == (T, amb, U.tolist()), (k, mproof)
            deferred[mproof] = st["deferred"]
            got = scan(dev, reads, k, mproof=mproof)
            assert (got.total, got.ambiguous, got.unique.tolist()) == (T, amb, U.tolist()), (k, mproof)
        assert deferred[1] < 0.5 * deferred[0], (k, deferred)
