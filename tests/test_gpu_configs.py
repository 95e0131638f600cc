"""GPU parity at the indexes of BASELINE configs 4 and 5 (the multi-GPU configs), one GPU's share each.

Config 5: 200 variants x 5 isolates x 100 kb (texts fwd + rc: 200 M symbols), paired 2 x 150 bp, k = 31. Config 4:
config 3's 50-variant index, 100 M reads over 8 GPUs -> one rank's 12.5 M-read shard (rank 7: start_index = 87.5 M
of the deterministic read stream, exactly what `bench.py` rank 7 scans). Every kernel (anchor-and-extend, k-mer
table, LF steps) is checked bit-exactly against the hash-map oracle with the bench's own defaults (GPU index build,
q = 12 tables, three-symbol planes, label table by size, blocks/CU by footprint). Reference loops:
/root/reference/src/fm_scanner.cpp:153-196 (single), :709-729 (paired global), :963-995 (paired local),
:1503-1539 (.dat pass).

Oracle budget (oracle/kmer_oracle.c, all host threads): config 5 — 13.6 GB of host memory (a 2^29-slot table over
200 M reference windows), build ~20-30 s, .dat pass ~8 s, 200 k pairs per scan ~4 s; config 4 shard — 0.4 GB of
table + 3.8 GB of reads, scan of 1.5 G windows ~10-20 s on 16 threads.
"""
import numpy as np
import pytest

from oracle.oracle import Oracle
from speq_amd import DeviceIndex, FmIndex, synth

pytestmark = pytest.mark.gpu
W_RTOL = 1e-10  # fp64 sums in a different order (see test_gpu_parity.py)

# anchor-and-extend (default), the k-mer-table kernel, LF steps with 1 and 2 windows per lane
VARIANTS = [dict(ax_scan=1, kmer_table=1, ilp=1), dict(ax_scan=0, kmer_table=1, ilp=1),
            dict(ax_scan=0, kmer_table=0, ilp=1), dict(ax_scan=0, kmer_table=0, ilp=2)]
DEFAULT = dict(ax_scan=1, kmer_table=1, ilp=1, ilp_local=1)


def _scan_all(dev, reads, k, paired, local, expect, variants=VARIANTS):
    T, amb, U, W = expect
    for v in variants:
        dev.tune(ilp=v["ilp"], ilp_local=v["ilp"], kmer_table=v["kmer_table"], ax_scan=v["ax_scan"])
        got = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, paired=paired, local=local)
        assert (got.total, got.ambiguous) == (T, amb), v
        assert np.array_equal(got.unique, U), v
        if local:
            np.testing.assert_allclose(got.weights, W, rtol=W_RTOL, atol=0)
    dev.tune(**DEFAULT)


@pytest.fixture(scope="module")
def cfg5():
    c = synth.CONFIGS[5]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True, triple_steps=True,
                        label_table="auto", gpu_device=0)
    dev = DeviceIndex(idx)
    orc = Oracle(ref.records, ref.groups, c["n_variants"], c["k"])
    yield c, ref, idx, dev, orc
    dev.close()


def test_config5_index_defaults(cfg5):
    """The bench's defaults at config 5: three-symbol planes, label table, 3 blocks/CU (planes beyond the 256 MB
    Infinity Cache), per-k structures for k = 31 built on the device."""
    c, ref, idx, dev, orc = cfg5
    info = idx.info()
    assert info.n > 200_000_000 and info.label_table == 1 and info.triple_steps == 1
    assert dev.tuning("blocks_per_cu") == 3
    prep = dev.prepare(c["k"])
    assert prep["distinct_kmers"] > 10_000_000


@pytest.mark.parametrize("local", [False, True])
def test_config5_paired_vs_oracle(cfg5, local):
    """200 k read pairs of config 5 (N bases and low-quality bases mixed in), paired k = 31, every kernel."""
    c, ref, idx, dev, orc = cfg5
    reads = synth.make_reads(ref, 200_000, paired=True, n_rate=0.0005, lowq_rate=0.001, start_index=12_345)
    expect = orc.scan(reads.seq, reads.qual, reads.offsets, paired=True, local=local)
    assert expect[0] > 0.9 * 400_000 * (150 - c["k"] + 1)
    _scan_all(dev, reads, c["k"], True, local, expect)


def test_config5_single_end_and_dat_vs_oracle(cfg5):
    """The same index scanned single-end (mates as independent reads) and the .dat reference-uniqueness pass."""
    c, ref, idx, dev, orc = cfg5
    reads = synth.make_reads(ref, 100_000, paired=True, start_index=777)
    expect = orc.scan(reads.seq, reads.qual, reads.offsets, paired=False)
    _scan_all(dev, reads, c["k"], False, False, expect, VARIANTS[:3])
    u, t = dev.count_unique_kmers_per_group(c["k"])
    ou, ot = orc.ref_unique()
    assert np.array_equal(u, ou) and np.array_equal(t, ot)
    assert int(t.sum()) == sum(2 * max(0, len(r) - c["k"] + 1) for r in ref.records)


def test_config4_rank_shard_vs_oracle():
    """Config 4's per-rank shard: 12.5 M reads of rank 7 (start_index = 7 x 12.5 M) on config 3's index, k = 31."""
    c = synth.CONFIGS[4]
    ranks = 8
    per_rank = c["n_reads"] // ranks
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True, triple_steps=True,
                        label_table="auto", gpu_device=0)
    dev = DeviceIndex(idx)
    assert dev.tuning("blocks_per_cu") == 4
    orc = Oracle(ref.records, ref.groups, c["n_variants"], c["k"])
    reads = synth.make_reads(ref, per_rank, start_index=(ranks - 1) * per_rank, n_rate=0.0002, lowq_rate=0.0005)
    assert reads.n == per_rank
    expect = orc.scan(reads.seq, reads.qual, reads.offsets)
    assert expect[0] > 0.9 * per_rank * (150 - c["k"] + 1)
    _scan_all(dev, reads, c["k"], False, False, expect, VARIANTS[:3])
    dev.close()
