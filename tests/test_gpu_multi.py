"""GPU: several replicas of one index in one process: reads dealt across replicas
(speq_scan_fastq_multi), the .dat pass split over them (speq_ref_unique_multi) and per-replica EM histograms folded
with speq_em_merge give exactly the single-replica results. Replicas share GPU 0 here (logical shards) and also use
distinct GPUs when more than one is visible. Integer counters and EM histograms bit-exact; W rtol 1e-12 (the
per-replica fp64 sums are added in replica order)."""
import ctypes as C

import numpy as np
import pytest

from speq_amd import DeviceIndex, EmHistogram, FmIndex, Node, SpeqError, lib, synth
from speq_amd._lib import SPEQ_E_ARG
from test_gpu_stream import same, split, write_fastq

pytestmark = pytest.mark.gpu


def device_sets():
    n = lib().speq_device_count()
    sets = [[0], [0, 0], [0, 0, 0]]
    if n >= 2:
        sets.append(list(range(min(n, 8))))
    return sets


@pytest.fixture(scope="module")
def data():
    ref = synth.make_reference(5, 2, 20_000, ref_n_rate=0.0005)
    idx = FmIndex.build(ref.records, ref.groups, 5, prefix_q=10, pair_steps=True, triple_steps=True)
    single = synth.make_reads(ref, 150_000, n_rate=0.001, lowq_rate=0.005, short_frac=0.01)
    pairs = synth.make_reads(ref, 40_000, paired=True, n_rate=0.001, lowq_rate=0.005)
    return ref, idx, single, pairs


def _files(tmp_path, reads, paired, **fmt):
    seqs, quals = split(reads)
    if not paired:
        write_fastq(tmp_path / "s.fq", seqs, quals, **fmt)
        return str(tmp_path / "s.fq"), None
    write_fastq(tmp_path / "p1.fq", seqs[0::2], quals[0::2], **fmt)
    write_fastq(tmp_path / "p2.fq", seqs[1::2], quals[1::2], **fmt)
    return str(tmp_path / "p1.fq"), str(tmp_path / "p2.fq")


@pytest.mark.parametrize("devices", device_sets(), ids=lambda d: "-".join(map(str, d)))
@pytest.mark.parametrize("paired", [False, True])
@pytest.mark.parametrize("local", [False, True])
def test_node_stream_equals_single_replica(tmp_path, data, devices, paired, local):
    ref, idx, single, pairs = data
    reads = pairs if paired else single
    p1, p2 = _files(tmp_path, reads, paired)
    one = DeviceIndex(idx, 0)
    em1 = EmHistogram(one)
    exp = em1.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21, paired=paired, local=local)
    em1.finalize()
    node = Node(idx, devices)
    ems = node.em_histograms()
    got, st = node.scan_fastq(p1, p2, k=21, local=local, threads=6, ems=ems)
    same(got, exp, local)
    assert st["records"] == reads.n and st["bases"] == int(reads.offsets[-1])
    em = Node.merge_em(ems)
    em.finalize()
    assert em.info() == em1.info()
    p = np.array([5.0, 10.0, 20.0, 30.0, 35.0])
    np.testing.assert_array_equal(em.step(p, [2, 2, 2, 2, 2], got.unique), em1.step(p, [2, 2, 2, 2, 2], exp.unique))
    for e in ems:
        e.close()
    node.close()


@pytest.mark.parametrize("devices", device_sets(), ids=lambda d: "-".join(map(str, d)))
@pytest.mark.parametrize("k", [15, 21, 31, 70])
def test_node_ref_unique_equals_single_replica(data, devices, k):
    ref, idx, _, _ = data
    one = DeviceIndex(idx, 0)
    node = Node(idx, devices)
    u1, t1 = one.count_unique_kmers_per_group(k)
    u, t = node.count_unique_kmers_per_group(k)
    assert u.tolist() == u1.tolist() and t.tolist() == t1.tolist()
    node.close()


def test_node_restart_clears_every_replica(tmp_path, monkeypatch, data):
    """A layout the parallel cut rejects late in the file restarts the stream sequentially: the counters and EM
    histograms of EVERY replica must be cleared first."""
    ref, idx, single, _ = data
    seqs, quals = split(single)
    p = tmp_path / "r.fq"
    write_fastq(p, seqs, quals)
    d = p.read_bytes()
    cut = d.index(b"\n@read", len(d) * 5 // 6) + 1
    p.write_bytes(d[:cut] + b"@w\nACGTACGTAC\nGTACGTACGT\n+\nIIIIIIIIII\nIIIIIIIIII\n" + d[cut:])
    one = DeviceIndex(idx, 0)
    em1 = EmHistogram(one)
    exp = em1.scan(single.seq.tobytes(), single.qual.tobytes(), single.offsets, k=21)
    em1.finalize()
    monkeypatch.setenv("SPEQ_SPLIT_CUT", "1")
    node = Node(idx, [0, 0, 0])
    ems = node.em_histograms()
    got, st = node.scan_fastq(str(p), k=21, threads=6, ems=ems)
    same(got, exp, False)
    assert st["records"] == single.n + 1
    em = Node.merge_em(ems)
    em.finalize()
    assert em.info() == em1.info()
    node.close()


def test_node_rejects_mixed_indexes(data):
    ref, idx, _, _ = data
    other = FmIndex.build(ref.records[:4], ref.groups[:4], 5, prefix_q=8)
    a, b = DeviceIndex(idx, 0), DeviceIndex(other, 0)
    with pytest.raises(SpeqError, match="different indexes"):
        Node.merge_em([EmHistogram(a), EmHistogram(b)])
    arr = (C.c_void_p * 2)(a.handle.value, b.handle.value)
    u, t = np.zeros(5, np.uint64), np.zeros(5, np.uint64)
    p64 = C.POINTER(C.c_uint64)
    assert lib().speq_ref_unique_multi(arr, 2, 21, u.ctypes.data_as(p64), t.ctypes.data_as(p64)) == SPEQ_E_ARG
    assert b"different indexes" in lib().speq_last_error()
