"""GPU: the one-process-per-GPU decomposition of `speq scan` (include/speq_scan.h, "one process per
GPU"), run shard by shard on one GPU. Rank r of W scans the FASTQ blocks b % W == r (speq_scan_fastq_shard) and
the r-th slice of the reference windows (speq_ref_unique_shard); the RCCL all-reduces then sum the shards. Here the
sums are taken on the host (one GPU cannot hold two RCCL ranks), and the product's RCCL calls run at nranks = 1.
The sums must equal the one-process scan bit for bit (fp64 weights: rtol 1e-12, different association). Reference
sums replaced: /root/reference/src/fm_scanner.cpp:224-233, :1544-1557."""
import numpy as np
import pytest

from speq_amd import Comm, DeviceIndex, EmHistogram, FmIndex, Node, SpeqError, synth

from test_gpu_stream import split, write_fastq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup(tmp_path_factory):
    d = tmp_path_factory.mktemp("ranks")
    ref = synth.make_reference(6, 2, 20_000)
    reads = synth.make_reads(ref, 100_000, read_len=100, n_rate=0.001, lowq_rate=0.002)  # 4 blocks of 32 k records
    seqs, quals = split(reads)
    write_fastq(d / "r.fq", seqs, quals)
    # a wrapped record three quarters in: the parallel cut cannot take the file
    data = (d / "r.fq").read_bytes()
    cut = data.index(b"\n@read", len(data) * 3 // 4) + 1
    (d / "w.fq").write_bytes(data[:cut] + b"@w\nACGTACGTAC\nGTAC\n+\nIIIIIIIIII\nIIII\n" + data[cut:])
    pairs = synth.make_reads(ref, 40_000, read_len=100, paired=True)
    ps, pq = split(pairs)
    write_fastq(d / "p1.fq", ps[0::2], pq[0::2])
    write_fastq(d / "p2.fq", ps[1::2], pq[1::2])
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 6, prefix_q=10, pair_steps=True, triple_steps=True,
                                    gpu_device=0))
    yield d, ref, dev
    dev.close()


def _sum(parts):
    tot = sum(p.total for p, _ in parts)
    amb = sum(p.ambiguous for p, _ in parts)
    U = sum(p.unique for p, _ in parts)
    W = sum(p.weights for p, _ in parts) if parts[0][0].weights is not None else None
    return tot, amb, U, W


@pytest.mark.parametrize("files", [("r.fq", None), ("p1.fq", "p2.fq")])
@pytest.mark.parametrize("local", [False, True])
def test_fastq_shards_sum_to_one_scan(setup, files, local):
    d, ref, dev = setup
    p1, p2 = str(d / files[0]), str(d / files[1]) if files[1] else None
    whole, wst = dev.scan_fastq(p1, p2, k=21, local=local, threads=4)
    for W in (1, 2, 3):
        for cut in (0, 1):
            parts = [dev.scan_fastq_shard(p1, p2, 21, r, W, cut=cut, local=local, threads=4) for r in range(W)]
            tot, amb, U, Wt = _sum(parts)
            assert (tot, amb, U.tolist()) == (whole.total, whole.ambiguous, whole.unique.tolist()), (W, cut)
            assert sum(st["records"] for _, st in parts) == wst["records"]
            if local:
                np.testing.assert_allclose(Wt, whole.weights, rtol=1e-12)


def test_parallel_cut_retry_and_sequential_fallback(setup):
    d, ref, dev = setup
    p = str(d / "w.fq")
    whole, _ = dev.scan_fastq(p, k=21, threads=4)
    retries = 0
    for r in range(2):
        try:
            dev.scan_fastq_shard(p, None, 21, r, 2, cut=1)
        except SpeqError as e:
            assert e.code == -6
            retries += 1
    assert retries >= 1
    parts = [dev.scan_fastq_shard(p, None, 21, r, 2, cut=0) for r in range(2)]
    tot, amb, U, _ = _sum(parts)
    assert (tot, amb, U.tolist()) == (whole.total, whole.ambiguous, whole.unique.tolist())
    with pytest.raises(SpeqError):
        dev.scan_fastq_shard(p, None, 21, 0, 2, cut=-1)  # several shards must agree on the cut


@pytest.mark.parametrize("k", [15, 21, 31, 70])
def test_dat_shards_sum_to_one_pass(setup, k):
    d, ref, dev = setup
    u, t = dev.count_unique_kmers_per_group(k)
    for W in (2, 3, 8):
        us, ts = zip(*(dev.count_unique_kmers_per_group_shard(k, r, W) for r in range(W)))
        assert np.array_equal(sum(us), u) and np.array_equal(sum(ts), t), (k, W)


def test_em_histograms_of_shards_and_rccl_single_rank(setup):
    """Shard histograms merged equal the one-scan histogram; speq_em_allreduce over a one-rank communicator leaves a
    histogram unchanged."""
    d, ref, dev = setup
    p = str(d / "r.fq")
    em_all = EmHistogram(dev)
    whole, _ = dev.scan_fastq(p, k=21, em=em_all, threads=4)
    ems = [EmHistogram(dev) for _ in range(3)]
    parts = [dev.scan_fastq_shard(p, None, 21, r, 3, cut=1, em=ems[r]) for r in range(3)]
    merged = Node.merge_em(ems)
    comm = Comm(1, 0, Comm.unique_id())
    merged.allreduce(comm)
    comm.close()
    merged.finalize()
    em_all.finalize()
    assert merged.info() == em_all.info()
    U = sum(pt.unique for pt, _ in parts)
    pct = np.linspace(5.0, 30.0, 6)
    cnt = [2] * 6
    np.testing.assert_allclose(merged.step(pct, cnt, U), em_all.step(pct, cnt, whole.unique), rtol=1e-12)


@pytest.mark.parametrize("world", [2, 3])
def test_em_allreduce_over_host_transport(setup, tmp_path, world):
    """The product's rank exchange with ranks sharing one GPU (speq_comm_connect picks host sockets): each rank
    (a thread here) scans its FASTQ shard into its own histogram, speq_em_allreduce sums multiplicities and takes
    the max of interval ends; positions a rank never wrote hold 0 (speq_em_create zeroes them, advisor finding), so
    every rank ends with the one-scan histogram, and the counters summed by speq_allreduce_host equal one scan's."""
    import threading
    d, ref, dev = setup
    p = str(d / "r.fq")
    em_all = EmHistogram(dev)
    whole, _ = dev.scan_fastq(p, k=21, em=em_all, threads=4)
    em_all.finalize()
    path = str(tmp_path / "rdzv")
    res, errs = {}, []

    def rank(r):
        try:
            c = Comm.connect(world, r, path, device=0, transport=Comm.AUTO, timeout_s=120)
            assert c.transport == Comm.HOST  # every rank on GPU 0
            em = EmHistogram(dev)
            part, _ = dev.scan_fastq_shard(p, None, 21, r, world, cut=1, em=em)
            counts = np.concatenate([[part.total, part.ambiguous], part.unique]).astype(np.uint64)
            c.allreduce_host(counts, device=0)
            em.allreduce(c)
            c.close()
            em.finalize()
            pct = np.linspace(5.0, 30.0, 6)
            res[r] = (counts, em.info(), em.step(pct, [2] * 6, counts[2:]))
            em.close()
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    assert not errs, errs
    pct = np.linspace(5.0, 30.0, 6)
    ref_step = em_all.step(pct, [2] * 6, whole.unique)
    for r in range(world):
        counts, info, step = res[r]
        assert counts.tolist() == [whole.total, whole.ambiguous] + whole.unique.tolist()
        assert info == em_all.info()
        np.testing.assert_allclose(step, ref_step, rtol=1e-12)
