"""GPU: the streaming front end (speq_scan_fastq: FASTQ/.gz reader thread -> parser threads -> pinned slots -> H2D on
a copy stream overlapped with k_scan) and the speq_pipeline_* slot API give exactly the counters of the in-memory
scan (and of the golden vectors). Integer counters bit-exact; W rtol 1e-12 (block order changes the fp64 sum order)."""
import gzip
import os

import numpy as np
import pytest

from golden_io import CASES, Case
from speq_amd import DeviceIndex, EmHistogram, FmIndex, Pipeline, SpeqError, synth

pytestmark = pytest.mark.gpu


def write_fastq(path, seqs, quals, wrap=0, crlf=False, blank=False, gz=False):
    nl = "\r\n" if crlf else "\n"
    out = []
    for i, (s, q) in enumerate(zip(seqs, quals)):
        s, q = s.decode(), q.decode()
        out.append(f"@read{i} extra words{nl}")
        if wrap:
            out += [s[j:j + wrap] + nl for j in range(0, max(len(s), 1), wrap)] if s else [nl]
            out.append("+" + nl)
            out += [q[j:j + wrap] + nl for j in range(0, len(q), wrap)]
        else:
            out += [s + nl, "+read" + nl, q + nl]
        if blank and i % 7 == 3:
            out.append(nl)
    data = "".join(out).encode()
    with (gzip.open(path, "wb", compresslevel=1) if gz else open(path, "wb")) as f:
        f.write(data)


def split(reads):
    seqs, quals = [], []
    for i in range(len(reads.offsets) - 1):
        a, b = int(reads.offsets[i]), int(reads.offsets[i + 1])
        seqs.append(reads.seq[a:b].tobytes())
        quals.append(reads.qual[a:b].tobytes())
    return seqs, quals


def same(a, b, local):
    assert (a.total, a.ambiguous, a.unique.tolist()) == (b.total, b.ambiguous, b.unique.tolist())
    if local:
        np.testing.assert_allclose(a.weights, b.weights, rtol=1e-12)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("gz", [False, True])
def test_scan_fastq_matches_golden(tmp_path, name, gz):
    c = Case(name)
    dev = DeviceIndex(FmIndex.build(c.records, c.groups, c.G, prefix_q=4))
    p1 = os.path.join(c.dir, "reads_1.fq")
    p2 = os.path.join(c.dir, "reads_2.fq") if c.paired else None
    if gz:
        for src in filter(None, [p1, p2]):
            with open(src, "rb") as f, gzip.open(tmp_path / (os.path.basename(src) + ".gz"), "wb") as g:
                g.write(f.read())
        p1 = str(tmp_path / "reads_1.fq.gz")
        p2 = str(tmp_path / "reads_2.fq.gz") if c.paired else None
    for k in c.ks:
        for mode in ("global", "local"):
            g = c.exp["by_k"][str(k)][mode]
            r, st = dev.scan_fastq(p1, p2, k=k, phred_cutoff=c.cutoff, local=mode == "local", threads=3)
            assert (r.total, r.ambiguous, r.unique.tolist()) == (g["T"], g["ambiguous"], g["U"])
            if mode == "local":
                np.testing.assert_allclose(r.weights, g["W"], rtol=1e-12)
            assert st["records"] == len(c.offsets) - 1


@pytest.mark.parametrize("pinned", ["register", "hostmalloc"])
def test_slot_memory_registered_or_host_malloced(tmp_path, monkeypatch, pinned):
    """The slots' page-locked host memory (registered aligned allocations, or hipHostMalloc where registration is
    refused: SPEQ_PINNED=hostmalloc) gives the in-memory scan's counters."""
    monkeypatch.setenv("SPEQ_PINNED", pinned)
    ref = synth.make_reference(3, 2, 15_000)
    reads = synth.make_reads(ref, 60_000, n_rate=0.001, lowq_rate=0.005)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 3, prefix_q=9))  # (a new replica: new slots)
    seqs, quals = split(reads)
    write_fastq(tmp_path / "r1.fq", seqs, quals)
    for local in (False, True):
        exp = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21, local=local)
        got, st = dev.scan_fastq(str(tmp_path / "r1.fq"), None, k=21, local=local, threads=4)
        same(got, exp, local)
        assert st["records"] == reads.n


@pytest.mark.parametrize("fmt", [dict(), dict(wrap=37, crlf=True, blank=True), dict(gz=True, wrap=60),
                                 dict(crlf=True), dict(gz=True)])
@pytest.mark.parametrize("paired", [False, True])
@pytest.mark.parametrize("pack", ["0", "1"])
def test_scan_fastq_formats_match_in_memory(tmp_path, monkeypatch, fmt, paired, pack):
    """FASTQ streams (plain / gzip, four-line or wrapped / CRLF / blank lines) equal the in-memory scan, with the
    records parsed on the GPU or (SPEQ_FASTQ_PACK=1) packed on the host; wrapped files take the general parser."""
    monkeypatch.setenv("SPEQ_FASTQ_PACK", pack)
    ref = synth.make_reference(4, 2, 20_000, ref_n_rate=0.0005)
    n = 150_000 if not fmt else 40_000  # > one 131072-record block for the plain case
    reads = synth.make_reads(ref, n // (2 if paired else 1), paired=paired, n_rate=0.001, lowq_rate=0.005,
                             short_frac=0.0 if paired else 0.02)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 4, prefix_q=10))
    seqs, quals = split(reads)
    if paired:
        write_fastq(tmp_path / "r1.fq", seqs[0::2], quals[0::2], **fmt)
        write_fastq(tmp_path / "r2.fq", seqs[1::2], quals[1::2], **fmt)
        p1, p2 = str(tmp_path / "r1.fq"), str(tmp_path / "r2.fq")
    else:
        write_fastq(tmp_path / "r1.fq", seqs, quals, **fmt)
        p1, p2 = str(tmp_path / "r1.fq"), None
    for local in (False, True):
        exp = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21, paired=paired, local=local)
        for threads in (1, 6):
            got, st = dev.scan_fastq(p1, p2, k=21, local=local, threads=threads)
            same(got, exp, local)
            assert st["records"] == reads.n and st["bases"] == int(reads.offsets[-1])


def test_paired_files_of_unequal_length_zip_to_the_shorter(tmp_path):
    ref = synth.make_reference(3, 1, 5_000)
    reads = synth.make_reads(ref, 500, paired=True)
    seqs, quals = split(reads)
    write_fastq(tmp_path / "r1.fq", seqs[0::2], quals[0::2])
    write_fastq(tmp_path / "r2.fq", seqs[1:401:2], quals[1:401:2])  # 200 mates only
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 3, prefix_q=6))
    got, st = dev.scan_fastq(str(tmp_path / "r1.fq"), str(tmp_path / "r2.fq"), k=21)
    exp = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets[:401], k=21, paired=True)
    same(got, exp, False)
    assert st["records"] == 400


def test_scan_fastq_errors(tmp_path):
    ref = synth.make_reference(2, 1, 2_000)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 2, prefix_q=4))
    (tmp_path / "a.fa").write_text(">r\nACGT\n")
    (tmp_path / "trunc.fq").write_text("@r\nACGTACGT\n")
    (tmp_path / "mismatch.fq").write_text("@r\nACGTACGT\n+\nIIII\n")
    (tmp_path / "bad.fq").write_text("@r\nACGT\n+\nIIII\nxyz\n")
    for f, msg in (("a.fa", "qualities are required"), ("trunc.fq", "truncated"), ("missing.fq", "cannot open"),
                   ("bad.fq", "malformed")):
        with pytest.raises(SpeqError, match=msg):
            dev.scan_fastq(str(tmp_path / f), k=3)
    with pytest.raises(SpeqError, match="mismatch"):
        dev.scan_fastq(str(tmp_path / "mismatch.fq"), k=3)
    (tmp_path / "empty.fq").write_text("")
    r, st = dev.scan_fastq(str(tmp_path / "empty.fq"), k=3)
    assert r.total == 0 and st["records"] == 0


@pytest.mark.parametrize("local", [False, True])
def test_pipeline_slots_equal_one_scan(local):
    ref = synth.make_reference(5, 1, 8_000)
    reads = synth.make_reads(ref, 6_000, n_rate=0.001, short_frac=0.05)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 5, prefix_q=8))
    exp = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=25, local=local)
    pl = Pipeline(dev, k=25, local=local, slot_bytes=64 << 10, slot_records=256, n_slots=3)
    seq, qual = reads.seq.tobytes(), reads.qual.tobytes()
    cuts = [0, 1, 700, 701, 3000, 5999, 6000]  # includes 1-record slots and one larger than the slot (grows)
    for a, b in zip(cuts, cuts[1:]):
        pl.put(seq, qual, reads.offsets[a:b + 1])
    same(pl.finish(), exp, local)
    # finish resets the counters
    pl.put(seq, qual, reads.offsets[:11])
    part = dev.scan(seq, qual, reads.offsets[:11], k=25, local=local)
    same(pl.finish(), part, local)
    pl.close()


def test_em_histogram_through_stream(tmp_path):
    ref = synth.make_reference(4, 2, 6_000)
    reads = synth.make_reads(ref, 3_000)
    seqs, quals = split(reads)
    write_fastq(tmp_path / "r.fq.gz", seqs, quals, gz=True)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 4, prefix_q=8))
    em1, em2 = EmHistogram(dev), EmHistogram(dev)
    r1 = em1.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21)
    r2, _ = dev.scan_fastq(str(tmp_path / "r.fq.gz"), k=21, em=em2, threads=4)
    same(r1, r2, False)
    em1.finalize()
    em2.finalize()
    assert em1.info() == em2.info()
    p = np.array([10.0, 20.0, 30.0, 40.0])
    np.testing.assert_array_equal(em1.step(p, [2, 2, 2, 2], r1.unique), em2.step(p, [2, 2, 2, 2], r2.unique))


def test_pipeline_rejects_bad_input():
    ref = synth.make_reference(2, 1, 2_000)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 2, prefix_q=4))
    with pytest.raises(SpeqError):
        Pipeline(dev, k=21, paired=True, slot_records=3)
    pl = Pipeline(dev, k=21, paired=True, slot_records=4)
    with pytest.raises(SpeqError, match="even"):
        pl.put(b"ACGT" * 3, b"IIII" * 3, np.array([0, 4, 8, 12], dtype=np.uint64))
    pl.close()


@pytest.mark.parametrize("fmt", [dict(), dict(crlf=True), dict(gz=True)])
@pytest.mark.parametrize("paired", [False, True])
def test_gpu_fastq_parse_equals_host_parse(tmp_path, fmt, paired):
    """Simple four-line blocks are split into records on the GPU (fastq_gpu.hip); the host parser (knob off) must
    give the same counters, EM histogram and stream statistics."""
    ref = synth.make_reference(4, 2, 20_000)
    reads = synth.make_reads(ref, 60_000 // (2 if paired else 1), paired=paired, n_rate=0.001, lowq_rate=0.01,
                             short_frac=0.0 if paired else 0.05)
    seqs, quals = split(reads)
    if paired:
        write_fastq(tmp_path / "r1.fq", seqs[0::2], quals[0::2], **fmt)
        write_fastq(tmp_path / "r2.fq", seqs[1::2], quals[1::2], **fmt)
        p1, p2 = str(tmp_path / "r1.fq"), str(tmp_path / "r2.fq")
    else:
        write_fastq(tmp_path / "r1.fq", seqs, quals, **fmt)
        p1, p2 = str(tmp_path / "r1.fq"), None
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 4, prefix_q=10, pair_steps=True, triple_steps=True))
    assert dev.tuning("fastq_gpu_parse") == 1
    res = {}
    for gpu in (1, 0):
        dev.tune(fastq_gpu_parse=gpu)
        for local in (False, True):
            em = EmHistogram(dev)
            r, st = dev.scan_fastq(p1, p2, k=21, local=local, threads=3, em=em)
            em.finalize()
            res[(gpu, local)] = (r, st, em.info(), em.step(np.full(4, 25.0), [2, 2, 2, 2], r.unique))
    exp = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21, paired=paired)
    for local in (False, True):
        (a, sa, ia, na), (b, sb, ib, nb) = res[(1, local)], res[(0, local)]
        same(a, b, local)
        assert (sa["records"], sa["bases"]) == (sb["records"], sb["bases"]) == (reads.n, int(reads.offsets[-1]))
        assert ia == ib
        np.testing.assert_allclose(na, nb, rtol=1e-12)
    same(res[(1, False)][0], exp, False)


def test_gpu_fastq_parse_blanks_and_errors(tmp_path):
    """Four-line records whose lines hold blanks (dropped) take the GPU path's compaction; a base/quality count
    mismatch that only the character filter reveals is an error on both paths."""
    ref = synth.make_reference(2, 1, 4_000)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 2, prefix_q=6, pair_steps=True, triple_steps=True))
    rd = synth.make_reads(ref, 500, read_len=60)
    seqs, quals = split(rd)
    lines = []
    for i, (s, q) in enumerate(zip(seqs, quals)):
        s, q = s.decode(), q.decode()
        if i % 3 == 0:  # one blank in each line: raw lengths stay equal, the filtered counts too
            s, q = s[:10] + " " + s[10:], q[:20] + " " + q[20:]
        lines.append(f"@r{i}\n{s}\n+\n{q}\n")
    (tmp_path / "b.fq").write_text("".join(lines))
    got = {}
    for gpu in (1, 0):
        dev.tune(fastq_gpu_parse=gpu)
        got[gpu] = dev.scan_fastq(str(tmp_path / "b.fq"), k=19, threads=2)
    same(got[1][0], got[0][0], False)
    assert got[1][1]["records"] == 500
    exp = dev.scan(rd.seq.tobytes(), rd.qual.tobytes(), rd.offsets, k=19)
    same(got[1][0], exp, False)
    (tmp_path / "bad.fq").write_text("@a\nACGTACGTAC\n+\nIIIIIIIIII\n@b\nACGT7\n+\nIIIII\n")
    for gpu in (1, 0):
        dev.tune(fastq_gpu_parse=gpu)
        with pytest.raises(SpeqError, match="mismatch"):
            dev.scan_fastq(str(tmp_path / "bad.fq"), k=3)
    dev.tune(fastq_gpu_parse=1)


PARALLEL_CASES = ["simple", "wrapped_late", "blank_late", "blank_tail", "crlf", "no_final_newline", "error_late",
                  "plus_base_line"]


@pytest.mark.parametrize("case", PARALLEL_CASES)
def test_parallel_cut_stream_and_restart(tmp_path, monkeypatch, case):
    """A single-end plain file is cut at guessed record starts in parallel (several blocks here) and parsed on the
    GPU without host checks; a layout the GPU's four-line checks reject late in the file makes the stream restart
    with the sequential cutter after blocks were already scanned, so the counters AND the EM histogram must have
    been cleared first. Counters, EM histogram and statistics equal the sequential run (SPEQ_SPLIT_CUT=0) and the
    in-memory scan; a malformed file raises the sequential reader's error."""
    ref = synth.make_reference(4, 2, 20_000)
    reads = synth.make_reads(ref, 120_000, read_len=100, n_rate=0.001, lowq_rate=0.01)
    seqs, quals = split(reads)
    p = tmp_path / "r.fq"
    write_fastq(p, seqs, quals, crlf=case == "crlf")
    data = p.read_bytes()
    cut = data.index(b"\n@read", len(data) * 5 // 6) + 1
    extra = {"wrapped_late": b"@w\nACGTACGTAC\nGTACGTACGT\n+\nIIIIIIIIII\nIIIIIIIIII\n", "blank_late": b"\n",
             "error_late": b"@e\nACGT\n+\nII\n", "plus_base_line": b"@p\n+ACGT\n+\nIIIII\n"}.get(case)
    if extra:
        data = data[:cut] + extra + data[cut:]
    if case == "blank_tail":
        data += b"\n\n"
    if case == "no_final_newline":
        data = data[:-1]
    p.write_bytes(data)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 4, prefix_q=10, pair_steps=True, triple_steps=True))
    if case in ("error_late", "plus_base_line"):
        for split_cut in ("1", "0"):
            monkeypatch.setenv("SPEQ_SPLIT_CUT", split_cut)
            with pytest.raises(SpeqError, match="mismatch" if case == "error_late" else "malformed"):
                dev.scan_fastq(str(p), k=21, threads=6)
        return
    emx = EmHistogram(dev)
    exp = emx.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21)
    emx.finalize()
    got = {}
    for split_cut in ("1", "0"):
        monkeypatch.setenv("SPEQ_SPLIT_CUT", split_cut)
        em = EmHistogram(dev)
        r, st = dev.scan_fastq(str(p), k=21, em=em, threads=6)
        em.finalize()
        got[split_cut] = (r, st, em.info())
    same(got["1"][0], got["0"][0], False)
    n_extra = 1 if case == "wrapped_late" else 0
    assert got["1"][1]["records"] == got["0"][1]["records"] == reads.n + n_extra
    assert got["1"][1]["bases"] == got["0"][1]["bases"] == int(reads.offsets[-1]) + 20 * n_extra
    assert got["1"][2] == got["0"][2]
    same(got["1"][0], exp, False)  # the extra record is shorter than k
    assert got["1"][2] == emx.info()


PAIRED_CASES = ["simple", "crlf", "no_final_newline", "unequal", "wrapped_late_2", "blank_late_1", "error_late_2"]


@pytest.mark.parametrize("case", PAIRED_CASES)
def test_paired_parallel_cut(tmp_path, monkeypatch, case):
    """Paired plain files are cut in parallel, newlines counted per block, and each file-1 block is paired with the
    same records of file 2; layouts the GPU checks reject, or files of different record counts, restart with the
    sequential reader. Counters, EM histogram and statistics equal the sequential run and the in-memory scan."""
    ref = synth.make_reference(4, 2, 20_000)
    reads = synth.make_reads(ref, 160_000, paired=True, n_rate=0.001, lowq_rate=0.01)
    seqs, quals = split(reads)
    p1, p2 = tmp_path / "r1.fq", tmp_path / "r2.fq"
    write_fastq(p1, seqs[0::2], quals[0::2], crlf=case == "crlf")
    write_fastq(p2, seqs[1::2], quals[1::2], crlf=case == "crlf")
    n_pairs = reads.n // 2

    def insert(path, extra):
        data = path.read_bytes()
        cut = data.index(b"\n@read", len(data) * 5 // 6) + 1
        path.write_bytes(data[:cut] + extra + data[cut:])

    if case == "no_final_newline":
        p2.write_bytes(p2.read_bytes()[:-1])
    elif case == "unequal":
        data = p2.read_bytes()
        cut = data.index(b"\n@read", len(data) * 3 // 4) + 1
        p2.write_bytes(data[:cut])
        n_pairs = data[:cut].count(b"\n@read") + 1
    elif case == "wrapped_late_2":
        insert(p2, b"@w\nACGTACGTAC\nGTACGTACGT\n+\nIIIIIIIIII\nIIIIIIIIII\n")
    elif case == "blank_late_1":
        insert(p1, b"\n")
    elif case == "error_late_2":
        insert(p2, b"@e\nACGT\n+\nII\n")
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 4, prefix_q=10, pair_steps=True, triple_steps=True))
    if case == "error_late_2":
        for split_cut in ("1", "0"):
            monkeypatch.setenv("SPEQ_SPLIT_CUT", split_cut)
            with pytest.raises(SpeqError, match="mismatch"):
                dev.scan_fastq(str(p1), str(p2), k=21, threads=6)
        return
    got = {}
    for split_cut in ("1", "0"):
        monkeypatch.setenv("SPEQ_SPLIT_CUT", split_cut)
        em = EmHistogram(dev)
        r, st = dev.scan_fastq(str(p1), str(p2), k=21, em=em, threads=6)
        em.finalize()
        got[split_cut] = (r, st, em.info())
    same(got["1"][0], got["0"][0], False)
    assert got["1"][1]["records"] == got["0"][1]["records"]
    assert got["1"][1]["bases"] == got["0"][1]["bases"]
    assert got["1"][2] == got["0"][2]
    if case != "wrapped_late_2":  # the inserted record shifts the pairing after it
        assert got["1"][1]["records"] == 2 * n_pairs
        m = 2 * n_pairs
        exp = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets[:m + 1], k=21, paired=True)
        same(got["1"][0], exp, False)


@pytest.mark.parametrize("seed", range(6))
def test_parallel_cut_fuzz(tmp_path, monkeypatch, seed):
    """Random irregularities (blank lines, wrapped records, CRLF lines, quality lines opening with '@' or '+',
    descriptions on the '+' line) dropped into a multi-block file at random places: the parallel cut (with its
    fallback) and the sequential reader agree on counters, EM histogram and statistics, or raise the same error."""
    rng = np.random.default_rng(1000 + seed)
    ref = synth.make_reference(3, 2, 15_000)
    reads = synth.make_reads(ref, 100_000, read_len=int(rng.integers(60, 200)), n_rate=0.002, lowq_rate=0.02,
                             short_frac=0.05)
    seqs, quals = split(reads)
    recs = []
    for i, (s, q) in enumerate(zip(seqs, quals)):
        q = bytearray(q)
        if q and rng.random() < 0.05:
            q[0] = ord("@") if rng.random() < 0.5 else ord("+")
        recs.append([b"@r%d" % i, s, b"+" if rng.random() < 0.7 else b"+r%d" % i, bytes(q)])
    n_irr = int(rng.integers(0, 4))
    for _ in range(n_irr):
        j = int(rng.integers(len(recs) // 2, len(recs)))
        kind = int(rng.integers(0, 3))
        if kind == 0:
            recs[j][0] = b"\n" + recs[j][0]  # blank line before the header
        elif kind == 1 and len(recs[j][1]) > 10:
            s, q = recs[j][1], recs[j][3]
            recs[j][1] = s[:7] + b"\n" + s[7:]
            recs[j][3] = q[:5] + b"\n" + q[5:]  # wrapped record
        else:
            recs[j][1] += b"\r"
            recs[j][3] += b"\r"
    data = b"".join(b"\n".join(r) + b"\n" for r in recs)
    p = tmp_path / "f.fq"
    p.write_bytes(data)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 3, prefix_q=8, pair_steps=True, triple_steps=True))
    out = {}
    for split_cut in ("1", "0"):
        monkeypatch.setenv("SPEQ_SPLIT_CUT", split_cut)
        em = EmHistogram(dev)
        try:
            r, st = dev.scan_fastq(str(p), k=19, em=em, threads=5)
            em.finalize()
            out[split_cut] = ((r.total, r.ambiguous, r.unique.tolist()), st["records"], st["bases"], em.info())
        except SpeqError as e:
            out[split_cut] = ("error", str(e))
    assert out["1"] == out["0"]
