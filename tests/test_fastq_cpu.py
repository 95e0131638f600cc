"""CPU: the streaming FASTQ reader/parsers (speq_scan_fastq's front end, via speq_fastq_checksum — no GPU) against
a plain-Python restatement of the grammar, over layouts the fast 4-line path does and does not take (wrapped
records, CRLF, blank lines, blanks/digits inside sequence lines, gzip), thread counts, block boundaries and
the paired zip-to-the-shorter-file rule (/root/reference/src/fm_scanner.cpp:651-655)."""
import ctypes as C
import gzip

import numpy as np
import pytest

from speq_amd import SpeqError, synth
from speq_amd._lib import check, lib

M64 = (1 << 64) - 1


def mix(z):
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
    return z ^ (z >> 31)


def digest(records):
    acc = 0
    for s, q in records:
        h = 0x9e3779b97f4a7c15 ^ len(s)
        for a, b in zip(s, q):
            h = ((h ^ (a << 8 | b)) * 0x100000001b3) & M64
        acc = (acc + mix(h)) & M64
    return acc


def parse_py(data: bytes):
    """The grammar of host_io.cpp / fastq_stream.cpp, line by line."""
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    lines = [ln.rstrip(b"\r") for ln in lines]
    i, out = 0, []
    ws = b" \t\n\v\f\r"
    while True:
        while i < len(lines) and lines[i] == b"":
            i += 1
        if i >= len(lines):
            return out
        assert lines[i][:1] == b"@"
        i += 1
        seq = b""
        while not lines[i][:1] == b"+":
            seq += bytes(c for c in lines[i] if c not in ws and not 48 <= c <= 57)
            i += 1
        i += 1
        qual = b""
        while len(qual) < len(seq) and i < len(lines):
            qual += bytes(c for c in lines[i] if c not in ws)
            i += 1
        assert len(qual) == len(seq)
        out.append((seq, qual))


def checksum(p1, p2=None, threads=3):
    r, b, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
    check(lib().speq_fastq_checksum(str(p1).encode(), str(p2).encode() if p2 else None, threads, C.byref(r),
                                    C.byref(b), C.byref(d)))
    return r.value, b.value, d.value


def records_of(reads):
    out = []
    for i in range(len(reads.offsets) - 1):
        a, b = int(reads.offsets[i]), int(reads.offsets[i + 1])
        out.append((reads.seq[a:b].tobytes(), reads.qual[a:b].tobytes()))
    return out


def render(records, wrap=0, crlf=False, blank=False, junk=False):
    nl = b"\r\n" if crlf else b"\n"
    parts = []
    for i, (s, q) in enumerate(records):
        if junk and i % 5 == 1 and len(s) > 10:
            s = s[:4] + b" 7" + s[4:]  # blank and digit inside the sequence line are dropped
        parts.append(b"@r%d desc%s" % (i, nl))
        if wrap:
            parts += [s[j:j + wrap] + nl for j in range(0, len(s), wrap)] or [nl]
            parts.append(b"+r" + nl)
            parts += [q[j:j + wrap] + nl for j in range(0, len(q), wrap)]
        else:
            parts += [s + nl, b"+" + nl, q + nl]
        if blank and i % 4 == 2:
            parts.append(nl)
    return b"".join(parts)


LAYOUTS = [dict(), dict(wrap=40), dict(crlf=True), dict(blank=True), dict(junk=True), dict(wrap=33, crlf=True)]


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("gz", [False, True])
def test_reader_matches_python_grammar(tmp_path, layout, gz):
    ref = synth.make_reference(2, 1, 3_000)
    recs = records_of(synth.make_reads(ref, 700, read_len=90, short_frac=0.1, n_rate=0.01, lowq_rate=0.05))
    data = render(recs, **layout)
    exp = parse_py(data)
    p = tmp_path / ("r.fq.gz" if gz else "r.fq")
    (gzip.open(p, "wb") if gz else open(p, "wb")).write(data)
    n, b, d = checksum(p)
    assert (n, b, d) == (len(exp), sum(len(s) for s, _ in exp), digest(exp))


def test_many_blocks_and_threads(tmp_path):
    ref = synth.make_reference(3, 1, 10_000)
    reads = synth.make_reads(ref, 300_000, read_len=60)  # > two 131072-record blocks
    recs = records_of(reads)
    data = render(recs)
    (tmp_path / "a.fq").write_bytes(data)
    with gzip.open(tmp_path / "a.fq.gz", "wb", compresslevel=1) as f:
        f.write(data)
    (tmp_path / "w.fq").write_bytes(render(recs, wrap=50, blank=True))
    base = checksum(tmp_path / "a.fq", threads=1)
    assert base[:2] == (reads.n, int(reads.offsets[-1]))
    for p, t in ((tmp_path / "a.fq", 7), (tmp_path / "a.fq.gz", 4), (tmp_path / "w.fq", 5)):
        assert checksum(p, threads=t) == base


def test_paired_zip_to_shorter(tmp_path):
    ref = synth.make_reference(2, 1, 3_000)
    reads = synth.make_reads(ref, 300, read_len=70, paired=True)
    recs = records_of(reads)
    m1, m2 = recs[0::2], recs[1::2]
    (tmp_path / "1.fq").write_bytes(render(m1))
    (tmp_path / "2.fq").write_bytes(render(m2[:120], wrap=30))
    n, b, d = checksum(tmp_path / "1.fq", tmp_path / "2.fq")
    zipped = [x for pair in zip(m1[:120], m2[:120]) for x in pair]
    assert (n, b, d) == (240, sum(len(s) for s, _ in zipped), digest(zipped))
    n2, _, _ = checksum(tmp_path / "2.fq", tmp_path / "1.fq")
    assert n2 == 240


@pytest.mark.parametrize("text,msg", [
    (b">r\nACGT\n", "qualities are required"),
    (b"@r\nACGTACGT\n", "truncated"),
    (b"@r\nACGTACGT\n+\nIIII\n", "mismatch"),
    (b"@r\nACGT\n+\nIIIIII\n", "mismatch"),
    (b"@r\nACGT\n+\nIIII\nxyz\n", "malformed"),
])
def test_reader_errors(tmp_path, text, msg):
    (tmp_path / "bad.fq").write_bytes(text)
    with pytest.raises(SpeqError, match=msg):
        checksum(tmp_path / "bad.fq")


def test_missing_and_empty(tmp_path):
    with pytest.raises(SpeqError, match="cannot open"):
        checksum(tmp_path / "nope.fq")
    (tmp_path / "e.fq").write_bytes(b"")
    assert checksum(tmp_path / "e.fq") == (0, 0, 0)
    (tmp_path / "b.fq").write_bytes(b"\n\n\r\n")
    assert checksum(tmp_path / "b.fq") == (0, 0, 0)
    # final record without a trailing newline
    (tmp_path / "t.fq").write_bytes(b"@a\nACGT\n+\nIIII\n@b\nGG\n+\nII")
    assert checksum(tmp_path / "t.fq")[:2] == (2, 6)


def write_bgzf(path, data: bytes, block=65280):
    """BGZF as bgzip writes it: independent raw-deflate gzip members with a BC extra field, then the EOF member."""
    import struct
    import zlib
    out = []
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        comp = co.compress(chunk) + co.flush()
        bsize = 18 + len(comp) + 8 - 1
        hdr = struct.pack("<BBBBIBBHBBHH", 0x1f, 0x8b, 8, 4, 0, 0, 0xff, 6, ord("B"), ord("C"), 2, bsize)
        out.append(hdr + comp + struct.pack("<II", zlib.crc32(chunk) & 0xffffffff, len(chunk)))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    with open(path, "wb") as f:
        f.write(b"".join(out))


@pytest.mark.parametrize("threads", [1, 4])
def test_bgzf_parallel_inflate(tmp_path, threads):
    """BGZF members are inflated in parallel into their final positions; same records as the plain file (> 16 MiB,
    so the reader's buffer fills mid-stream and members continue in the next read)."""
    ref = synth.make_reference(2, 1, 3_000)
    recs = records_of(synth.make_reads(ref, 110_000, read_len=90))
    data = render(recs)
    (tmp_path / "p.fq").write_bytes(data)
    write_bgzf(tmp_path / "b.fq.gz", data)
    assert checksum(tmp_path / "b.fq.gz", threads=threads) == checksum(tmp_path / "p.fq", threads=threads)
    # plain gzip readers accept BGZF too (concatenated members): same records
    assert gzip.decompress((tmp_path / "b.fq.gz").read_bytes()) == data


def test_bgzf_corruption_is_reported(tmp_path):
    data = render([(b"ACGT" * 10, b"I" * 40)] * 100)
    write_bgzf(tmp_path / "b.fq.gz", data, block=1000)
    raw = bytearray((tmp_path / "b.fq.gz").read_bytes())
    raw[40] ^= 0xFF  # inside the first member's deflate data
    (tmp_path / "c.fq.gz").write_bytes(bytes(raw))
    with pytest.raises(SpeqError):
        checksum(tmp_path / "c.fq.gz")


def _simple_records(n, seed, at_frac=0.3):
    """Short four-line records whose quality lines often start with '@' (a header look-alike for the cutter)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(8, 40, n)
    bases = np.frombuffer(b"ACGTN", np.uint8)
    out = []
    for i, L in enumerate(lens):
        s = bases[rng.integers(0, 5, L)].tobytes()
        q = bytearray(rng.integers(35, 74, L).astype(np.uint8).tobytes())
        if rng.random() < at_frac:
            q[0] = ord("@")
        out.append((s, bytes(q)))
    return out


@pytest.mark.parametrize("case", ["simple", "no_final_newline", "wrapped_late", "blank_tail", "crlf", "error_late"])
def test_parallel_cut_matches_sequential(tmp_path, monkeypatch, case):
    """Single-end mapped files are cut at guessed headers (find_cut) and every block is checked as a chain of
    four-line records; anything else restarts with the sequential cutter. Either way the records are the ones the
    sequential cutter and the Python grammar find."""
    recs = _simple_records(160_000, 7)  # ~9 MB: several 1 MiB+ blocks
    data = render(recs, crlf=case == "crlf")
    if case == "no_final_newline":
        data = data[:-1]
    elif case == "wrapped_late":
        cut = len(data) * 3 // 4
        cut = data.index(b"\n@r", cut) + 1
        data = data[:cut] + b"@w\nACGT\nAC\n+\nIIII\nII\n" + data[cut:]
    elif case == "blank_tail":
        data += b"\n\n"
    elif case == "error_late":
        cut = data.index(b"\n@r", len(data) * 2 // 3) + 1
        data = data[:cut] + b"@e\nACGT\n+\nII\n" + data[cut:]
    p = tmp_path / "s.fq"
    p.write_bytes(data)
    if case == "error_late":
        with pytest.raises(SpeqError, match="mismatch"):
            checksum(p, threads=4)
        return
    exp = parse_py(data)
    want = (len(exp), sum(len(s) for s, _ in exp), digest(exp))
    for t in (1, 4, 8):
        assert checksum(p, threads=t) == want
    monkeypatch.setenv("SPEQ_SPLIT_CUT", "0")
    assert checksum(p, threads=4) == want


def checksum_shard(p1, p2, shard, n_shards, cut, threads=3):
    r, b, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
    check(lib().speq_fastq_checksum_shard(str(p1).encode(), str(p2).encode() if p2 else None, threads, shard,
                                          n_shards, cut, C.byref(r), C.byref(b), C.byref(d)))
    return r.value, b.value, d.value


@pytest.mark.parametrize("case", ["simple", "wrapped_late", "gz", "paired"])
def test_rank_shards_partition_the_records(tmp_path, case):
    """`speq scan` with one process per GPU (speq_scan_fastq_shard): rank r of W takes the blocks b with b % W == r of
    the same cut on every rank, so the W shards' records, bases and digests sum to the whole input. With the parallel
    cut (cut = 1) a file it cannot take fails with SPEQ_E_RETRY on the rank that meets the irregular block (the CLI
    then all-reduces that flag and every rank rescans with the sequential cutter, cut = 0)."""
    recs = _simple_records(160_000, 11)
    p2 = None
    if case == "paired":
        data1, data2 = render(recs[0::2]), render(recs[1::2])
        p, p2 = tmp_path / "1.fq", tmp_path / "2.fq"
        p.write_bytes(data1)
        p2.write_bytes(data2)
        exp = [r for pair in zip(parse_py(data1), parse_py(data2)) for r in pair]
    else:
        data = render(recs)
        if case == "wrapped_late":
            cut = data.index(b"\n@r", len(data) * 3 // 4) + 1
            data = data[:cut] + b"@w\nACGT\nAC\n+\nIIII\nII\n" + data[cut:]
        p = tmp_path / ("s.fq.gz" if case == "gz" else "s.fq")
        (gzip.open(p, "wb", compresslevel=1) if case == "gz" else open(p, "wb")).write(data)
        exp = parse_py(data)
    want = (len(exp), sum(len(s) for s, _ in exp), digest(exp))
    for W in (1, 2, 3, 4):
        for cut in (0, 1):
            parts, retry = [], 0
            for r in range(W):
                try:
                    parts.append(checksum_shard(p, p2, r, W, cut))
                except SpeqError as e:
                    assert e.code == -6 and cut == 1 and case == "wrapped_late"
                    retry += 1
            if case == "wrapped_late" and cut == 1:
                assert retry == 1  # exactly the rank holding the wrapped record's block
                continue
            tot = (sum(x[0] for x in parts), sum(x[1] for x in parts), sum(x[2] for x in parts) & M64)
            assert tot == want, (W, cut)
            if W > 1 and case != "paired":
                assert all(x[0] > 0 for x in parts)  # several blocks: every rank has work
    with pytest.raises(SpeqError):
        checksum_shard(p, p2, 2, 2, 0)
