"""CPU: FM-index construction (SA-IS, occ blocks, label runs, q-mer table) and persistence."""
import numpy as np
import pytest

from fm_numpy import NumpyFm, ascii_to_syms
from oracle.oracle import Oracle
from speq_amd import FmIndex, SpeqError, synth
from speq_amd._lib import SPEQ_E_ARG, SPEQ_E_GROUPS, SPEQ_E_IO

SYMS = b"ACGTN"


def _random_records(rng, n, maxlen, alphabet=b"ACGT", n_rate=0.0):
    recs = []
    for _ in range(n):
        L = int(rng.integers(0, maxlen + 1))
        r = bytearray(rng.choice(list(alphabet), size=L).astype(np.uint8).tobytes())
        for i in range(L):
            if rng.random() < n_rate:
                r[i] = ord("N")
        recs.append(bytes(r))
    return recs


@pytest.mark.parametrize("seed", range(6))
def test_suffix_array_is_sorted(seed):
    rng = np.random.default_rng(seed)
    # tiny alphabets and repeats stress SA-IS recursion; empty records and N included
    alph = [b"A", b"AC", b"ACGT"][seed % 3]
    recs = _random_records(rng, int(rng.integers(1, 7)), 120, alph, n_rate=0.05 * (seed % 2))
    if all(len(r) == 0 for r in recs):
        recs[0] = b"ACGTTGCA"
    G = 2
    groups = [i % G for i in range(len(recs))]
    idx = FmIndex.build(recs, groups, G)
    text = idx.array("text", np.uint8).tobytes()
    sa = idx.array("sa", np.int32)
    assert sorted(range(len(text)), key=lambda i: text[i:]) == sa.tolist()
    n = len(text)
    assert idx.info().n == n and text[-1] == 0


@pytest.mark.parametrize("seed", range(4))
def test_occ_ranks_match_bwt(seed):
    rng = np.random.default_rng(100 + seed)
    recs = _random_records(rng, 5, 400, b"ACGT", n_rate=0.02)
    idx = FmIndex.build(recs, [0, 1, 0, 2, 1], 3, prefix_q=3)
    text = idx.array("text", np.uint8)
    sa = idx.array("sa", np.int32)
    bwt = np.where(sa == 0, 0, text[sa - 1])
    fm = NumpyFm(idx)
    n = len(text)
    pos = np.arange(n + 1)
    for s in range(5):  # A C G T N  -> SA alphabet 2..6
        code = s + 2
        expect = np.concatenate([[0], np.cumsum(bwt == code)])
        got = fm.rank(np.full(n + 1, s), pos)
        assert np.array_equal(got, expect), s
    # label runs: run_of(i) changes exactly where the group of the suffix changes
    ts = idx.array("text_start", np.uint64).astype(np.int64)
    tg = idx.array("text_group", np.int32)
    tid = np.clip(np.searchsorted(ts, sa, side="right") - 1, 0, len(tg) - 1)
    lab = tg[tid]
    runs = fm.run_of(np.arange(n))
    assert np.array_equal(fm.run_label[runs], lab)
    assert np.array_equal(np.diff(runs) != 0, np.diff(lab) != 0)


def test_prefix_table_equals_search():
    ref = synth.make_reference(3, 2, 2000)
    idx = FmIndex.build(ref.records, ref.groups, 3, prefix_q=5)
    fm = NumpyFm(idx)
    rng = np.random.default_rng(5)
    q = rng.integers(0, 4, size=(300, 5))
    a = fm.classify(q, use_prefix=True)
    b = fm.classify(q, use_prefix=False)
    assert np.array_equal(a, b)


def test_save_load_roundtrip(tmp_path):
    ref = synth.make_reference(3, 1, 3000, ref_n_rate=0.01)
    idx = FmIndex.build(ref.records, ref.groups, 3, prefix_q=6, pair_steps=True, triple_steps=True, label_table=True)
    p = str(tmp_path / "x.idx")
    idx.save(p, b"hello header")
    back = FmIndex.load(p)
    assert back.header == b"hello header"
    assert back.info().triple_steps == 1 and back.info().pair_steps == 1 and back.info().label_table == 1
    for name, dt in (("text", np.uint8), ("occ", np.uint32), ("occ2", np.uint32), ("occ3", np.uint32),
                     ("lab", np.uint32), ("runs", np.uint32),
                     ("run_label", np.uint16), ("prefix", np.uint32), ("C", np.uint32), ("text_start", np.uint64),
                     ("text_group", np.int32)):
        assert np.array_equal(idx.array(name, dt), back.array(name, dt)), name
    i1, i2 = idx.info(), back.info()
    assert (i1.n, i1.n_texts, i1.n_groups, i1.prefix_q, i1.n_runs) == (i2.n, i2.n_texts, i2.n_groups, i2.prefix_q,
                                                                       i2.n_runs)
    assert back.array("sa", np.int32).size == 0  # the suffix array is host-build only


def test_loaded_index_classifies_like_oracle(tmp_path):
    ref = synth.make_reference(4, 1, 2000)
    idx = FmIndex.build(ref.records, ref.groups, 4, prefix_q=4)
    p = str(tmp_path / "y.idx")
    idx.save(p)
    fm = NumpyFm(FmIndex.load(p))
    orc = Oracle(ref.records, ref.groups, 4, 15)
    reads = synth.make_reads(ref, 50, read_len=60)
    wins = [reads.seq[int(reads.offsets[i]) + j:int(reads.offsets[i]) + j + 15].tobytes()
            for i in range(reads.n) for j in range(60 - 15 + 1)]
    got = fm.classify(np.stack([ascii_to_syms(w) for w in wins]))
    assert got.tolist() == [orc.lookup(w) for w in wins]


def test_unassigned_records_are_rejected():
    recs = [b"ACGTACGT", b"GGGGCCCC", b"TTTTAAAA"]
    with pytest.raises(SpeqError) as e:
        FmIndex.build(recs, [0, -1, 1], 2)  # a gap in the groupings (-1)
    assert e.value.code == SPEQ_E_GROUPS
    with pytest.raises(SpeqError) as e:
        FmIndex.build(recs, [0, 1], 2)  # groupings shorter than the reference
    assert e.value.code == SPEQ_E_GROUPS
    with pytest.raises(SpeqError) as e:
        FmIndex.build(recs, [0, 1, 5], 2)  # group id out of range
    assert e.value.code == SPEQ_E_GROUPS
    # extra entries beyond the records are ignored (zip truncation, fm_scanner.cpp:1494)
    FmIndex.build(recs, [0, 1, 0, 1, 1], 2)


def test_bad_arguments():
    with pytest.raises(SpeqError) as e:
        FmIndex.build([b"ACGT"], [0], 0)
    assert e.value.code == SPEQ_E_ARG
    with pytest.raises(SpeqError) as e:
        FmIndex.build([b"ACGT"], [0], 1, prefix_q=14)
    assert e.value.code == SPEQ_E_ARG


def test_load_rejects_garbage(tmp_path):
    p = tmp_path / "bad.idx"
    p.write_bytes(b"not an index at all")
    with pytest.raises(SpeqError) as e:
        FmIndex.load(str(p))
    assert e.value.code == SPEQ_E_IO
    with pytest.raises(SpeqError):
        FmIndex.load(str(tmp_path / "missing.idx"))


def test_label_table_saturated_runs():
    """Label runs longer than 65535 positions saturate the table's distance; wide intervals (k = 1, 2) must then
    fall back to the rank path and still classify exactly (NumpyFm asserts table == rank path)."""
    ref = synth.make_reference(1, 2, 150_000)
    groups = [0, 0]
    idx = FmIndex.build(ref.records, groups, 2, prefix_q=0, label_table=True)  # group 1 is empty
    fm = NumpyFm(idx)
    assert fm.lab is not None and (fm.lab >> 16).max() == 0xFFFF
    for k in (1, 2, 9):
        kmers = np.array([[s % 4 for s in range(j, j + k)] for j in range(16)])
        got = fm.classify(kmers)
        assert set(got.tolist()) <= {0, -1}


def test_gpu_build_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(SpeqError, match="no GPU"):
        FmIndex.build([b"ACGT"], [0], 1, gpu_device=0)


@pytest.mark.parametrize("seed", range(3))
def test_three_symbol_planes_match_bwt(seed):
    """occ3 plane 16a+4b+c counts the SA rows whose suffix is preceded by abc, offset by C3[abc] = #suffixes < abc;
    a three-symbol LF step equals three single steps."""
    rng = np.random.default_rng(300 + seed)
    recs = _random_records(rng, 4, 500, b"ACGT", n_rate=0.02)
    idx = FmIndex.build(recs, [0, 1, 1, 2], 3, prefix_q=0, pair_steps=True, triple_steps=True)
    text = idx.array("text", np.uint8).astype(np.int64)
    sa = idx.array("sa", np.int32).astype(np.int64)
    fm = NumpyFm(idx)
    n = len(text)
    code = np.full(n, -1)
    ok = sa >= 3
    x, y, z = (np.where(ok, text[np.maximum(sa - d, 0)], 0) for d in (3, 2, 1))
    good = ok & (x >= 2) & (x <= 5) & (y >= 2) & (y <= 5) & (z >= 2) & (z <= 5)
    code[good] = (x[good] - 2) * 16 + (y[good] - 2) * 4 + (z[good] - 2)
    pos = np.arange(n + 1)
    for pl in range(64):
        a, b, c = pl // 16, (pl // 4) % 4, pl % 4
        rank = fm.lf3(np.full(n + 1, a), np.full(n + 1, b), np.full(n + 1, c), pos)
        expect = np.concatenate([[0], np.cumsum(code == pl)])
        base = rank - expect
        assert (base == base[0]).all(), pl  # constant offset C3[abc]
        # the offset is the number of suffixes < "abc"
        suffix_lt = sum(1 for p_ in range(n) if tuple(text[p_:p_ + 3]) < (a + 2, b + 2, c + 2))
        assert base[0] == suffix_lt, pl
    # LF3 == three single steps on random intervals of random patterns
    for _ in range(200):
        lo, hi = sorted(rng.integers(0, n + 1, 2))
        a, b, c = rng.integers(0, 4, 3)
        l1, h1 = fm.lf(np.array([c]), np.array([lo])), fm.lf(np.array([c]), np.array([hi]))
        l1, h1 = fm.lf(np.array([b]), l1), fm.lf(np.array([b]), h1)
        l1, h1 = fm.lf(np.array([a]), l1), fm.lf(np.array([a]), h1)
        l3, h3 = fm.lf3(np.array([a]), np.array([b]), np.array([c]), np.array([lo])), \
            fm.lf3(np.array([a]), np.array([b]), np.array([c]), np.array([hi]))
        if lo < hi and (h1 - l1)[0] > 0:
            assert (l1[0], h1[0]) == (l3[0], h3[0])
        else:
            assert (h3 - l3)[0] == (h1 - l1)[0] or lo >= hi


def test_triple_steps_need_pairs():
    with pytest.raises(SpeqError):
        FmIndex.build([b"ACGTACGT"], [0], 1, pair_steps=False, triple_steps=True)
