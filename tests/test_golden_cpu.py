"""CPU: the oracle and the FM-index layout (walked with numpy) against the committed golden vectors."""
import numpy as np
import pytest

from fm_numpy import NumpyFm, ascii_to_syms
from golden_io import CASES, Case
from oracle.oracle import Oracle
from speq_amd import FmIndex, file_to_map


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_golden(name):
    c = Case(name)
    for k in c.ks:
        e = c.exp["by_k"][str(k)]
        orc = Oracle(c.records, c.groups, c.G, k)
        u, t = orc.ref_unique()
        assert u.tolist() == e["u_ref"] and t.tolist() == e["tot_ref"]
        for mode in ("global", "local"):
            T, amb, U, W = orc.scan(c.seq, c.qual, c.offsets, phred_cutoff=c.cutoff, paired=c.paired,
                                    local=mode == "local")
            g = e[mode]
            assert (T, amb, U.tolist()) == (g["T"], g["ambiguous"], g["U"]), (name, k, mode)
            if mode == "local":
                np.testing.assert_allclose(W, g["W"], rtol=1e-12)


@pytest.mark.parametrize("name", CASES)
def test_groupings_file_matches_golden(name):
    c = Case(name)
    g = file_to_map(f"{c.dir}/groups.txt")
    assert g.scaffolds[:len(c.records)] == c.groups
    assert len(g.names) == c.G


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("q", [0, 3, 6])
@pytest.mark.parametrize("steps", [1, 2, 3])
@pytest.mark.parametrize("lab", [False, True])
def test_fm_layout_classifies_like_oracle(name, q, steps, lab):
    """Backward search over the host arrays of OUR index reproduces the oracle label of every read window
    and every reference window (N included), with single-base, two-base and three-base LF steps."""
    c = Case(name)
    idx = FmIndex.build(c.records, c.groups, c.G, prefix_q=q, pair_steps=steps >= 2, label_table=lab,
                        triple_steps=steps == 3)
    fm = NumpyFm(idx)
    for k in c.ks:
        orc = Oracle(c.records, c.groups, c.G, k)
        wins = []
        for r in c.records:
            wins += [r[j:j + k] for j in range(len(r) - k + 1)]
        for i in range(len(c.offsets) - 1):
            s = c.seq[int(c.offsets[i]):int(c.offsets[i + 1])]
            wins += [s[j:j + k] for j in range(len(s) - k + 1)]
        syms = np.stack([ascii_to_syms(w) for w in wins])
        got = fm.classify(syms)
        exp = np.array([orc.lookup(w) for w in wins])
        assert np.array_equal(got, exp), (name, k, q)
