"""GPU: EM refinement from the one-scan interval histogram against the literal per-window EM of the reference
(golden trajectories from the pure-Python brute force; the C oracle on larger inputs). fp64 sums are reordered
(per-window weights cancel, multiplicities multiply), so next_tkpg is compared with rtol 1e-9."""
import numpy as np
import pytest

from golden_io import CASES, Case
from oracle.oracle import Oracle
from speq_amd import DeviceIndex, EmHistogram, FmIndex, em_refine, synth, unique_to_percent

pytestmark = pytest.mark.gpu
RTOL = 1e-9


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("mode", ["global", "local"])
def test_em_trajectory_matches_golden(name, mode):
    c = Case(name)
    k = c.ks[0]
    g = c.exp["by_k"][str(k)][mode]
    e = c.exp["by_k"][str(k)]
    dev = DeviceIndex(FmIndex.build(c.records, c.groups, c.G, prefix_q=4, pair_steps=True, label_table=True))
    em = EmHistogram(dev)
    r = em.scan(c.seq, c.qual, c.offsets, k=k, phred_cutoff=c.cutoff, paired=c.paired, local=mode == "local")
    assert (r.total, r.ambiguous, r.unique.tolist()) == (g["T"], g["ambiguous"], g["U"])
    em.finalize()
    counts = c.exp["group_counts"]
    # step by step from the golden percentages
    percent = g["percent"]
    for it in g["em"]:
        nxt = em.step(percent, counts, r.unique)
        np.testing.assert_allclose(nxt, it["next_tkpg"], rtol=RTOL)
        percent = it["percent"]
    # the whole loop from our own scan
    ut = r.weights if mode == "local" else r.unique / (c.exp["fixed_accuracy"] ** k)
    p0 = unique_to_percent(ut, r.total, e["u_ref"], e["tot_ref"])
    traj = em_refine(lambda p: em.step(p, counts, r.unique), ut, r.total, p0)
    assert len(traj) == len(g["em"])
    np.testing.assert_allclose(traj[-1][0], g["em"][-1]["percent"], rtol=1e-7)


@pytest.mark.parametrize("paired,label_table", [(False, True), (True, True), (False, False)])
def test_em_step_matches_oracle_larger(paired, label_table):
    # (label_table: the rows walk the label table, one load per label run; without it, the run bitvector's rank path)
    ref = synth.make_reference(5, 3, 6_000, ref_n_rate=0.001)
    reads = synth.make_reads(ref, 2_000, read_len=100, paired=paired, n_rate=0.002, lowq_rate=0.01)
    G, k, cutoff = 5, 21, 30
    counts = [3, 3, 2, 3, 1]
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, G, prefix_q=9, pair_steps=True, label_table=label_table))
    em = EmHistogram(dev)
    r = em.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, phred_cutoff=cutoff, paired=paired,
                local=True)
    em.finalize()
    orc = Oracle(ref.records, ref.groups, G, k)
    # the histogram holds exactly the passing windows that hit more than one group
    multi = 0
    for i in range(len(reads.offsets) - 1):
        a, b = int(reads.offsets[i]), int(reads.offsets[i + 1])
        s, q = reads.seq[a:b].tobytes(), reads.qual[a:b].astype(np.int32) - 33
        for j in range(len(s) - k + 1):
            if q[j:j + k].min() > cutoff and b"N" not in s[j:j + k] and orc.lookup(s[j:j + k]) == -2:
                multi += 1
    n_int, n_ent, n_win = em.info()
    assert n_win == multi and n_int <= n_win and n_ent >= 2 * n_int
    rng = np.random.default_rng(3)
    for percent in (np.full(G, 20.0), rng.uniform(0, 50, G), np.array([0.0, 10.0, 0.0, 5.0, 1.0])):
        got = em.step(percent, counts, r.unique)
        exp = orc.em_pass(reads.seq, reads.qual, reads.offsets, percent, counts, phred_cutoff=cutoff, paired=paired,
                          local=True)
        np.testing.assert_allclose(got, exp, rtol=RTOL, atol=1e-9)
