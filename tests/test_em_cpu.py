"""CPU: the oracle's literal EM pass reproduces the brute-force EM trajectory committed in the goldens."""
import numpy as np
import pytest

from golden_io import CASES, Case
from oracle.oracle import Oracle


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("mode", ["global", "local"])
def test_oracle_em_pass_matches_golden(name, mode):
    c = Case(name)
    k = c.ks[0]
    g = c.exp["by_k"][str(k)][mode]
    traj = g["em"]
    assert traj, "golden EM trajectory missing"
    orc = Oracle(c.records, c.groups, c.G, k)
    pp = c.exp["fixed_accuracy"] ** k
    percent = g["percent"]
    for it in traj:
        nxt = orc.em_pass(c.seq, c.qual, c.offsets, percent, c.exp["group_counts"], phred_cutoff=c.cutoff,
                          local=mode == "local", percent_perfect=pp)
        np.testing.assert_allclose(nxt, it["next_tkpg"], rtol=1e-12, atol=1e-12)
        percent = it["percent"]
