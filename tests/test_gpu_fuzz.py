"""GPU: randomized parameter sweep against the C oracle (same seeded inputs): reference shapes (record counts and
lengths, N rate, groups), index options (q, one/two/three-symbol steps, label table, host or GPU build), scan
options (k, cutoff, paired, local) and launch knobs (windows per lane, occupancy cap, grid, q-mer table level,
k-mer interval table, anchor-and-extend scan and its table load).
Integer counters bit-exact, W to rtol 1e-10."""
import numpy as np
import pytest

from oracle.oracle import Oracle
from speq_amd import DeviceIndex, FmIndex, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(24))
def test_random_configurations(seed):
    rng = np.random.default_rng(4242 + seed)
    V, I = int(rng.integers(1, 6)), int(rng.integers(1, 4))
    length = int(rng.integers(200, 6000))
    ref = synth.make_reference(V, I, length, ref_n_rate=float(rng.choice([0.0, 0.001, 0.01])))
    G = V
    groups = list(ref.groups)
    if rng.random() < 0.3:  # regroup records at random (every group non-empty is not required)
        G = int(rng.integers(1, V * I + 1))
        groups = [int(g) for g in rng.integers(0, G, V * I)]
    steps = int(rng.integers(1, 4))
    q = int(rng.choice([0, 3, 6, 9]))
    idx = FmIndex.build(ref.records, groups, G, prefix_q=q, pair_steps=steps >= 2, triple_steps=steps == 3,
                        label_table=bool(rng.random() < 0.5), gpu_device=0 if rng.random() < 0.5 else None)
    dev = DeviceIndex(idx)
    dev.tune(ilp=int(rng.integers(1, 3)), ilp_local=int(rng.integers(1, 3)),
             blocks_per_cu=int(rng.choice([0, 2, 4])), grid_blocks=int(rng.choice([7, 64, 16384])),
             prefix_level=int(rng.choice([-1, 0, 1, 2])) if q >= 3 else -1,
             sparse_prefix=int(rng.choice([-1, 0, 1])), kmer_table=int(rng.integers(0, 2)),
             ax_scan=int(rng.random() < 0.7), ax_load=int(rng.choice([10, 35, 90])),
             grid_blocks_ax=int(rng.choice([1, 7, 65535])))
    paired = bool(rng.random() < 0.4)
    reads = synth.make_reads(ref, int(rng.integers(50, 1500)), read_len=int(rng.integers(20, 250)),
                             paired=paired, fragment=int(rng.integers(250, 600)), n_rate=0.003,
                             lowq_rate=float(rng.choice([0.0, 0.02])), short_frac=0.0 if paired else 0.1,
                             start_index=int(rng.integers(0, 10_000)))
    for _ in range(2):
        k = int(rng.choice([1, 5, 11, 16, 21, 31, 32, 33, 47, 70]))
        cutoff = int(rng.choice([0, 20, 30, 40]))
        local = bool(rng.random() < 0.5)
        orc = Oracle(ref.records, groups, G, k)
        got = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=k, phred_cutoff=cutoff,
                       paired=paired, local=local)
        T, amb, U, W = orc.scan(reads.seq, reads.qual, reads.offsets, phred_cutoff=cutoff, paired=paired,
                                local=local)
        assert (got.total, got.ambiguous, got.unique.tolist()) == (T, amb, U.tolist()), (seed, k, cutoff, local)
        if local:
            np.testing.assert_allclose(got.weights, W, rtol=1e-10)
        u, t = dev.count_unique_kmers_per_group(k)
        ou, ot = orc.ref_unique()
        assert np.array_equal(u, ou) and np.array_equal(t, ot), (seed, k)
