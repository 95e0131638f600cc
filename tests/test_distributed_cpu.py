"""CPU (gloo, world_size 2): the multi-GPU decomposition of bench.py / SURVEY.md §8(e).

Reads shard by contiguous ranges of the deterministic read stream (pairs never split), the index is replicated, and
the only exchange is one all-reduce (sum) of the G+2 counters. Here each rank's scanner is the oracle (CPU), so the
test checks the decomposition and the collective: sum over shards == unsharded counts, ambiguity included.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from speq_amd import synth

N_PER_RANK = 1500


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, paired, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle.oracle import Oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ref = synth.make_reference(4, 2, 3000)
    reads = synth.make_reads(ref, N_PER_RANK, start_index=rank * N_PER_RANK, paired=paired, n_rate=0.003)
    orc = Oracle(ref.records, ref.groups, 4, 21)
    T, amb, U, W = orc.scan(reads.seq, reads.qual, reads.offsets, paired=paired, local=True, threads=1)
    counts = torch.tensor([T, amb] + U.tolist(), dtype=torch.int64)
    w = torch.tensor(W, dtype=torch.float64)
    dist.all_reduce(counts)
    dist.all_reduce(w)
    if rank == 0:
        q.put((counts.numpy().copy(), w.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("paired", [False, True])
def test_sharded_allreduce_equals_unsharded(paired):
    from oracle.oracle import Oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, paired, q)) for r in range(world)]
    for p in procs:
        p.start()
    counts, w = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = synth.make_reference(4, 2, 3000)
    whole = synth.make_reads(ref, world * N_PER_RANK, paired=paired, n_rate=0.003)
    orc = Oracle(ref.records, ref.groups, 4, 21)
    T, amb, U, W = orc.scan(whole.seq, whole.qual, whole.offsets, paired=paired, local=True, threads=1)
    assert counts.tolist() == [T, amb] + U.tolist()
    np.testing.assert_allclose(w, W, rtol=1e-12)


def test_read_stream_is_shardable():
    """make_reads(start_index=r*n) shards concatenate to the unsharded stream (weak-scaling inputs of bench.py)."""
    ref = synth.make_reference(3, 1, 2000)
    a = synth.make_reads(ref, 100, start_index=0)
    b = synth.make_reads(ref, 100, start_index=100)
    ab = synth.make_reads(ref, 200)
    assert np.array_equal(np.concatenate([a.seq, b.seq]), ab.seq)
    assert np.array_equal(np.concatenate([a.qual, b.qual]), ab.qual)
