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


# ---- the product's own host-socket transport (speq_comm_connect, SPEQ_COMM_HOST): no GPU needed ----

def _host_rank(rank, world, path, out, errs):
    from speq_amd import Comm
    try:
        c = Comm.connect(world, rank, path, device=-1, transport=Comm.HOST, timeout_s=60)
        assert c.transport == Comm.HOST
        u = np.arange(5, dtype=np.uint64) * np.uint64(rank + 1)
        f = np.array([0.1 * (rank + 1), 1e300, -2.5], dtype=np.float64)
        c.allreduce_host(u)
        c.allreduce_host(f)
        out[rank] = (u.copy(), f.copy())
        c.close()
    except Exception as e:  # noqa: BLE001 - reported by the test thread
        errs.append((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_host_transport_allreduce(tmp_path, world):
    """speq_comm_connect over loopback sockets: every rank ends with the same sums, f64 added in rank order."""
    import threading
    path = str(tmp_path / "rdzv")
    out, errs = {}, []
    ts = [threading.Thread(target=_host_rank, args=(r, world, path, out, errs)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
    su = sum(np.arange(5, dtype=np.uint64) * np.uint64(r + 1) for r in range(world))
    fsum = np.array([0.1, 1e300, -2.5])
    for r in range(1, world):
        fsum = fsum + np.array([0.1 * (r + 1), 1e300, -2.5])
    for r in range(world):
        assert np.array_equal(out[r][0], su)
        assert np.array_equal(out[r][1], fsum)  # bit-identical: rank 0 adds in rank order
    assert not os.path.exists(path), "rank 0 removes the rendezvous file once every rank has joined"


def test_host_transport_skips_a_stale_rendezvous(tmp_path):
    """A rendezvous file left by a dead run (its port refuses) is skipped until rank 0 publishes a live one."""
    import struct
    import threading
    import time
    path = str(tmp_path / "rdzv")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    dead_port = s.getsockname()[1]
    s.close()
    with open(path, "wb") as f:  # {magic "SPEQRDZ1", nonce, port}
        f.write(struct.pack("<QQQ", 0x5350455152445A31, 12345, dead_port))
    out, errs = {}, []
    t1 = threading.Thread(target=_host_rank, args=(1, 2, path, out, errs))
    t1.start()
    time.sleep(0.5)  # rank 1 meets the stale file first
    t0 = threading.Thread(target=_host_rank, args=(0, 2, path, out, errs))
    t0.start()
    t0.join(120)
    t1.join(120)
    assert not errs, errs
    assert np.array_equal(out[0][0], out[1][0])
