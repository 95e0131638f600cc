"""GPU: the HIP path reproduces the committed golden vectors (tests/golden/*/expected.json) bit-exactly
(fp64 Phred weights to rtol 1e-12), for every k of every case and several q-mer table sizes, with each read-scan
kernel (anchor-and-extend, k-mer interval table, LF steps); plus the RCCL
counter all-reduce through the C ABI on a single-rank communicator."""
import ctypes as C

import numpy as np
import pytest

from golden_io import CASES, Case
from speq_amd import DeviceIndex, FmIndex, lib
from speq_amd._lib import check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("q", [0, 4, 8])
@pytest.mark.parametrize("steps", [1, 2, 3])
def test_gpu_matches_golden(name, q, steps):
    c = Case(name)
    dev = DeviceIndex(FmIndex.build(c.records, c.groups, c.G, prefix_q=q, pair_steps=steps >= 2,
                                    label_table=steps == 2, triple_steps=steps == 3))
    variants = [(1, 1, 1), (1, 1, 0), (1, 0, 0), (2, 0, 0)]  # (ilp, k-mer table, anchor-and-extend)
    for k, ilp, kt, ax in [(k,) + v for k in c.ks for v in variants]:
        dev.tune(ilp=ilp, ilp_local=ilp, kmer_table=kt, ax_scan=ax)
        e = c.exp["by_k"][str(k)]
        u, t = dev.count_unique_kmers_per_group(k)
        assert u.tolist() == e["u_ref"] and t.tolist() == e["tot_ref"], (name, k)
        for mode in ("global", "local"):
            r = dev.scan(c.seq, c.qual, c.offsets, k=k, phred_cutoff=c.cutoff, paired=c.paired,
                         local=mode == "local")
            g = e[mode]
            assert (r.total, r.ambiguous, r.unique.tolist()) == (g["T"], g["ambiguous"], g["U"]), (name, k, mode)
            if mode == "local":
                np.testing.assert_allclose(r.weights, g["W"], rtol=1e-12)


def test_rccl_allreduce_single_rank():
    torch = pytest.importorskip("torch")
    L = lib()
    uid = C.create_string_buffer(128)
    check(L.speq_comm_unique_id(uid))
    comm = C.c_void_p()
    check(L.speq_comm_init(1, 0, uid, C.byref(comm)))
    x = torch.arange(12, dtype=torch.int64, device="cuda:0")
    y = torch.full((5,), 0.25, dtype=torch.float64, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    check(L.speq_allreduce_u64(comm, x.data_ptr(), 12, s))
    check(L.speq_allreduce_f64(comm, y.data_ptr(), 5, s))
    torch.cuda.synchronize()
    assert x.cpu().tolist() == list(range(12)) and y.cpu().tolist() == [0.25] * 5
    check(L.speq_comm_destroy(comm))


def test_comm_class_scan_allreduce_single_rank():
    """The one-process-per-GPU step of bench.py at nranks = 1: scan on HBM-resident reads, then the product's RCCL
    all-reduce (speq_amd.Comm -> speq_allreduce_u64/_f64) on the scan's stream leaves the counters unchanged."""
    torch = pytest.importorskip("torch")
    from speq_amd import Comm, DeviceIndex, FmIndex, synth
    ref = synth.make_reference(4, 1, 8_000)
    reads = synth.make_reads(ref, 3_000)
    dev = DeviceIndex(FmIndex.build(ref.records, ref.groups, 4, prefix_q=8, pair_steps=True))
    host = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21, local=True)
    comm = Comm(1, 0, Comm.unique_id())
    d_seq = torch.from_numpy(reads.seq).cuda()
    d_qual = torch.from_numpy(reads.qual).cuda()
    d_off = torch.from_numpy(reads.offsets.astype(np.int64)).cuda()
    c = torch.zeros(6, dtype=torch.int64, device="cuda")
    w = torch.zeros(4, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    dev.scan_device(d_seq.data_ptr(), d_qual.data_ptr(), d_off.data_ptr(), reads.n, 21, c.data_ptr(), w.data_ptr(),
                    local=True, stream=s)
    comm.allreduce_u64(c.data_ptr(), 6, s)
    comm.allreduce_f64(w.data_ptr(), 4, s)
    torch.cuda.synchronize()
    got = c.cpu().numpy().astype(np.uint64)
    assert got[0] == host.total and got[1] == host.ambiguous and np.array_equal(got[2:], host.unique)
    np.testing.assert_allclose(w.cpu().numpy(), host.weights, rtol=1e-12)
    comm.close()
    with pytest.raises(ValueError):
        Comm(1, 0, b"short")
