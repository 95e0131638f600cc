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
