"""GPU: batches in flight on two HIP streams. speq_scan_reads_device keeps no
per-launch state, so two batches scanned on two streams at once, each into its own counters, must give exactly what
each batch gives alone on one stream; bench.py's default timing depends on it. Batches of different reads, both
modes, launched back to back many times so that the launches overlap."""
import numpy as np
import pytest
import torch

from speq_amd import DeviceIndex, FmIndex, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    ref = synth.make_reference(6, 2, 20_000, ref_n_rate=0.001)
    idx = FmIndex.build(ref.records, ref.groups, 6, prefix_q=10, pair_steps=True, triple_steps=True)
    return ref, idx


@pytest.mark.parametrize("local", [False, True])
@pytest.mark.parametrize("k", [21, 70])
def test_two_streams_equal_one(setup, local, k):
    ref, idx = setup
    G = 6
    dev = DeviceIndex(idx)
    dev.prepare(k)
    batches = []
    for b in range(2):
        r = synth.make_reads(ref, 60_000, start_index=b * 60_000, err_rate=0.003, lowq_rate=0.01)
        r = synth.apply_quality_profile(r, "variable") if b == 1 else r
        batches.append(dict(seq=torch.from_numpy(r.seq).cuda(), qual=torch.from_numpy(r.qual).cuda(),
                            off=torch.from_numpy(r.offsets.astype(np.int64)).cuda(), n=r.n))

    def scan(b, cnt, w, stream):
        with torch.cuda.stream(stream):
            cnt.zero_()
            w.zero_()
            dev.scan_device(b["seq"].data_ptr(), b["qual"].data_ptr(), b["off"].data_ptr(), b["n"], k,
                            cnt.data_ptr(), w.data_ptr(), local=local, stream=stream.cuda_stream)

    one = torch.cuda.Stream()
    alone = []
    for b in batches:
        cnt = torch.zeros(G + 2, dtype=torch.int64, device="cuda")
        w = torch.zeros(G, dtype=torch.float64, device="cuda")
        scan(b, cnt, w, one)
        torch.cuda.synchronize()
        alone.append((cnt.cpu().numpy(), w.cpu().numpy()))
    assert alone[0][0][0] > 0 and alone[1][0][0] > 0

    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    cnts = [torch.zeros(G + 2, dtype=torch.int64, device="cuda") for _ in range(2)]
    ws = [torch.zeros(G, dtype=torch.float64, device="cuda") for _ in range(2)]
    for i in range(40):
        scan(batches[i & 1], cnts[i & 1], ws[i & 1], streams[i & 1])
    torch.cuda.synchronize()
    for i in range(2):
        np.testing.assert_array_equal(cnts[i].cpu().numpy(), alone[i][0])
        np.testing.assert_allclose(ws[i].cpu().numpy(), alone[i][1], rtol=1e-12, atol=0)
    dev.close()
