"""GPU: `python bench.py --gpus 2` on the one-GPU box — the bench's N > 1 path end to end.

Without a launcher bench.py starts torch.distributed.run over two local ranks itself (launch_plan "relaunch"). Both
ranks share the one GPU, so the transport is "host" (torch.distributed over gloo for the barrier and the
max-over-ranks timing; the product's speq_allreduce_u64 over its host-socket transport for the counters — the same
C ABI call the 8-GPU run makes over RCCL). Each rank scans its own shard of the deterministic read stream
(make_reads(start_index = rank * n)); the line's check must equal ONE process scanning both shards, and n_gpus must
say 2. Reference reduction replaced: /root/reference/src/fm_scanner.cpp:224-233."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from speq_amd import DeviceIndex, FmIndex, synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

READS = 100_000


@pytest.mark.parametrize("streams", [1, 2])
def test_bench_two_ranks_on_one_gpu(tmp_path, streams):
    """streams = 2: each rank pipelines two batches on two HIP streams, the counters all-reduced on a third (the
    communication stream) in step order; the line's check is stream 0's batch, the other stream's is checked by the
    bench itself against its batch scanned again on one stream."""
    detail = tmp_path / "detail.json"
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2",
           "--streams", str(streams),
           "--reads", str(READS), "--no-extra", "--no-cpu-baseline", "--no-pcie", "--no-lf-compare",
           "--detail", str(detail)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SPEQ_BENCH_NO_STATS"] = "1"
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert "host-socket" in out["config"]["collective"]
    assert out["config"]["parallelism"].startswith("dp2")

    # one process, both shards (reads 0 .. 2n-1 of the same stream), same index options as the bench
    c = synth.CONFIGS[2]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True, label_table="auto",
                        threads=16, gpu_device=0, triple_steps=True)
    dev = DeviceIndex(idx, 0)
    try:
        reads = synth.make_reads(ref, 2 * READS, err_rate=0.001)
        r = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21)
    finally:
        dev.close()
    assert out["check"]["T"] == r.total
    assert out["check"]["ambiguous"] == r.ambiguous
    assert out["check"]["U_sha1"] == bench.u_sha1(r.unique)
    kmers = int(np.maximum(np.diff(reads.offsets).astype(np.int64) - 21 + 1, 0).sum())
    # value = all ranks' k-mers / max-over-ranks time
    assert out["streams"] == streams
    assert out["value"] == pytest.approx(kmers * 4 / (out["ms_per_step"] * 4 / 1e3), rel=1e-6)
    assert out["value_min"] <= out["value"] <= out["value_max"]


@pytest.mark.parametrize("allreduce", ["job", "step"])
def test_bench_rccl_one_rank_keeps_batches_in_flight(tmp_path, allreduce):
    """the 8-GPU line's code path on one GPU — torch's NCCL process group and the product's RCCL
    communicator (a one-member one) are initialised, every step's counters are all-reduced with ncclAllReduce on the
    communication stream — and the two scan streams must still overlap: the pipelined step at most 0.9x the one-stream
    step measured in the same run (the bench's median of its timed regions), with the counts of the HBM-resident
    config-2 batch equal to a plain scan of the same reads (the one-member all-reduce is the identity).
    Reference reduction replaced: /root/reference/src/fm_scanner.cpp:224-233."""
    n = 1_000_000
    detail = tmp_path / "detail.json"
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--transport", "rccl", "--steps", "20",
           "--warmup", "3", "--streams", "2", "--allreduce", allreduce, "--no-extra", "--no-cpu-baseline", "--no-pcie", "--no-lf-compare",
           "--detail", str(detail)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["SPEQ_BENCH_NO_STATS"] = "1"
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 1 and "RCCL" in out["config"]["collective"]
    assert out["one_stream"] is not None
    # the streams did not serialise behind RCCL's: pipelined <= 0.9 x one stream (overlap >= 1 / 0.9)
    det = json.loads(detail.read_text())["head"]["timing"]
    assert out["overlap"] >= 1.0 / 0.9, (out["overlap"], out["ms_per_step"], out["one_stream"], det)
    assert out["ms_per_step"] <= 0.9 * out["one_stream"]["ms_per_step"]

    c = synth.CONFIGS[2]
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=12, pair_steps=True, label_table="auto",
                        threads=16, gpu_device=0, triple_steps=True)
    dev = DeviceIndex(idx, 0)
    try:
        reads = synth.make_reads(ref, n, err_rate=0.001)
        r = dev.scan(reads.seq.tobytes(), reads.qual.tobytes(), reads.offsets, k=21)
    finally:
        dev.close()
    assert (out["check"]["T"], out["check"]["ambiguous"], out["check"]["U_sha1"]) == (
        r.total, r.ambiguous, bench.u_sha1(r.unique))
