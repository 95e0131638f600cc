"""CPU: bench.py's stdout line stays driver-parseable (round 3's 22.8 KB line was not parsed: BENCH_r03 `parsed: null`).

The line builder runs on canned results as large as the real ones (20-entry work counters, 200-entry U and W vectors
per line, ten secondary lines); the line must stay under 8 KB and carry the BASELINE keys, `roofline` and
`cpu_baseline`, while the vectors and counters go to the detail file only."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _line(G=200, local=True):
    ax = {k: 123456789 for k in ("wave_iters", "lookup_lanes", "run_lanes", "lookup_waves", "run_waves",
                                 "run_windows", "deferred", "filter_pass", "p2_probes", "p2_verify", "chunks",
                                 "segments", "qual_bytes", "run_tallied", "run_granules", "refills", "busy_1_4",
                                 "busy_5_16", "busy_17_32", "busy_33_64")}
    rf = bench.roofline_of("no-such-key", 0.25e-3, 7.6e8, 3.08e8, 21, 130_000_000)
    rf["kernel"] = bench.KERNEL_NAME[3]
    cpu = {"value": 1.1e7, "unit": "k-mers/s", "cores": 16, "kind": "port", "checked": True,
           "sample": "x" * 180, "host": {"cpu_model": "AMD EPYC 9575F 64-Core Processor", "rule": "y" * 80},
           "hash_port": {"value": 3.3e8, "sample": "z" * 150}, "label_run_port": {"value": 1e9, "sample": "w" * 150}}
    timing = {"regions": 5, "steps_per_region": 20, "value_median": 5.1e11, "value_min": 5.012345e11,
              "value_max": 5.212345e11, "ms_per_step": [0.2561234] * 5, "avg_kernel_ms": [0.2481234] * 5,
              "avg_kernel_ms_median": 0.2481234, "avg_kernel_ms_min": 0.2461234, "avg_kernel_ms_max": 0.2501234,
              "one_stream": {"value": 4.1234567e11, "ms_per_step": 0.3161234, "ms_per_step_all": [0.3161234] * 5},
              "overlap": 1.2345678}
    return {"value": 5.1e11, "ms_per_step": 0.2561234, "avg_kernel_ms": 0.2481234, "k": 21, "mode": "local",
            "timing": timing,
            "workload": "w" * 160, "roofline": rf, "cpu_baseline": cpu,
            "check": {"T": 130000000, "ambiguous": 3633, "U_sha1": "0123456789abcdef", "W_sum": 1.23456789e8},
            "detail": {"U": [10 ** 8] * G, "W": [1.234567891234e7] * G if local else None, "ax_work": ax}}


def test_compact_line_is_small_and_complete():
    head = _line()
    lines = {name: _line() for name in ("local_mode", "k31", "cli_e2e", "k70_reference_defaults", "k70_err05",
                                        "fastq_e2e", "local_varq", "cfg5_paired", "cfg5_paired_local", "extra")}
    meta = {"metric": "k-mers scanned/sec (whole node) at k=21, 150 bp reads", "n_gpus": 8, "steps": 20,
            "warmup": 2, "detail_file": "profiles/r04/bench_detail_n8.json",
            "config": {"workload": "v" * 160, "k": 21, "reads_per_gpu": 1000000, "paired": False, "mode": "global",
                       "parallelism": "dp8 (reads sharded, index replicated)", "collective": "c" * 100,
                       "index_build_s": 0.2, "index_builder": "gpu", "fm_text_len": 1000021,
                       "kmer_table": {"bytes": 15733384, "build_s": 0.004}}}
    out = bench.compact_result(head, lines, meta)
    s = json.dumps(out)
    assert len(s) < bench.LINE_LIMIT, len(s)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in out
    assert out["roofline"]["frac"] is not None and out["roofline"]["bound"] == "hbm"
    assert {"achieved", "peak", "unit", "frac", "traffic", "avg_kernel_ms", "traffic_source"} <= set(out["roofline"])
    assert out["cpu_baseline"]["cores"] == 16 and out["cpu_baseline"]["kind"] == "port"
    assert "ax_work" not in s and "hash_port" not in s  # detail only
    assert out["overlap"] == pytest.approx(1.2345678) and out["one_stream"]["value"] == pytest.approx(4.1234567e11)
    assert out["value_min"] <= out["value"] <= out["value_max"]
    assert "median of 5 timed regions" in out["timing"]
    for r in out["lines"].values():
        assert {"value", "avg_kernel_ms", "frac", "traffic_frac", "check", "overlap"} <= set(r)
        assert "U" not in r["check"]


def test_roofline_uses_calibrated_fabric_bytes(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    key = bench.workload_key(2, 21, "global", 1_000_000, "ax")
    assert key == "cfg2_k21_global_reads1000000_ax"
    assert bench.workload_key(2, 70, "local", 1_000_000, "ax", err=0.005) == "cfg2_k70_local_reads1000000_ax_err0.005"
    (prof / "traffic.json").write_text(json.dumps({
        key: {"fabric_bytes_per_launch": 4.0e8, "source": "r04/pmc_x.json", "l2_hit_rate": 0.6},
        "old": {"hbm_bytes_per_launch": 2.5e8, "source": "r03/pmc_y.json"}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    rf = bench.roofline_of(key, 0.25e-3, 7.6e8, 3.08e8, 21, 130_000_000)
    assert rf["frac_basis"] == "fabric" and rf["traffic"] == 4.0e8
    assert rf["frac"] == pytest.approx(4.0e8 / 0.25e-3 / 1e9 / 8000.0)
    assert rf["traffic_frac"] == pytest.approx(rf["frac"])
    assert rf["l2_request_frac"] == pytest.approx(7.6e8 / 0.25e-3 / 1e9 / 8000.0)
    # an uncalibrated (pre-round-4) entry is not used: the compulsory read bytes are the basis then
    rf2 = bench.roofline_of("old", 0.25e-3, None, 3.08e8, 21, 130_000_000)
    assert rf2["frac_basis"] == "compulsory" and rf2["traffic"] is None
    assert rf2["frac"] == pytest.approx(3.08e8 / 0.25e-3 / 1e9 / 8000.0)


def test_write_fastq_round_trip(tmp_path):
    import numpy as np

    from speq_amd import synth
    ref = synth.make_reference(2, 1, 2000)
    reads = synth.make_reads(ref, 2500)
    p = tmp_path / "r.fq"
    n = bench.write_fastq(str(p), reads, chunk=1000)
    data = p.read_bytes()
    assert len(data) == n
    lines = data.split(b"\n")
    assert lines[0] == b"@r000000000" and lines[4 * 2499] == b"@r000002499"
    seq = b"".join(lines[1::4][:2500])
    assert seq == reads.seq.tobytes()
    assert b"".join(lines[3::4][:2500]) == reads.qual.tobytes()
    assert np.all(np.diff(reads.offsets) == 150)


# ---- bench.py --gpus N: who launches the ranks (decided before anything touches a GPU) ----

def test_launch_plan():
    assert bench.launch_plan(1, {}) == "run"
    assert bench.launch_plan(8, {}) == "relaunch"  # `python bench.py --gpus 8` starts its own 8 ranks
    assert bench.launch_plan(2, {"WORLD_SIZE": ""}) == "relaunch"
    assert bench.launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}) == "run"  # a rank of the driver's launcher
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == "run"
    for gpus, ws in ((1, "8"), (8, "4"), (2, "1")):
        with pytest.raises(bench.LaunchError):
            bench.launch_plan(gpus, {"WORLD_SIZE": ws})
    with pytest.raises(bench.LaunchError):
        bench.launch_plan(0, {})


def test_pick_transport():
    assert bench.pick_transport("auto", 1, 1) == "none"
    assert bench.pick_transport("rccl", 1, 1) == "rccl"   # forced: a one-member RCCL communicator (GPU test)
    assert bench.pick_transport("rccl", 1, 0) == "none"
    assert bench.pick_transport("host", 1, 1) == "none"
    assert bench.pick_transport("auto", 8, 8) == "rccl"   # the driver's 8-GPU node: one rank per GPU
    assert bench.pick_transport("auto", 2, 1) == "host"   # two ranks on the one-GPU box
    assert bench.pick_transport("host", 8, 8) == "host"
    assert bench.pick_transport("rccl", 2, 1) == "rccl"   # forced (RCCL will refuse to share the GPU)
    with pytest.raises(bench.LaunchError):
        bench.pick_transport("mpi", 2, 2)


def test_relaunch_cmd_keeps_the_arguments():
    cmd = bench.relaunch_cmd(4, ["--gpus", "4", "--steps", "5"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "5"]


def test_world_size_mismatch_exits_nonzero():
    """A launcher with WORLD_SIZE != --gpus: bench.py refuses before importing torch (no GPU needed)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 2, (p.returncode, p.stderr[-500:])
    assert "WORLD_SIZE=2" in p.stderr and p.stdout == ""
