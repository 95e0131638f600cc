"""The `speq` CLI (index|scan|all): options, defaults, cache files and stderr output of the reference.

CPU tests cover argument handling and `speq index`; `speq scan` needs the GPU (marked gpu)."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import cereal_dat
from golden_io import CASES, Case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPEQ = os.path.join(ROOT, "bin", "speq")


def run(args, cwd):
    return subprocess.run([SPEQ] + args, cwd=cwd, capture_output=True, text=True, timeout=300)


@pytest.fixture
def work(tmp_path):
    c = Case("tiny_single")
    for f in ("refs.fa", "groups.txt", "reads_1.fq"):
        shutil.copy(os.path.join(c.dir, f), tmp_path / f)
    return tmp_path


def test_help_and_unknown_subcommand(work):
    r = run(["--help"], work)
    assert r.returncode == 0 and "speq [index|scan|all]" in r.stdout
    r = run(["frobnicate"], work)
    assert r.returncode == 1 and "SPeQ Error" in r.stderr


def test_index_builds_and_is_cached(work):
    r = run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref", "-o", "out.txt"], work)
    assert r.returncode == 0, r.stderr
    idx = work / "ref.idx"
    assert idx.exists()
    m1 = idx.stat().st_mtime_ns
    # unchanged inputs: not rebuilt (fm_indexer.cpp:68-97)
    r = run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref.idx", "-o", "out2.txt"], work)
    assert r.returncode == 0 and idx.stat().st_mtime_ns == m1
    # -f forces a rebuild
    r = run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref.idx", "-o", "out2.txt", "-f"], work)
    assert r.returncode == 0 and idx.stat().st_mtime_ns != m1


def test_index_rebuilds_when_groupings_change(work):
    assert run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref", "-o", "o.txt"], work).returncode == 0
    m1 = (work / "ref.idx").stat().st_mtime_ns
    os.utime(work / "groups.txt", ns=(m1 + 10**9, m1 + 10**9))
    assert run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref", "-o", "o2.txt"], work).returncode == 0
    assert (work / "ref.idx").stat().st_mtime_ns != m1


def test_argument_errors(work):
    r = run(["index", "-r", "missing.fa", "-g", "groups.txt"], work)
    assert r.returncode == 1 and "argument parsing error" in r.stderr and "was not found" in r.stderr
    (work / "output.txt").write_text("x")
    r = run(["index", "-r", "refs.fa", "-g", "groups.txt"], work)  # default -o output.txt exists
    assert r.returncode == 1 and "Cowardly refusing" in r.stderr
    r = run(["scan", "-1", "reads_1.fq", "-x", "nope", "-o", "s.txt"], work)
    assert r.returncode == 1 and "was not found" in r.stderr
    r = run(["scan", "-1", "reads_1.fq", "-t", "1", "-o", "s.txt"], work)
    assert r.returncode == 1 and "threads" in r.stderr
    r = run(["scan", "-1", "reads_1.fq", "--fixed-accuracy", "1.5", "-o", "s.txt"], work)
    assert r.returncode == 1 and "fixed-accuracy" in r.stderr


def test_groupings_without_counts_fail_index(work):
    shutil.copy(os.path.join(ROOT, "tests", "golden", "genome_groupings.txt"), work / "g0.txt")
    r = run(["index", "-r", "refs.fa", "-g", "g0.txt", "-x", "bad", "-o", "o.txt"], work)
    assert r.returncode == 2 and "(count)" in r.stderr


def _parse_vec(line):
    assert line.startswith("[") and line.endswith("]"), line
    body = line[1:-1]
    return [float(x) for x in body.split(",")] if body else []


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("mode", ["global", "local"])
def test_scan_end_to_end(tmp_path, name, mode):
    c = Case(name)
    for f in os.listdir(c.dir):
        shutil.copy(os.path.join(c.dir, f), tmp_path / f)
    k = c.ks[0]
    e = c.exp["by_k"][str(k)]
    r = run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref", "-o", "i.txt", "--prefix-q", "4"], tmp_path)
    assert r.returncode == 0, r.stderr
    args = ["scan", "-1", "reads_1.fq", "-x", "ref", "-k", str(k), "--phred-cutoff", str(c.cutoff)]
    if c.paired:
        args += ["-2", "reads_2.fq"]
    if mode == "global":
        args += ["--fixed-accuracy", str(c.exp["fixed_accuracy"])]
    r = run(args + ["-o", "p.txt"], tmp_path)
    assert r.returncode == 0, r.stderr
    lines = r.stderr.strip().split("\n")
    # first scan computes the .dat pass and prints U_ref / Tot_ref (fm_scanner.cpp:1572-1573)
    assert _parse_vec(lines[0]) == e["u_ref"] and _parse_vec(lines[1]) == e["tot_ref"]
    # the .dat holds cereal's bytes of {file_time_type of the .idx, U_ref, Tot_ref} (fm_scanner.cpp:1561-1571)
    dat = (tmp_path / f"ref_{k}mer.dat").read_bytes()
    stamp = cereal_dat.file_time_ns((tmp_path / "ref.idx").stat().st_mtime_ns)
    assert dat == cereal_dat.encode(stamp, [int(x) for x in e["u_ref"]], [int(x) for x in e["tot_ref"]])
    g = e[mode]
    np.testing.assert_allclose(_parse_vec(lines[2]), g["percent"], rtol=1e-5)
    tl = [ln for ln in lines if "\t" in ln]
    assert tl[0] == f"{g['T']}\t{g['ambiguous']}"
    if c.paired and mode == "local":  # fusion map with its always-empty key (fm_scanner.cpp:916, :1033)
        fm = lines[lines.index(tl[0]) + 1]
        assert fm == (f"[([],{g['ambiguous']})]" if g["ambiguous"] else "[]")
    # second scan reuses the .dat (no U_ref/Tot_ref lines) and writes the percentages to -o
    r2 = run(args + ["-o", "p2.txt"], tmp_path)
    assert r2.returncode == 0
    assert r2.stderr.strip().split("\n")[0] == lines[2]
    out = (tmp_path / "p2.txt").read_text().strip().split("\n")
    assert len(out) == c.G
    # EM refinement: one stderr block per iteration, and -o holds the refined percentages
    em = g["em"]
    blocks = r.stderr.strip().split("\n\n")
    assert len(blocks) == len(em)  # the first iteration follows the initial lines directly
    last = blocks[-1].split("\n")
    if mode == "local" and not c.paired:
        assert last[0].startswith("1: ") and last[3].startswith("Percent of each group: ")
        np.testing.assert_allclose(_parse_vec(last[2][3:]), em[-1]["next_tkpg"], rtol=1e-5)
    else:
        np.testing.assert_allclose(_parse_vec(last[1]), em[-1]["next_tkpg"], rtol=1e-5)
    got = [float(ln.split("\t")[1]) for ln in out]
    np.testing.assert_allclose(got, em[-1]["percent"], rtol=1e-5, atol=1e-9)


@pytest.mark.gpu
def test_all_subcommand_and_gzip_reads(tmp_path):
    """`speq all` (index + scan in one call) on gzip-compressed reads gives the same percentages as index then
    scan on the plain file."""
    import gzip
    c = Case("tiny_single")
    for f in os.listdir(c.dir):
        shutil.copy(os.path.join(c.dir, f), tmp_path / f)
    with open(tmp_path / "reads_1.fq", "rb") as f, gzip.open(tmp_path / "reads_1.fq.gz", "wb") as g:
        g.write(f.read())
    k = c.ks[0]
    r = run(["all", "-r", "refs.fa", "-g", "groups.txt", "-1", "reads_1.fq.gz", "-x", "ref", "-k", str(k),
             "--phred-cutoff", str(c.cutoff), "--prefix-q", "5", "-o", "pa.txt"], tmp_path)
    assert r.returncode == 0, r.stderr
    r2 = run(["scan", "-1", "reads_1.fq", "-x", "ref", "-k", str(k), "--phred-cutoff", str(c.cutoff),
              "-o", "pb.txt"], tmp_path)
    assert r2.returncode == 0, r2.stderr
    assert (tmp_path / "pa.txt").read_text() == (tmp_path / "pb.txt").read_text()
    g = c.exp["by_k"][str(k)]["local"]
    tl = [ln for ln in r.stderr.split("\n") if "\t" in ln]
    assert tl[0] == f"{g['T']}\t{g['ambiguous']}"


@pytest.mark.gpu
@pytest.mark.parametrize("paired", [False, True])
def test_scan_sharded_over_replicas_matches_one_gpu(tmp_path, paired):
    """`speq scan --devices 0,0,0` (three replicas: reads dealt across them, the .dat pass split three ways, EM
    histograms merged) prints exactly what the one-GPU scan prints, and `--gpus 0` (every visible GPU) too."""
    from speq_amd import synth
    from test_gpu_stream import split, write_fastq
    ref = synth.make_reference(4, 2, 20_000)
    reads = synth.make_reads(ref, 60_000 if paired else 120_000, paired=paired, lowq_rate=0.002)
    (tmp_path / "refs.fa").write_text(ref.fasta_text())
    (tmp_path / "groups.txt").write_text(ref.groupings_text())
    seqs, quals = split(reads)
    if paired:
        write_fastq(tmp_path / "r1.fq", seqs[0::2], quals[0::2])
        write_fastq(tmp_path / "r2.fq", seqs[1::2], quals[1::2])
    else:
        write_fastq(tmp_path / "r1.fq", seqs, quals)
    r = run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref", "-o", "i.txt"], tmp_path)
    assert r.returncode == 0, r.stderr
    base = ["scan", "-1", "r1.fq", "-x", "ref", "-k", "21", "-t", "4", "--fixed-accuracy", "0.99"]
    if paired:
        base += ["-2", "r2.fq"]
    outs = {}
    for name, extra in (("one", []), ("three", ["--devices", "0,0,0"]), ("all", ["--gpus", "0"])):
        for f in tmp_path.glob("ref_21mer.dat"):
            f.unlink()  # every run recomputes the .dat pass (sharded when several replicas)
        r = run(base + extra + ["-o", f"{name}.txt", "-f"], tmp_path)
        assert r.returncode == 0, r.stderr
        outs[name] = (r.stderr, (tmp_path / f"{name}.txt").read_text())
    assert outs["three"] == outs["one"]
    assert outs["all"] == outs["one"]
    assert "\t" in outs["one"][0]


@pytest.mark.gpu
@pytest.mark.parametrize("paired", [False, True])
def test_scan_one_process_per_gpu_matches_one_process(tmp_path, paired):
    """`torchrun --no-python bin/speq scan ...` with WORLD_SIZE = 2: each rank scans its share of the FASTQ blocks
    and of the .dat windows on GPU $LOCAL_RANK and the counters, weights, .dat sums and EM histograms are summed
    (speq_allreduce_host / speq_em_allreduce); rank 0 prints and writes exactly what one process prints. With one
    visible GPU both ranks use GPU 0 (--device 0) and speq_comm_connect picks the host-socket transport (RCCL refuses
    two ranks on one GPU); with two or more GPUs the ranks use RCCL."""
    import socket
    import sys
    from speq_amd import synth
    from test_gpu_stream import split, write_fastq
    ref = synth.make_reference(4, 2, 20_000)
    reads = synth.make_reads(ref, 60_000 if paired else 120_000, paired=paired, lowq_rate=0.002)
    (tmp_path / "refs.fa").write_text(ref.fasta_text())
    (tmp_path / "groups.txt").write_text(ref.groupings_text())
    seqs, quals = split(reads)
    if paired:
        write_fastq(tmp_path / "r1.fq", seqs[0::2], quals[0::2])
        write_fastq(tmp_path / "r2.fq", seqs[1::2], quals[1::2])
    else:
        write_fastq(tmp_path / "r1.fq", seqs, quals)
    r = run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref", "-o", "i.txt"], tmp_path)
    assert r.returncode == 0, r.stderr
    base = ["scan", "-1", "r1.fq", "-x", "ref", "-k", "21", "-t", "4"] + (["-2", "r2.fq"] if paired else [])
    one = run(base + ["-o", "one.txt", "-f"], tmp_path)
    assert one.returncode == 0, one.stderr
    one_dat = (tmp_path / "ref_21mer.dat").read_bytes()
    (tmp_path / "ref_21mer.dat").unlink()  # the ranks recompute the .dat pass, split two ways
    import torch
    extra = [] if torch.cuda.device_count() >= 2 else ["--device", "0"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, SPEQ_RENDEZVOUS=str(tmp_path / "rdzv"))
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), "--no-python", SPEQ] + base +
                         extra + ["-o", "two.txt", "-f"], cwd=tmp_path, capture_output=True, text=True, timeout=300,
                         env=env)
    assert two.returncode == 0, two.stderr[-3000:]
    assert (tmp_path / "two.txt").read_text() == (tmp_path / "one.txt").read_text()
    for line in one.stderr.splitlines():  # every result line of the one-process run, once, from rank 0
        assert line in two.stderr, line
    assert (tmp_path / "ref_21mer.dat").read_bytes() == one_dat  # written by rank 0 from the summed shards


def test_cereal_dat_restatement_round_trips():
    """The cereal restatement the .dat tests use: fixed layout (i64 stamp, u64 n, u64[n], u64 n, u64[n])."""
    b = cereal_dat.encode(-5, [1, 2, 3], [4, 5, 6])
    assert len(b) == 8 + 2 * (8 + 3 * 8) and b[:8] == (-5).to_bytes(8, "little", signed=True)
    assert cereal_dat.decode(b) == (-5, [1, 2, 3], [4, 5, 6])
    assert cereal_dat.file_time_ns(6437664000 * 10**9) == 0


@pytest.mark.gpu
def test_scan_reads_a_cereal_dat_and_recounts_a_stale_one(work):
    """A .dat written by cereal (restated in tests/cereal_dat.py) with the .idx's file time is used as is: the
    scan prints no U_ref/Tot_ref lines and its percentages follow the file's U_ref (here doubled, so every
    percentage halves; fm_scanner.cpp:89-121, :1455-1474). A .dat with another stamp is recomputed and rewritten
    (:97-107)."""
    c = Case("tiny_single")
    k = c.ks[0]
    e = c.exp["by_k"][str(k)]
    r = run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref", "-o", "i.txt", "--prefix-q", "4"], work)
    assert r.returncode == 0, r.stderr
    args = ["scan", "-1", "reads_1.fq", "-x", "ref", "-k", str(k), "--phred-cutoff", str(c.cutoff), "-o", "p.txt",
            "-f"]
    stamp = cereal_dat.file_time_ns((work / "ref.idx").stat().st_mtime_ns)
    u = [int(x) for x in e["u_ref"]]
    t = [int(x) for x in e["tot_ref"]]
    dat = work / f"ref_{k}mer.dat"
    dat.write_bytes(cereal_dat.encode(stamp, [2 * x for x in u], t))
    r = run(args, work)
    assert r.returncode == 0, r.stderr
    lines = r.stderr.strip().split("\n")
    np.testing.assert_allclose(_parse_vec(lines[0]), np.asarray(e["local"]["percent"]) / 2, rtol=1e-5)
    dat.write_bytes(cereal_dat.encode(stamp - 1, [2 * x for x in u], t))  # stale: recounted and rewritten
    r = run(args, work)
    assert r.returncode == 0, r.stderr
    lines = r.stderr.strip().split("\n")
    assert _parse_vec(lines[0]) == e["u_ref"] and _parse_vec(lines[1]) == e["tot_ref"]
    np.testing.assert_allclose(_parse_vec(lines[2]), e["local"]["percent"], rtol=1e-5)
    assert cereal_dat.decode(dat.read_bytes()) == (stamp, u, t)
