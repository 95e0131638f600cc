#!/usr/bin/env python3
"""End-to-end `speq` CLI on files (SURVEY 8(d) secondary metric): writes a BASELINE config's references, groupings
and FASTQ reads to a scratch directory, then times `speq index` and `speq scan` (FASTQ parse + H2D + scan + .dat
pass on the first run + EM refinement). One JSON line per command."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reads", type=int, default=0)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    a = ap.parse_args()
    from speq_amd import synth
    c = synth.CONFIGS[a.config]
    n = a.reads or c["n_reads"]
    work = tempfile.mkdtemp(prefix="speq_cli_", dir=a.dir)
    ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
    with open(os.path.join(work, "refs.fa"), "w") as f:
        for i, r in enumerate(ref.records):
            f.write(f">rec{i}\n{r.decode()}\n")
    with open(os.path.join(work, "groups.txt"), "w") as f:
        f.write(ref.groupings_text())
    reads = synth.make_reads(ref, n, paired=c["paired"])
    files = ["r1.fq", "r2.fq"] if c["paired"] else ["r1.fq"]
    handles = [open(os.path.join(work, fn), "wb") for fn in files]
    seq, qual = reads.seq.tobytes(), reads.qual.tobytes()
    for i in range(reads.n):
        s0, s1 = int(reads.offsets[i]), int(reads.offsets[i + 1])
        handles[i % len(handles) if c["paired"] else 0].write(b"@r%d\n%s\n+\n%s\n" % (i, seq[s0:s1], qual[s0:s1]))
    for h in handles:
        h.close()
    fq_bytes = sum(os.path.getsize(os.path.join(work, fn)) for fn in files)
    lens = np.diff(reads.offsets).astype(np.int64)
    kmers = int(np.maximum(lens - c["k"] + 1, 0).sum())
    speq = os.path.join(ROOT, "bin", "speq")
    env = dict(os.environ, SPEQ_STREAM_STATS="1", SPEQ_CLI_TIMING="1")

    def run(args, label):
        t0 = time.perf_counter()
        p = subprocess.run([speq] + args, cwd=work, capture_output=True, text=True, env=env)
        dt = time.perf_counter() - t0
        stream = [ln for ln in p.stderr.splitlines() if ln.startswith("speq: streamed")]
        phases = {}
        for ln in p.stderr.splitlines():
            if ln.startswith("speq: ") and ln.endswith(" s") and not ln.startswith("speq: streamed"):
                name, sec = ln[6:-2].rsplit(None, 1)
                phases[name.strip()] = float(sec)
        em_iters = p.stderr.count("\n\n")
        print(json.dumps({"config": a.config, "command": label, "rc": p.returncode, "seconds": dt,
                          "reads": reads.n, "kmers": kmers, "fastq_bytes": fq_bytes,
                          "kmers_per_s": kmers / dt if label.startswith("scan") else None,
                          "stream": stream[0] if stream else None, "em_iterations": em_iters, "phases": phases,
                          "stderr_tail": p.stderr[-300:] if p.returncode else None}), flush=True)
        return p.returncode

    rc = run(["index", "-r", "refs.fa", "-g", "groups.txt", "-x", "ref", "-t", str(a.threads)], "index")
    scan = ["scan", "-1", "r1.fq"] + (["-2", "r2.fq"] if c["paired"] else []) + \
        ["-x", "ref", "-k", str(c["k"]), "-t", str(a.threads), "--fixed-accuracy", "0.99", "-o", "out.txt"]
    if rc == 0:
        run(scan, "scan (first: + .dat pass)")
        run(scan[:-2] + ["-o", "out2.txt"], "scan (cached .dat)")
        run(scan[:-4] + ["-o", "out_local.txt"], "scan local/Phred (cached .dat)")
    subprocess.run(["rm", "-rf", work])


if __name__ == "__main__":
    main()
