#!/usr/bin/env python3
"""Index build time, host SA-IS vs GPU (build_gpu.hip), per BASELINE config; one JSON line per build.
SPEQ_BUILD_TIMING=1 prints the phases to stderr."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,5")
    ap.add_argument("--host", type=int, default=1, help="also time the host build")
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch  # noqa: F401
    from speq_amd import FmIndex, synth
    for cfg in [int(x) for x in a.configs.split(",")]:
        c = synth.CONFIGS[cfg]
        ref = synth.make_reference(c["n_variants"], c["n_isolates"], c["length"])
        for gpu in ([None, 0] if a.host else [0]):
            t0 = time.perf_counter()
            idx = FmIndex.build(ref.records, ref.groups, c["n_variants"], prefix_q=11, pair_steps=True,
                                label_table=True, threads=a.threads, gpu_device=gpu)
            dt = time.perf_counter() - t0
            info = idx.info()
            print(json.dumps({"config": cfg, "builder": "host" if gpu is None else "gpu", "seconds": dt,
                              "n": info.n, "n_runs": info.n_runs, "device_bytes": info.device_bytes,
                              "threads": a.threads}), flush=True)
            del idx


if __name__ == "__main__":
    main()
