"""Teardown time of a GPU process by what it holds (tools/exit_probe.cpp): for each case, the time from the child's
last print (just before its _Exit) to its end as the parent sees it. Run on the GPU box from the repo root."""
import subprocess
import sys
import time

CASES = [(0, 0, 1, 0), (0, 0, 1, 4), (0, 0, 1, 8), (1024, 0, 64, 0), (2048, 300, 128, 0), (2048, 300, 128, 6)]


def once(vram, pinned, nbuf, streams):
    t_start = time.time()
    p = subprocess.Popen(["tools/build/exit_probe", str(vram), str(pinned), str(nbuf), str(streams)],
                         stdout=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    rc = p.wait()
    t_end = time.time()
    if rc != 0 or not line.strip():
        raise SystemExit(f"exit_probe {vram} {pinned} {nbuf} {streams}: rc {rc}")
    t_print = int(line) * 1e-9
    return t_print - t_start, t_end - t_print


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for rep in range(reps):
        for c in CASES:
            run, tail = once(*c)
            print(f"vram {c[0]:5d} MiB in {c[2]:3d} buffers, pinned {c[1]:4d} MiB, {c[3]} streams: start-to-print "
                  f"{run * 1e3:7.1f} ms, exit {tail * 1e3:7.1f} ms", flush=True)
            time.sleep(1.0)


if __name__ == "__main__":
    main()
