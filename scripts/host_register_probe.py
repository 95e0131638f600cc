#!/usr/bin/env python3
"""Probe (GPU box): can the FASTQ path skip its pinned-slot copy by registering the page-cache mapping of the file?

Times, for a config-2-sized file (316 MB) on local disk with the page cache warm:
  * hipHostRegister of the read-only mmap of the file (page pinning) and hipHostUnregister;
  * H2D copies from the registered mapping (one hipMemcpyAsync, and 8 MiB pieces on one stream);
  * H2D copies from a pinned buffer (the ceiling) and from the unregistered mapping (pageable);
  * a host memcpy of the mapping into a pinned buffer (what the pinned-slot path pays per byte, one thread).
Prints one JSON line per measurement. Usage: python scripts/host_register_probe.py [MB]"""
import ctypes as C
import json
import mmap
import os
import sys
import tempfile
import time

import torch

MB = int(sys.argv[1]) if len(sys.argv) > 1 else 316
hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
H2D = 1


def out(**kw):
    print(json.dumps(kw), flush=True)


def main():
    torch.cuda.init()
    n = MB << 20
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        path = os.path.join(td, "reads.fq")
        with open(path, "wb") as f:
            f.write(os.urandom(1 << 20) * MB)
        with open(path, "rb") as f:
            f.read()  # page cache warm
        fd = os.open(path, os.O_RDONLY)
        # the read-only shared mapping of the file (libc mmap: ctypes cannot take the address of a read-only mmap)
        libc = C.CDLL(None)
        libc.mmap.restype = C.c_void_p
        libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
        libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
        addr = libc.mmap(None, n, mmap.PROT_READ, mmap.MAP_SHARED, fd, 0)

        def copy(src, pieces):
            step = n // pieces
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(pieces):
                rc = hip.hipMemcpyAsync(C.c_void_p(d.data_ptr() + i * step), C.c_void_p(src + i * step), step, H2D,
                                        C.c_void_p(stream))
                if rc != 0:
                    raise RuntimeError(f"hipMemcpyAsync: {rc}")
            hip.hipStreamSynchronize(C.c_void_p(stream))
            return time.perf_counter() - t0

        # pageable mapping (the driver stages it through its own pinned buffers)
        for pieces in (1, MB // 8):
            dt = min(copy(addr, pieces) for _ in range(3))
            out(case="pageable_mmap", pieces=pieces, ms=round(dt * 1e3, 3), GBps=round(n / dt / 1e9, 1))
        # registered mapping
        for flags, name in ((0, "default"), (8, "read_only")):
            t0 = time.perf_counter()
            rc = hip.hipHostRegister(C.c_void_p(addr), n, flags)
            reg = time.perf_counter() - t0
            out(case="register", flags=name, rc=rc, ms=round(reg * 1e3, 3))
            if rc != 0:
                continue
            for pieces in (1, MB // 8):
                dt = min(copy(addr, pieces) for _ in range(3))
                out(case="registered_mmap", flags=name, pieces=pieces, ms=round(dt * 1e3, 3),
                    GBps=round(n / dt / 1e9, 1), with_register_GBps=round(n / (dt + reg) / 1e9, 1))
            t0 = time.perf_counter()
            hip.hipHostUnregister(C.c_void_p(addr))
            out(case="unregister", flags=name, ms=round((time.perf_counter() - t0) * 1e3, 3))
        # pinned ceiling and the host copy the pinned-slot path pays
        h = torch.empty(n, dtype=torch.uint8).pin_memory()
        for pieces in (1, MB // 8):
            dt = min(copy(h.data_ptr(), pieces) for _ in range(3))
            out(case="pinned", pieces=pieces, ms=round(dt * 1e3, 3), GBps=round(n / dt / 1e9, 1))
        t0 = time.perf_counter()
        C.memmove(h.data_ptr(), addr, n)
        dt = time.perf_counter() - t0
        out(case="host_memcpy_mmap_to_pinned_1thread", ms=round(dt * 1e3, 3), GBps=round(n / dt / 1e9, 1))
        libc.munmap(C.c_void_p(addr), n)
        os.close(fd)


if __name__ == "__main__":
    main()
