#!/usr/bin/env python3
"""Pinned host -> device copy rate on the GPU box (torch), one and two streams: the PCIe ceiling of the streaming paths."""
import torch, time, json
for mb in (8, 16, 64, 300):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    for _ in range(3): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    reps = max(3, 2000 // mb)
    t0 = time.perf_counter()
    for _ in range(reps): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(json.dumps({"MB": mb, "GBps_h2d": round(n / dt / 1e9, 1)}), flush=True)
# two streams concurrently
n = 64 << 20
hs = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(2)]
ds = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(2)]
ss = [torch.cuda.Stream() for _ in range(2)]
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    for i in range(2):
        with torch.cuda.stream(ss[i]): ds[i].copy_(hs[i], non_blocking=True)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"two_streams_MB": 128, "GBps_h2d": round(20 * 2 * n / dt / 1e9, 1)}))
