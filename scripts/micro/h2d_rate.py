"""Pinned host -> device copy rate at the tracking step's upload size (65
images of 1280x720 u8 = 59.9 MB), alone on a side stream, and with a busy
kernel load on the default stream (the bench's situation)."""
import time

import torch

n = 65 * 1280 * 720
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(2)]
cs = torch.cuda.Stream()
for _ in range(3):
    with torch.cuda.stream(cs):
        d[0].copy_(h, non_blocking=True)
torch.cuda.synchronize()
N = 40
t0 = time.perf_counter()
for i in range(N):
    with torch.cuda.stream(cs):
        d[i % 2].copy_(h, non_blocking=True)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / N
print(f"H2D pinned {n / 1e6:.1f} MB: {dt * 1e3:.3f} ms per copy, {n / dt / 1e9:.1f} GB/s")
a = torch.randn(8192, 8192, device="cuda")
t0 = time.perf_counter()
for i in range(N):
    with torch.cuda.stream(cs):
        d[i % 2].copy_(h, non_blocking=True)
    for _ in range(4):
        a = a * 1.0000001 + 1e-9
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / N
print(f"H2D pinned with concurrent HBM-bound kernels: {dt * 1e3:.3f} ms per iteration")
d2h = torch.empty(n, dtype=torch.uint8).pin_memory()
t0 = time.perf_counter()
for i in range(N):
    with torch.cuda.stream(cs):
        d[0].copy_(h, non_blocking=True)
        d2h.copy_(d[1], non_blocking=True)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / N
print(f"H2D + D2H same stream: {dt * 1e3:.3f} ms per pair")
