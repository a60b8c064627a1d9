"""Host-side cost of issuing the step's 59.9 MB pinned H2D upload: torch
copy_(non_blocking=True) vs hipMemcpyAsync through ctypes, each on a side
stream, timed on the host (call return) and on the device (completion)."""
import ctypes
import time

import torch

n = 65 * 1280 * 720
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
cs = torch.cuda.Stream()
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpyAsync.restype = ctypes.c_int
for _ in range(3):
    with torch.cuda.stream(cs):
        d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
N = 20
for name in ("torch copy_", "hipMemcpyAsync"):
    host = 0.0
    t0 = time.perf_counter()
    for i in range(N):
        a = time.perf_counter()
        if name == "torch copy_":
            with torch.cuda.stream(cs):
                d.copy_(h, non_blocking=True)
        else:
            rc = hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(h.data_ptr()), n, 1,
                                    ctypes.c_void_p(cs.cuda_stream))
            assert rc == 0, rc
        host += time.perf_counter() - a
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{name}: host {host / N * 1e3:.3f} ms per call, {dt / N * 1e3:.3f} ms per copy (wall)")
