"""Does the box copy host->device and device->host at the same time?  Pinned 512 MB buffers:
H2D alone, D2H alone, both at once on two streams, and both at once in 8 chunks each."""
import os
import sys
import time

import torch

torch.cuda.set_device(0)
NB = 512 << 20
h_a = torch.empty(NB, dtype=torch.uint8).pin_memory()
h_b = torch.empty(NB, dtype=torch.uint8).pin_memory()
d_a = torch.empty(NB, dtype=torch.uint8, device="cuda")
d_b = torch.empty(NB, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(f, reps=5):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def h2d():
    with torch.cuda.stream(s1):
        d_a.copy_(h_a, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_b.copy_(d_b, non_blocking=True)


def both():
    h2d()
    d2h()


def both_chunked(nc=8):
    c = NB // nc
    for i in range(nc):
        with torch.cuda.stream(s1):
            d_a[i * c:(i + 1) * c].copy_(h_a[i * c:(i + 1) * c], non_blocking=True)
        with torch.cuda.stream(s2):
            h_b[i * c:(i + 1) * c].copy_(d_b[i * c:(i + 1) * c], non_blocking=True)


for name, f, nbytes in [("H2D", h2d, NB), ("D2H", d2h, NB), ("H2D+D2H", both, 2 * NB),
                        ("H2D+D2H 8 chunks", both_chunked, 2 * NB)]:
    dt = run(f)
    print(f"{name:18s} {dt * 1e3:7.2f} ms  {nbytes / dt / 1e9:6.1f} GB/s", flush=True)
print("GPU_MAX_HW_QUEUES =", os.environ.get("GPU_MAX_HW_QUEUES"), file=sys.stderr)
