"""Raw PCIe copy rates on the box (pinned host <-> device): the ceiling of the host-resident rate."""
import time

import torch

dev = torch.device("cuda:0")
for mb in (8, 64, 256):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    for name, f in (("H2D", lambda: d.copy_(h, non_blocking=True)), ("D2H", lambda: h.copy_(d, non_blocking=True))):
        f()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 10
        print(f"{name} {mb} MiB: {n / dt / 1e9:.1f} GB/s", flush=True)
