"""PCIe copy bandwidth with pinned host memory (256 MB, 10 copies each way).
Usage: python scripts/dbg/pcie_bw.py"""
import torch, time
n = 256 << 20
d = torch.empty(n, dtype=torch.uint8, device='cuda'); d.fill_(1)
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
for name, fn in (("D2H", lambda: h.copy_(d, non_blocking=True)), ("H2D", lambda: d.copy_(h, non_blocking=True))):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10): fn()
    torch.cuda.synchronize()
    print(name, round(10 * n / (time.perf_counter() - t) / 1e9, 1), "GB/s", flush=True)
