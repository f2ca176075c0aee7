"""Lab: PCIe copy rates on one MI355X -- H2D alone, D2H alone, and both at once on two
streams (pinned host buffers, torch copies = hipMemcpyAsync), at the snappy e2e sizes
(0.61 GB of table bytes in, 1.07 GB of decoded values out), whole and in 64 MiB pieces."""
import time
import torch

dev = torch.device("cuda:0")
H, D = int(0.61e9), int(1.07e9)
hs = torch.empty(H, dtype=torch.uint8).pin_memory()
hd = torch.empty(D, dtype=torch.uint8).pin_memory()
ds = torch.empty(H, dtype=torch.uint8, device=dev)
dd = torch.empty(D, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
P = 64 << 20


def h2d(piece):
    with torch.cuda.stream(s1):
        for o in range(0, H, piece):
            ds[o:o + piece].copy_(hs[o:o + piece], non_blocking=True)


def d2h(piece):
    with torch.cuda.stream(s2):
        for o in range(0, D, piece):
            hd[o:o + piece].copy_(dd[o:o + piece], non_blocking=True)


def t(f, reps=3):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for piece in (max(H, D), P):
    a = t(lambda: h2d(piece))
    b = t(lambda: d2h(piece))
    c = t(lambda: (h2d(piece), d2h(piece)))
    print("piece %d MiB: H2D %.2f ms (%.1f GB/s)  D2H %.2f ms (%.1f GB/s)  both %.2f ms (sum %.2f)"
          % (piece >> 20, a, H / a / 1e6, b, D / b / 1e6, c, a + b), flush=True)
