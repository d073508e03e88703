"""PCIe copy roofs of this box: H2D and D2H alone and concurrently (pinned host memory, 256 MB
transfers, one stream per direction), GB/s.  The host-buffer entry's e2e rate is bounded by them."""
import time

import torch

n = 256 << 20
dev = torch.device("cuda", 0)
h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
d_a = torch.empty(n, dtype=torch.uint8, device=dev)
d_b = torch.ones(n, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def run(h2d: bool, d2h: bool, reps: int = 8) -> float:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_in, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_out.copy_(d_b, non_blocking=True)
    torch.cuda.synchronize()
    return reps * n / (time.perf_counter() - t0) / 1e9


run(True, True, 2)
print(f"H2D alone {run(True, False):.1f} GB/s   D2H alone {run(False, True):.1f} GB/s   "
      f"both at once {run(True, True):.1f} GB/s per direction")
