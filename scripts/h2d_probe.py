"""H2D feed bandwidth on the box: one CaffeNet minibatch of uint8 256x256x3 images (50.3 MB)
from pinned host memory, as one copy, split over 2 / 4 copy streams, and (run under
HSA_ENABLE_SDMA=0 by the caller) through the blit-kernel path."""
import os
import sys
import time

import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n = B * 256 * 256 * 3
src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
src.random_(0, 255)
dst = torch.empty(n, dtype=torch.uint8, device="cuda")
streams = [torch.cuda.Stream() for _ in range(4)]


def run(k, reps=20):
    chunk = -(-n // k)
    for _ in range(3):
        for i in range(k):
            with torch.cuda.stream(streams[i]):
                dst[i * chunk:(i + 1) * chunk].copy_(src[i * chunk:(i + 1) * chunk], non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        for i in range(k):
            with torch.cuda.stream(streams[i]):
                dst[i * chunk:(i + 1) * chunk].copy_(src[i * chunk:(i + 1) * chunk], non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return dt


for k in (1, 2, 4):
    dt = run(k)
    print(f"SDMA={os.environ.get('HSA_ENABLE_SDMA', '1')} streams={k}: {n / 1e6:.1f} MB in {dt * 1e3:.3f} ms = "
          f"{n / dt / 1e9:.1f} GB/s", flush=True)
