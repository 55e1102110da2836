#!/usr/bin/env python3
"""Pinned host -> device copy bandwidth of one CaffeNet minibatch (50 MB uint8): one copy
on one stream vs the batch split over 2 / 4 streams (several SDMA engines), with and
without binding this process to the GPU's NUMA node."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.parallel.topology import bind_to_gpu_numa, gpu_numa_node  # noqa: E402

node = bind_to_gpu_numa(0) if os.environ.get("BIND") else -1
print("gpu numa node", gpu_numa_node(0), "bound", node, flush=True)
x = torch.randint(0, 256, (256, 3, 256, 256), dtype=torch.uint8).pin_memory()
d = torch.empty_like(x, device="cuda")
for ns in (1, 2, 4, 8):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    parts = x.chunk(ns)
    dparts = d.chunk(ns)
    for _ in range(3):
        for s, p, q in zip(streams, parts, dparts):
            with torch.cuda.stream(s):
                q.copy_(p, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        for s, p, q in zip(streams, parts, dparts):
            with torch.cuda.stream(s):
                q.copy_(p, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20
    print(f"{ns} stream(s): {dt * 1e3:.2f} ms per 50 MB batch = {x.numel() / dt / 1e9:.1f} GB/s", flush=True)
