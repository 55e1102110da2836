"""2x2 / stride-2 max-pool backward at VGG-16's pool shapes (b256): one thread per window
block (pool_bwd_k2s2) vs the per-pixel gather (SN_POOL_K2S2=0); us per launch and the
effective HBM rate (dy + mask read, dx written)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sparknet_amd.ops import hip  # noqa: E402
from sparknet_amd.ops.spec import POOL_MAX, PoolSpec  # noqa: E402

for H, C in ((224, 64), (112, 128), (56, 256), (28, 512), (14, 512)):
    s = PoolSpec(256, H, H, C, 2, 2, 2, 2, 0, 0, POOL_MAX)
    x = torch.relu(torch.randn(256, H, H, C, device="cuda")).to(torch.bfloat16)
    _, mask = hip.pool_forward_mask(x, s, gate=True)
    dy = torch.randn(256, s.P, s.Q, C, device="cuda").to(torch.bfloat16)
    nbytes = x.numel() * 2 + dy.numel() * 2 + mask.numel()
    for v in ("0", "1"):
        os.environ["SN_POOL_K2S2"] = v
        hip.pool_backward(dy, x, s, mask, gate=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            hip.pool_backward(dy, x, s, mask, gate=True)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 20
        print(f"pool {H}x{H}x{C} k2s2={v}: {us:.1f} us  {nbytes / us / 1e6:.2f} TB/s", flush=True)
# GoogLeNet's 3x3 / stride-1 / pad-1 Inception pools at b128
for H, C in ((28, 192), (28, 256), (14, 480), (14, 528), (7, 832)):
    s = PoolSpec(128, H, H, C, 3, 3, 1, 1, 1, 1, POOL_MAX)
    x = torch.relu(torch.randn(128, H, H, C, device="cuda")).to(torch.bfloat16)
    _, mask = hip.pool_forward_mask(x, s, gate=True)
    dy = torch.randn(128, s.P, s.Q, C, device="cuda").to(torch.bfloat16)
    nbytes = x.numel() * 2 + dy.numel() * 2 + mask.numel()
    for v in ("0", "1"):
        os.environ["SN_POOL_K3S1"] = v
        hip.pool_backward(dy, x, s, mask, gate=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            hip.pool_backward(dy, x, s, mask, gate=True)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 20
        print(f"pool3s1 {H}x{H}x{C} k3s1={v}: {us:.1f} us  {nbytes / us / 1e6:.2f} TB/s", flush=True)
        e0.record()
        for _ in range(20):
            hip.pool_forward_mask(x, s, gate=True)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 20
        print(f"pool3s1 forward {H}x{H}x{C} k3s1={v}: {us:.1f} us  {nbytes / us / 1e6:.2f} TB/s", flush=True)
