"""Fused LRN -> max-pool backward (csrc/kernels/pool_lrn.hip lrn_pool_bwd) at CaffeNet's two
shapes under LDS budgets / channel groups (SN_PLRN_LDS / SN_PLRN_CG, read per launch):
microseconds per launch and effective HBM rate (pooled + dy + mask read, dx written)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sparknet_amd.ops import hip  # noqa: E402
from sparknet_amd.ops.spec import PoolSpec  # noqa: E402

shapes = {"pool1/norm1": PoolSpec(256, 55, 55, 96, 3, 3, 2, 2), "pool2/norm2": PoolSpec(256, 27, 27, 256, 3, 3, 2, 2)}
budgets = [int(b) for b in (sys.argv[1].split(",") if len(sys.argv) > 1 and sys.argv[1] else
                            "12000,16000,20000,26000,32768,42000,56000,65536".split(","))]
cgs = [None] + [int(c) for c in (sys.argv[2].split(",") if len(sys.argv) > 2 else [])]
for name, s in shapes.items():
    x = torch.relu(torch.randn(s.N, s.H, s.W, s.C, device="cuda")).to(torch.bfloat16)
    pooled, mask, y = hip.pool_lrn_forward(x, s, False, 5, 1e-4, 0.75, 1.0)
    dy = torch.randn_like(y)
    refs = None
    for items in (64, 128, 256, 512):
        os.environ["SN_PLRN_FWD_ITEMS"] = str(items)
        outs = hip.pool_lrn_forward(x, s, False, 5, 1e-4, 0.75, 1.0)
        refs = refs or outs
        assert all(torch.equal(a, b) for a, b in zip(outs, refs))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            hip.pool_lrn_forward(x, s, False, 5, 1e-4, 0.75, 1.0)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 50
        fb = x.numel() * 2 + 2 * y.numel() * 2 + mask.numel()
        print(f"{name} forward items {items}: {us:.1f} us  {fb / us / 1e6:.2f} TB/s", flush=True)
    os.environ.pop("SN_PLRN_FWD_ITEMS")
    nbytes = 2 * pooled.numel() * 2 + mask.numel() + x.numel() * 2
    ref = None
    for cg, mlds in [(c, m) for m in ("0", "1") for c in cgs]:
        os.environ["SN_PLRN_MASK_LDS"] = mlds
        for b in budgets:
            os.environ["SN_PLRN_LDS"] = str(b)
            if cg is None:
                os.environ.pop("SN_PLRN_CG", None)
            else:
                os.environ["SN_PLRN_CG"] = str(cg)
            try:
                dx = hip.lrn_pool_backward(dy, pooled, mask, s, 5, 1e-4, 0.75, 1.0)
            except RuntimeError as e:
                print(f"{name} budget {b} cg {cg}: n/a ({e})")
                continue
            if ref is None:
                ref = dx.clone()
            assert torch.equal(dx, ref), "tile shape changed the result"
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                hip.lrn_pool_backward(dy, pooled, mask, s, 5, 1e-4, 0.75, 1.0)
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1000 / 50
            print(f"{name} mask_lds {mlds} budget {b} cg {cg}: {us:.1f} us  {nbytes / us / 1e6:.2f} TB/s", flush=True)
    z = torch.empty_like(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        z.copy_(x)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 50
    print(f"{name} reference: copy of the input-sized tensor {us:.1f} us = {2 * x.numel() * 2 / us / 1e6:.2f} TB/s")
