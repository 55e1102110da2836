"""Micro-timings of the CaffeNet b256 pool/LRN pairs (fused vs unfused) and of the fused
augment + S2D input fold under its tile switches (SN_PLRN_LDS / SN_PLRN_CG,
SN_AUGMENT_DIRECT are read at every launch)."""
import os

import torch

from sparknet_amd.ops import hip
from sparknet_amd.ops.spec import ConvSpec, PoolSpec


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def setenv(**kw):
    for k, v in kw.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = str(v)


N = 256
for name, (H, C) in {"pool1/norm1": (55, 96), "pool2/norm2": (27, 256)}.items():
    s = PoolSpec(N, H, H, C, 3, 3, 2, 2, 0, 0)
    x = torch.randn(N, H, H, C, device="cuda").clamp_min(0).to(torch.bfloat16)
    dy = torch.randn(N, s.P, s.Q, C, device="cuda").to(torch.bfloat16)
    pooled, mask, y = hip.pool_lrn_forward(x, s, True, 5, 1e-4, 0.75, 1.0)
    t_uf = timeit(lambda: hip.lrn_forward(hip.pool_forward_mask(x, s, True)[0], 5, 1e-4, 0.75, 1.0))
    t_f = timeit(lambda: hip.pool_lrn_forward(x, s, True, 5, 1e-4, 0.75, 1.0))
    print(f"{name} fwd: unfused {t_uf:.1f} us, fused {t_f:.1f} us")
    t_ub = timeit(lambda: hip.pool_backward(hip.lrn_backward(dy, pooled, 5, 1e-4, 0.75, 1.0), x, s, mask))
    print(f"{name} bwd: unfused {t_ub:.1f} us")
    for lds in (24576, 32768):
        for cg in (None, C // 8):
            setenv(SN_PLRN_LDS=lds, SN_PLRN_CG=cg)
            try:
                t = timeit(lambda: hip.lrn_pool_backward(dy, pooled, mask, s, 5, 1e-4, 0.75, 1.0))
                print(f"{name} bwd fused lds={lds} cg={cg}: {t:.1f} us")
            except RuntimeError as e:
                print(f"{name} bwd fused lds={lds} cg={cg}: n/a ({str(e)[:40]})")
    setenv(SN_PLRN_LDS=None, SN_PLRN_CG=None)

s = ConvSpec(N, 227, 227, 3, 96, 11, 11, 4, 4, 0, 0)
plan = hip.s2d_plan(s)
img = torch.randint(0, 256, (N, 3, 256, 256), dtype=torch.uint8, device="cuda")
mean = torch.rand(3, device="cuda") * 200
rng = torch.tensor([11, 5], dtype=torch.int64, device="cuda")
x2 = torch.empty((N, plan[4].H, plan[4].W, plan[4].C), dtype=torch.bfloat16, device="cuda")
for direct in (1, None, 1, None):
    setenv(SN_AUGMENT_DIRECT=direct)
    print(f"augment_s2d {'direct' if direct else 'staged'} stores: "
          f"{timeit(lambda: hip.augment_s2d(img, x2, 227, plan, s, mean, 1, 1.0, rng, True, True)):.1f} us")
setenv(SN_AUGMENT_DIRECT=None)
