"""Time the fused max-pool -> LRN kernels (csrc/kernels/pool_lrn.hip: pool_lrn_fwd, lrn_pool_bwd)
at CaffeNet b256's pool1/norm1 and pool2/norm2 shapes, with the bytes each must move and a
device copy of the same size as the bandwidth yardstick.  SN_KERNEL_LIB selects a kernel build
(same-box A/B of variants)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sparknet_amd.ops import hip  # noqa: E402
from sparknet_amd.ops.spec import PoolSpec  # noqa: E402

CASES = {"pool1/norm1": (256, 55, 55, 96), "pool2/norm2": (256, 27, 27, 256)}


def timeit(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def main():
    for name, (N, H, W, C) in CASES.items():
        s = PoolSpec(N, H, W, C, 3, 3, 2, 2, 0, 0)
        alpha, beta, k = 1e-4, 0.75, 1.0
        x = torch.randn(N, H, W, C, device="cuda").clamp_min(0).to(torch.bfloat16)
        pooled, mask, y = hip.pool_lrn_forward(x, s, True, 5, alpha, beta, k)
        dy = torch.randn_like(y)
        t_f = timeit(lambda: hip.pool_lrn_forward(x, s, True, 5, alpha, beta, k))
        t_b = timeit(lambda: hip.lrn_pool_backward(dy, pooled, mask, s, 5, alpha, beta, k))
        fwd_mb = (x.numel() * 2 + pooled.numel() * 5) / 1e6
        bwd_mb = (x.numel() * 2 + pooled.numel() * 5) / 1e6
        buf = torch.empty(int(bwd_mb * 1e6) // 2, dtype=torch.bfloat16, device="cuda")
        out = torch.empty_like(buf)
        t_c = timeit(lambda: out.copy_(buf))
        print(f"{name}: fwd {t_f:.1f} us ({fwd_mb / t_f:.2f} TB/s of {fwd_mb:.0f} MB) | bwd {t_b:.1f} us "
              f"({bwd_mb / t_b:.2f} TB/s of {bwd_mb:.0f} MB) | copy of {bwd_mb:.0f} MB {t_c:.1f} us", flush=True)


if __name__ == "__main__":
    main()
