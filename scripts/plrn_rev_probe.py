"""Time the LRN -> max-pool backward (csrc/kernels/pool_lrn.hip: pool_lrn_bwd_rev) against the
unfused pool_bwd_k3s2 + lrn_across_bwd at AlexNet b256 and GoogLeNet b128 shapes, bitwise check
included.  (The round-6 sweep of the phase-1 items per workgroup, 128-1024, is recorded in
profiles/r6_lrn_pool_rev.txt; the kernel now fixes 256.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sparknet_amd.ops import hip  # noqa: E402
from sparknet_amd.ops.spec import PoolSpec  # noqa: E402

CASES = {"alex_norm1": (256, 55, 55, 96), "alex_norm2": (256, 27, 27, 256), "goog_norm2": (128, 56, 56, 192)}


def timeit(fn, reps=20):
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
        y = hip.lrn_forward(x, 5, alpha, beta, k)
        _, mask = hip.pool_forward_mask(y, s, False)
        dy = torch.randn(N, s.P, s.Q, C, device="cuda").to(torch.bfloat16)

        def unfused():
            dl = hip.pool_backward(dy, y, s, mask)
            return hip.lrn_backward(dl, x, 5, alpha, beta, k, gate=True)

        ref = unfused()
        t_u = timeit(unfused)
        row = [f"{name} N={N} {H}x{W}x{C}: unfused {t_u:.1f} us"]
        fused = lambda: hip.pool_lrn_backward_rev(dy, mask, x, s, 5, alpha, beta, k, True)  # noqa: E731
        eq = torch.equal(fused(), ref)
        row.append(f"fused {timeit(fused):.1f} us{'' if eq else ' MISMATCH'}")
        mb = (x.numel() * 2 * 2 + dy.numel() * 2 + mask.numel()) / 1e6
        row.append(f"(fused floor traffic {mb:.0f} MB)")
        print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
