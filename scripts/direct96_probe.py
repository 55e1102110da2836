#!/usr/bin/env python3
"""GoogLeNet conv2/3x3 (128 x 56 x 56 x 64 -> 192, 3x3 pad 1): the implicit-GEMM forward vs the
LDS-resident direct kernel (csrc/kernels/conv3x3.hip) run as two 96-output halves — is the
direct form worth an output-stride variant?  Times only (the halves write 96-wide outputs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(fn, reps=20, passes=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(passes):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(out)[len(out) // 2]


from sparknet_amd.ops import _lib, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402
N, H, W, C = 128, 56, 56, 64
x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
for K in (192, 96, 64):
    s = ConvSpec(N, H, W, C, K, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    w = (torch.randn(K, 3, 3, C, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.randn(K, device="cuda")
    hip._DIRECT96 = False
    tg = timed(lambda: hip.conv_forward(x, w, b, s, relu=True))
    hip._DIRECT96 = True
    ts = timed(lambda: hip.conv_forward(x, w, b, s, relu=True))
    td = None
    if K in (64, 96):
        y = torch.empty(N, H, W, K, device="cuda", dtype=torch.bfloat16)
        td = timed(lambda: _lib.call("conv3x3_direct", x, w, b, None, y, N, H, W, C, K, 1, 1, 0))
    fl = 2.0 * N * H * W * K * 9 * C
    print(f"K={K}: implicit GEMM {tg:7.1f} us ({fl / tg / 1e6:.0f} TF/s), dispatched {ts:7.1f} us" +
          (f" | direct {td:7.1f} us ({fl / td / 1e6:.0f} TF/s)" if td else ""), flush=True)

# 1x1, 64 -> 64 (GoogLeNet conv2/3x3_reduce) on the packed direct kernel's <1, 64> instance
s = ConvSpec(N, H, W, C, 64, 1, 1, 1, 1, 0, 0, 1, 1, 1)
w = (torch.randn(64, 1, 1, C, device="cuda") * 0.05).to(torch.bfloat16)
b = torch.randn(64, device="cuda")
hip._PACKED11 = False
tg = timed(lambda: hip.conv_forward(x, w, b, s, relu=True))
hip._PACKED11 = True
tp = timed(lambda: hip.conv_forward(x, w, b, s, relu=True))
print(f"1x1 64->64: implicit GEMM {tg:7.1f} us | packed <1, 64> {tp:7.1f} us", flush=True)
