#!/usr/bin/env python3
"""VGG conv1_2 shape (64 -> 64, 3x3, pad 1, 224x224): bf16 direct conv (conv3x3.hip) vs the e4m3
direct conv (conv3x3_fp8.hip) vs the fp8 implicit GEMM, forward and data gradient, at batch B
(default 256; per-image cost is what the b2048 step pays 2048x)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


_lib.kernels()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
s = ConvSpec(B, 224, 224, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1)
x = (torch.randn(B, 224, 224, 64, device="cuda")).to(torch.bfloat16)
w = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).to(torch.bfloat16)
b = torch.zeros(64, device="cuda")
dy = (torch.randn(B, 224, 224, 64, device="cuda") * 1e-3).to(torch.bfloat16)
fl = 2.0 * B * 224 * 224 * 64 * 64 * 9
sc = hip.Fp8Scales(4, "cuda")
xq = hip.quant_fp8(x, sc.slot(0))
wq = hip.quant_fp8(w, sc.slot(1))
res = {}
res["fwd bf16 direct"] = timed(lambda: hip.conv_forward(x, w, b, s, relu=True))
res["fwd fp8 direct"] = timed(lambda: hip.conv_forward_fp8(xq, wq, b, s, sc.deq(0), sc.deq(1), relu=True))
hip._DIRECT_FP8 = False
res["fwd fp8 gemm"] = timed(lambda: hip.conv_forward_fp8(xq, wq, b, s, sc.deq(0), sc.deq(1), relu=True))
hip._DIRECT_FP8 = True
res["dgrad bf16 direct"] = timed(lambda: hip.conv_backward(dy, x, w, s, True, gate=x))
ws = {"fp8_dgrad": (sc, 2, 3)}
res["dgrad fp8 direct (+dy quant, flip)"] = timed(lambda: hip.conv_backward(dy, x, w, s, True, gate=x, ws=dict(ws)))
res["quant_fp8 of x"] = timed(lambda: hip.quant_fp8(x, sc.slot(0)))
for k, v in res.items():
    print(f"{k:36s} {v:9.1f} us  {fl / v / 1e6:7.0f} TF/s")
