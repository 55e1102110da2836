#!/usr/bin/env python3
"""fp8 (e4m3, scaled MFMA) vs bf16 GEMM / conv throughput on identical shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from scripts.bench_kernels import timeit  # noqa: E402
from sparknet_amd.ops import _lib, gemm, hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402

_lib.kernels()
dev = "cuda"
one = torch.ones(1, device=dev)
for n in (4096, 8192):
    a = torch.randn(n, n, device=dev)
    b = torch.randn(n, n, device=dev)
    ab, bb = a.to(torch.bfloat16), b.to(torch.bfloat16)
    aq = a.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    bq = b.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    t16 = timeit(lambda: gemm.linear_fwd(ab, bb, out=c))
    t8 = timeit(lambda: hip.linear_forward_fp8(aq, bq, None, one, one))
    fl = 2 * n ** 3
    print(f"dense {n}^3: bf16 {fl / t16 / 1e9:7.1f} TF   fp8 {fl / t8 / 1e9:7.1f} TF", flush=True)
for name, s in {"vgg conv3_x": ConvSpec(64, 56, 56, 256, 256, 3, 3, 1, 1, 1, 1),
                "vgg conv4_x": ConvSpec(64, 28, 28, 512, 512, 3, 3, 1, 1, 1, 1),
                "vgg conv2_x": ConvSpec(64, 112, 112, 128, 128, 3, 3, 1, 1, 1, 1),
                "vgg conv1_2": ConvSpec(64, 224, 224, 64, 64, 3, 3, 1, 1, 1, 1)}.items():
    x = torch.randn(s.N, s.H, s.W, s.C, device=dev)
    w = torch.randn(s.K, s.R, s.S, s.Cg, device=dev) * 0.05
    xb, wb = x.to(torch.bfloat16), w.to(torch.bfloat16)
    xq = x.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    wq = (w * 64).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    t16 = timeit(lambda: hip.conv_forward(xb, wb, None, s))
    t8 = timeit(lambda: hip.conv_forward_fp8(xq, wq, None, s, one, one))
    sl = hip.Fp8Scales(1, dev)
    tq = timeit(lambda: hip.quant_fp8(xb, sl.slot(0)))
    fl = 2.0 * s.N * s.P * s.Q * s.K * s.R * s.S * s.Cg
    print(f"{name}: bf16 {fl / t16 / 1e9:7.1f} TF  fp8 {fl / t8 / 1e9:7.1f} TF  (quant of input {tq * 1e3:.1f} us)",
          flush=True)
