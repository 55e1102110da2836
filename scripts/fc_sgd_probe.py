#!/usr/bin/env python3
"""FC weight-gradient + SGD epilogue probe (CaffeNet fc6/fc7/fc8 shapes): fused EPI_SGD
GEMM vs plain fp32 wgrad GEMM vs the standalone solver_update kernel on the same
parameter count; prints us and effective HBM TB/s of each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm as G, hip  # noqa: E402

_lib.kernels()
dev = torch.device("cuda")


def med(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1000.0


hyper = torch.tensor([0.01, 0.9, 0.0005, 0.0, 1.0, 0, 0, 0], dtype=torch.float32, device=dev)
for name, (B, O, I) in {"fc6": (256, 4096, 9216), "fc7": (256, 4096, 4096), "fc8": (256, 1000, 4096)}.items():
    dy = (torch.randn(B, O, device=dev) * 0.01).to(torch.bfloat16)
    x = torch.randn(B, I, device=dev).to(torch.bfloat16)
    w = torch.randn(O, I, device=dev) * 0.01
    h = torch.zeros(O, I, device=dev)
    sh = w.to(torch.bfloat16)
    db = torch.zeros(O, device=dev)
    sgd = dict(w=w, h=h, shadow=sh, hyper=hyper, lr_mult=1.0, decay_mult=1.0, flags=0)
    t_sgd = med(lambda: G.linear_wgrad_sgd(dy, x, sgd, db))
    g = torch.zeros(O, I, device=dev)
    t_f32 = med(lambda: G.linear_wgrad(dy, x, g, accumulate=False))
    n = O * I
    tables = hip.solver_tables([(0, n, 1.0, 1.0)], n, dev)
    t_upd = med(lambda: hip.solver_update(0, w.view(-1), g.view(-1), [h.view(-1)], sh.view(-1), tables, hyper, 0, 0))
    print(f"{name}: fused_sgd {t_sgd:7.1f}us ({18 * n / t_sgd / 1e6:.2f} TB/s)  wgrad_f32 {t_f32:7.1f}us "
          f"({2 * B * O * I / t_f32 / 1e6:.0f} TF/s, {4 * n / t_f32 / 1e6:.2f} TB/s)  solver_update {t_upd:7.1f}us "
          f"({22 * n / t_upd / 1e6:.2f} TB/s)", flush=True)
    bw = torch.empty(n * 3 // 2, device=dev)
    t_cp = med(lambda: bw.copy_(w.view(-1).repeat(1)[: n * 3 // 2] if False else torch.empty(0, device=dev)) if False else bw.zero_())
    print(f"   memset {bw.numel() * 4 / 1e6:.0f}MB {t_cp:.1f}us ({bw.numel() * 4 / t_cp / 1e6:.2f} TB/s)", flush=True)
