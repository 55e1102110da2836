#!/usr/bin/env python3
"""Small-reduction data gradients of GoogLeNet's 1x1 convolutions (dX = dY W with K = the
layer's 16-160 output channels, N = its 480-512 input channels, M = 25088 / 100352 pixels,
ReLU gate of the layer below): every tile, with and without the gate, against the bytes the
product must move (dY + W + gate read, dX written).

    python scripts/smallk_probe.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timed(fn, reps=20, passes=5):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(passes):
        torch.cuda._sleep(1 << 18)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / reps)
    best.sort()
    return best[len(best) // 2]


def main():
    from sparknet_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    for M, N, K in ((25088, 512, 24), (25088, 512, 128), (100352, 256, 32), (25088, 480, 16)):
        dy = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, N, device=dev) * 0.1).to(torch.bfloat16)
        gate = torch.randn(M, N, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = (dy.float() @ w.float()) * (gate.float() > 0)
        nbytes = (M * K + K * N + 2 * M * N) * 2
        res = []
        for t in (-1, 0, 1, 2, 5, 10, 11, 12, 13, 16, 19, 20, 21):
            G._FORCE_TILE = t
            for g in (gate, None):
                def run():
                    G.gemm(M, N, K, G.Dense(dy, K, True), G.Dense(w, N, False), out, N, epi=G.EPI_BF16, gate=g,
                           splits=None if t < 0 else 1)
                try:
                    run()
                    torch.cuda.synchronize()
                except (RuntimeError, AssertionError):
                    continue
                if g is not None:
                    err = float((out.float() - ref).abs().max() / (ref.abs().max() + 1e-6))
                    if err > 2e-2:
                        res.append(f"{t}:ERR")
                        continue
                us = timed(run)
                res.append(f"{t}{'g' if g is not None else ''}:{us:.1f}")
        G._FORCE_TILE = -1
        print(f"M={M} N={N} K={K}: floor {nbytes / 5e12 * 1e6:.1f} us at 5 TB/s | " + " ".join(res), flush=True)


if __name__ == "__main__":
    main()
