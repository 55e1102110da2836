#!/usr/bin/env python3
"""A/B of the persistent ring-pipelined GEMM tiles (30-36, csrc/kernels/gemm_pk.h) against
the tuned one-shot tiles, on (1) dense shapes vs hipBLASLt and (2) every GEMM launch of one
eager training step of a model (the real implicit-conv geometry and epilogues).  Each pk
candidate's output is checked against the recorded configuration's output.

    python scripts/pk_probe.py [--model caffenet] [--dense] [--reps 8]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timed(fn, reps, passes=5):
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


def dense(args):
    from sparknet_amd.ops import gemm
    shapes = [("caffenet conv3 fwd", 43264, 384, 2304), ("caffenet conv2 fwd/g", 186624, 128, 1200),
              ("caffenet conv5 fwd/g", 43264, 128, 1728), ("vgg conv3_2 fwd", 802816, 256, 2304),
              ("vgg conv4_2 fwd", 200704, 512, 4608), ("fc6 fwd b256", 256, 4096, 9216),
              ("square 4096", 4096, 4096, 4096), ("square 8192", 8192, 8192, 8192)]
    for name, M, N, K in shapes:
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        reps = max(2, min(50, int(3e13 / fl)))
        rows = min(M, 2048)
        ref = x[:rows].float() @ w.float().t()
        res = []
        gemm._FORCE_TILE = -1
        t_def = timed(lambda: gemm.linear_fwd(x, w), reps)
        t_blas = timed(lambda: torch.matmul(x, w.t()), reps)
        for t in ([0, 11, 13, 16] + sorted(gemm.PK_TILES) if args.tiles is None else args.tiles):
            gemm._FORCE_TILE = t
            try:
                y = gemm.linear_fwd(x, w)
                err = ((y[:rows].float() - ref).abs().max() / ref.abs().max()).item()
                us = timed(lambda: gemm.linear_fwd(x, w), reps)
                res.append(f"{t}:{fl / us / 1e6:.0f}{'!' if err > 8e-3 else ''}")
            except RuntimeError:
                res.append(f"{t}:-")
        gemm._FORCE_TILE = -1
        print(f"{name:22s} {M:7d} {N:5d} {K:5d} tuned {fl / t_def / 1e6:6.0f}  blas {fl / t_blas / 1e6:6.0f}  "
              + " ".join(res), flush=True)
        del x, w, ref


def model(args):
    import bench
    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, SyntheticSource
    from sparknet_amd.engine import LocalSGDTrainer, fuse_input_fold, fuse_relu
    from sparknet_amd.ops import gemm

    dev = torch.device("cuda", 0)
    B, C, HW, crop, classes, mean, in_scale = bench.DEFAULTS[args.model]
    B = args.batch or B
    kw = dict(train_batch=B, test_batch=max(1, min(B, 50)))
    if args.model in ("caffenet", "alexnet", "googlenet", "vgg16"):
        kw["crop"] = crop
    solver = Solver(models.solver_for(args.model, **kw), device=dev, seed=1701, build_test_nets=False)
    net = solver.net
    fuse_relu(net)
    src = SyntheticSource(B, C, HW, HW, classes=classes, pool=3, seed=0)
    feeder = DeviceFeeder(src, net.blob_by_name("data"), net.blob_by_name("label"), crop=crop, mean=mean,
                          scale=in_scale, mirror=True, train=True, rng_state=net.ctx.rng_state, device=dev)
    fuse_input_fold(net, feeder)
    trainer = LocalSGDTrainer(solver, None, tau=50, feeder=feeder, use_graph=False)
    trainer.local_step()
    torch.cuda.synchronize()

    where = ["?"]
    for layer in net.layers:
        f, b = layer.forward, layer.backward

        def fw(*a, _f=f, _n=layer.name):
            where[0] = _n + ":fwd"
            return _f(*a)

        def bw(*a, _b=b, _n=layer.name):
            where[0] = _n + ":bwd"
            return _b(*a)
        layer.forward, layer.backward = fw, bw
    rec = []
    orig = gemm._launch

    def spy(*a, **k):
        rec.append((where[0], a, k))
        return orig(*a, **k)
    gemm._launch = spy
    trainer.local_step()
    torch.cuda.synchronize()
    gemm._launch = orig

    tot_old = tot_new = 0.0
    flops = 0.0
    print(f"{'layer:pass':26s} {'M':>7s} {'N':>5s} {'K':>6s} g  old(t/s)      us  best-pk(t/s)     us   err  all")
    for name, a, k in rec:
        a = list(a)
        M, N, K, groups = a[0], a[1], a[2], a[3]
        epi, out, deq = a[5], a[6], (a[19] if len(a) > 19 else k.get("deq"))
        tile, splits, kchunk = a[16], a[17], a[18]
        fl = 2.0 * M * N * K * groups
        flops += fl
        reps = max(2, min(40, int(2e12 / fl)))
        saved = out.clone()
        bg = a[12]
        bsaved = bg.clone() if bg is not None else None

        def restore():
            out.copy_(saved)
            if bg is not None:
                bg.copy_(bsaved)

        def run(t, s, kc):
            b = list(a)
            b[16], b[17], b[18] = t, s, kc
            orig(*b, **k)
        t_old = timed(lambda: run(tile, splits, kchunk), reps)
        tot_old += t_old
        if deq is not None or epi == gemm.EPI_SGD:
            tot_new += t_old
            print(f"{name:26s} {M:7d} {N:5d} {K:6d} {groups}  {tile:3d}/{splits:<3d} {t_old:8.1f}  (kept)", flush=True)
            continue
        restore()
        run(tile, splits, kchunk)
        ref = out.float().clone()
        scale = ref.abs().max().item() + 1e-6
        best = (t_old, tile, splits, 0.0)
        alls = []
        for t in (sorted(gemm.PK_TILES) if args.tiles is None else args.tiles):
            for s in dict.fromkeys((1, splits, gemm.choose_splits(M, N, K, groups, t)[0])):
                kc = -(-(-(-K // s)) // 64) * 64
                s2 = max(1, -(-K // kc))
                if s2 > 1 and s2 * M * N * groups * 4 > (256 << 20):
                    continue
                try:
                    restore()
                    run(t, s2, kc)
                except RuntimeError:
                    continue
                err = (out.float() - ref).abs().max().item() / scale
                us = timed(lambda: run(t, s2, kc), reps)
                alls.append(f"{t}/{s2}:{us:.0f}{'!' if err > 1e-2 else ''}")
                if err <= 1e-2 and us < best[0]:
                    best = (us, t, s2, err)
        restore()
        tot_new += best[0]
        print(f"{name:26s} {M:7d} {N:5d} {K:6d} {groups}  {tile:3d}/{splits:<3d} {t_old:8.1f}  {best[1]:3d}/{best[2]:<3d}"
              f" {best[0]:8.1f} {best[3]:.0e}  {' '.join(alls)}", flush=True)
    print(f"total GEMM: old {tot_old:.1f} us ({flops / tot_old / 1e6:.0f} TF/s)  best-with-pk {tot_new:.1f} us "
          f"({flops / tot_new / 1e6:.0f} TF/s)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--dense", action="store_true")
    ap.add_argument("--tiles", default=None, help="comma-separated candidate tiles ('' = time the recorded configs only)")
    args = ap.parse_args()
    if args.tiles is not None:
        args.tiles = [int(t) for t in args.tiles.split(",") if t]
    from sparknet_amd.ops import _lib
    _lib.kernels()
    if args.dense:
        dense(args)
    if args.model:
        model(args)


if __name__ == "__main__":
    main()
