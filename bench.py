#!/usr/bin/env python3
"""Headline benchmark: AlexNet/CaffeNet (bvlc_reference_caffenet, 227x227) training
images/sec on N MI355X GPUs — SparkNet's ImageNetApp algorithm: per-GPU batch 256,
tau = 50 local SGD steps per round, then an RCCL all-reduce weight average.

Every timed step is a full training iteration: H2D of a uint8 256x3x256x256 synthetic
batch on a side stream, on-device random crop 227 + mirror + mean subtraction, forward,
backward, fused SGD/momentum/weight-decay update (bf16 compute, fp32 masters), and every
tau-th step the cross-GPU weight average.  Random-init weights, synthetic data.

Single GPU:  python bench.py --steps 50 --warmup 10
N GPUs:      python bench.py --gpus N ...   (starts N ranks itself: parallel/launch.py), or
             python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
                 --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
Every rank runs on its own GPU; the JSON line (rank 0) reports the whole-job img/s from the
slowest rank's time, the per-rank ms/step, the measured all-reduce time per averaging and
an RCCL bus-bandwidth probe of the 244 MB averaging payload at three bucket sizes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# dmabuf IPC is the only mode the host driver supports; torchrun-launched ranks must get it
# before their first GPU call exactly like parallel/launch.spawn_local's children
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

BASELINE_IMG_S = 193.2  # CaffeNet training, Caffe no-cuDNN, K40


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--model", default="caffenet", choices=["caffenet", "alexnet", "googlenet", "vgg16",
                                                            "cifar10_quick", "cifar10_full"])
    p.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: the model's train batch)")
    p.add_argument("--tau", type=int, default=50)
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"],
                   help="fp8: e4m3 forward and data-gradient products with per-tensor delayed scaling; fp32: the "
                        "reference's numerics (fp32 activations, im2col + exact-f32 MFMA products, ops/f32dev.py; "
                        "eager, no fusions) for a precision-matched comparison with the fp32 K40 number")
    p.add_argument("--fp8-min-work", type=float, default=1000.0,
                   help="--dtype fp8: only layers with at least this many forward MACs per input element "
                        "run e4m3 (engine.enable_fp8 min_macs_per_input; VGG-16 b512: 0 -> 7.3k, 1000 -> 8.0k, "
                        "bf16 7.6k img/s, profiles/r2_fp8_select_ab.txt)")
    p.add_argument("--no-fp8-dgrad", dest="fp8_dgrad", action="store_false",
                   help="--dtype fp8: keep the data gradients in bf16 (default: the data gradients of stride-1 "
                        "convs run as fp8 products too, engine.enable_fp8 dgrad; weight gradients stay bf16; "
                        "VGG-16 b2048 8.82k vs 8.47k img/s, profiles/r3_fp8_dgrad.txt)")
    p.add_argument("--no-fp8-wgrad", dest="fp8_wgrad", action="store_false",
                   help="--dtype fp8: keep the weight gradients in bf16 (default: layers with an fp8 forward AND an "
                        "fp8 data gradient also run their weight gradient as an fp8 product, reduction over pixels)")
    p.add_argument("--fp8-dgrad-format", default="e4m3", choices=["e4m3", "e5m2"],
                   help="fp8 data gradients: format of the quantised output gradients")
    p.add_argument("--overlap-update", action="store_true",
                   help="run large layers' solver updates on a side stream during backward")
    p.add_argument("--no-fuse-fc", action="store_true",
                   help="store InnerProduct weight gradients and update them in the solver kernel")
    p.add_argument("--streams", type=int, default=3,
                   help="HIP streams for parallel branches (Inception towers) inside the graph; 1 = sequential "
                        "(>= 3 uses the star topology, see engine.BranchStreams); GoogLeNet b128 with the "
                        "round-5 database: 1 / 2 / 3 / 4 / 6 streams = 18.1 / 20.2 / 21.4 / 20.7-20.8 / 20.1 k img/s "
                        "(profiles/r5_googlenet_streams.txt)")
    p.add_argument("--feed-group", type=int, default=2,
                   help="H2D minibatch copies issued in groups of this many steps under one copy/compute "
                        "fence pair (DeviceFeeder group; 1 = one fence pair per step: 97k vs 102-105k img/s "
                        "in the 20-step window, profiles/r2_feed_group_ab.txt)")
    p.add_argument("--share-gpu", action="store_true",
                   help="rehearse the N-rank path on ONE GPU: every rank runs on device 0 and the collectives "
                        "use gloo (RCCL refuses two ranks on one device); everything else is the production "
                        "path. The img/s of such a run is not a multi-GPU number")
    p.add_argument("--verify-average", action="store_true",
                   help="after the timed window, check that every rank holds bitwise-identical averaged "
                        "masters and that the bf16 shadow the graph reads is bf16(master) (JSON avg_check)")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--step-times", action="store_true",
                   help="record a GPU event after every timed step and print the per-step ms to stderr")
    p.add_argument("--cpu", action="store_true",
                   help="fp32 reference engine on the CPU with gloo (tests the launcher / JSON path; not a benchmark)")
    p.add_argument("--host-profile", action="store_true",
                   help="after the timed run, report the host time per step part (stderr)")
    p.add_argument("--save-tuned", default="",
                   help="merge this run's GEMM tile / split-K choices into a tuning database (JSON)")
    p.add_argument("--loss-trace", action="store_true",
                   help="print every timed step's loss (full precision) to stderr after the window")
    p.add_argument("--autotune", action="store_true",
                   help="time GEMM products the tuning database lacks on first use (off by default: the "
                        "committed database + cost model give every process and rank the same kernels; with "
                        "N > 1 ranks rank 0's choices are adopted by all before graph capture)")
    return p.parse_args()


DEFAULTS = {  # model: (batch, channels, src hw, crop, classes, mean, input scale)
    "caffenet": (256, 3, 256, 227, 1000, [104.0, 117.0, 123.0], 1.0),
    "alexnet": (256, 3, 256, 227, 1000, [104.0, 117.0, 123.0], 1.0),
    "googlenet": (128, 3, 256, 224, 1000, [104.0, 117.0, 123.0], 1.0),
    # msra-initialised 13-conv stack: unit-scale input keeps the random-init logits finite;
    # BASELINE config 5 sizes the per-GPU batch for the 288 GB of HBM: 512 (38 GB, 7.5k img/s;
    # 1024: 73 GB, 7.8k; 64: 6.5 GB, 6.1k — profiles/r2_vgg16_batch_sweep.txt)
    "vgg16": (2048, 3, 256, 224, 1000, [104.0, 117.0, 123.0], 0.017),
    "cifar10_quick": (100, 3, 32, 32, 10, [125.0, 123.0, 114.0], 1.0),
    "cifar10_full": (100, 3, 32, 32, 10, [125.0, 123.0, 114.0], 1.0),
}
HEADLINE = ("caffenet", "alexnet")


def main():
    args = parse()
    from sparknet_amd.parallel.launch import launched_world, spawn_local
    if args.share_gpu:
        os.environ["SN_SHARE_GPU"] = "1"  # inherited by the ranks spawn_local starts
    args.share_gpu = args.share_gpu or os.environ.get("SN_SHARE_GPU", "0") == "1"
    world_env = launched_world()
    if world_env is None and args.gpus > 1:
        # `python bench.py --gpus N`: start N ranks (one per GPU) before any GPU call here
        return spawn_local(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:])
    world = world_env or 1
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s); launch with "
              f"torch.distributed.run --nproc-per-node {args.gpus} or run `python bench.py --gpus {args.gpus}`",
              file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.model == "vgg16":
        # VGG-16 at per-GPU batch 2048 fills ~170 GB with tensors of 6-13 GB: cached blocks above
        # 1 GB are not split for smaller requests, so the caching allocator cannot fragment the
        # 288 GB into partly used giant segments (expandable segments are not supported on
        # ROCm here); set before the first HIP call
        os.environ.setdefault("PYTORCH_ALLOC_CONF", "max_split_size_mb:1024")
    import torch
    if args.cpu:
        dev = torch.device("cpu")
        numa = -1
    else:
        gpu = 0 if args.share_gpu else local_rank
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
        from sparknet_amd.parallel.topology import bind_to_gpu_numa
        numa = bind_to_gpu_numa(gpu) if world > 1 else -1

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    from sparknet_amd import models
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, SyntheticSource
    from sparknet_amd.engine import LocalSGDTrainer, enable_fp8, fuse_input_fold, fuse_relu
    from sparknet_amd.ops import _lib
    from sparknet_amd.parallel import Comm

    from sparknet_amd.parallel import diag
    rccl_log = None
    # SN_COMM_FORCE=1 under torch.distributed.run --nproc-per-node 1: the process group, the
    # initial broadcast and every window's averaging all-reduce run over RCCL at world 1
    force_comm = os.environ.get("SN_COMM_FORCE", "0") == "1" and "MASTER_ADDR" in os.environ
    if (world > 1 or force_comm) and dev.type == "cuda" and not args.share_gpu:
        rccl_log = diag.rccl_debug_env()  # channels / transports for the JSON (RCCL debug log)
    if dev.type == "cuda":
        _lib.kernels()
        from sparknet_amd.ops import gemm as G
        G.set_autotune(args.autotune)
    # --cpu runs gloo even on a GPU host (nccl has no CPU tensors)
    comm = (Comm(backend="gloo" if (args.share_gpu or dev.type != "cuda") else None,
                 device=dev if dev.type == "cuda" else None,
                 watchdog=True, timeout_s=600.0) if world > 1 or force_comm else None)
    bad = diag.check_placement(comm, args.gpus, args.share_gpu or dev.type != "cuda",
                               torch.cuda.current_device() if dev.type == "cuda" else local_rank, local_rank)
    if bad is not None:
        print(f"bench.py rank {rank}: FATAL placement error: {bad}", file=sys.stderr, flush=True)
        if comm is not None:
            comm.abort()
        return 3
    B, C, HW, crop, classes, mean, in_scale = DEFAULTS[args.model]
    B = args.batch or B
    kw = dict(train_batch=B, test_batch=max(1, min(B, 50)))
    if args.model in ("caffenet", "alexnet", "googlenet", "vgg16"):
        kw["crop"] = crop
    solver_param = models.solver_for(args.model, **kw)
    fp32 = args.dtype == "fp32"
    solver = Solver(solver_param, device=dev, seed=1701 + rank, build_test_nets=False,
                    dtype=torch.float32 if fp32 else None)
    net = solver.net
    if dev.type == "cuda":
        fuse_relu(net)  # (a no-op on fp32 nets: the fp32 device mode runs the plain layer graph)
    src = SyntheticSource(B, C, HW, HW, classes=classes, pool=3, seed=rank)
    feeder = DeviceFeeder(src, net.blob_by_name("data"), net.blob_by_name("label"), crop=crop, mean=mean,
                          scale=in_scale, mirror=True, train=True, rng_state=net.ctx.rng_state, device=dev,
                          group=args.feed_group)
    fused_fold = fuse_input_fold(net, feeder)  # augment writes conv1's S2D-folded input directly
    n_fp8 = (enable_fp8(net, args.fp8_min_work, dgrad=args.fp8_dgrad, dgrad_format=args.fp8_dgrad_format,
                        wgrad=args.fp8_dgrad and args.fp8_wgrad) if args.dtype == "fp8" else 0)
    trainer = LocalSGDTrainer(solver, comm, tau=args.tau, feeder=feeder,
                              use_graph=not args.no_graph and not args.cpu and not fp32,
                              overlap_update=args.overlap_update, fuse_fc=not args.no_fuse_fc,
                              streams=args.streams)
    trainer.broadcast_initial()

    # warmup (includes hipGraph capture and one averaging collective to set up RCCL)
    for _ in range(max(1, args.warmup)):
        trainer.local_step()
    if comm is not None:
        trainer.average()
    sync()
    if comm is not None:
        comm.barrier()
    sync()

    avg_events = []
    step_evs = []
    if args.step_times and dev.type == "cuda":
        step_evs.append(torch.cuda.Event(enable_timing=True))
        step_evs[0].record()
    t0 = time.perf_counter()
    loss = None
    averaged = False
    trace = []
    for k in range(args.steps):
        loss = trainer.local_step()
        if args.loss_trace:
            trace.append(loss.detach().clone() if hasattr(loss, "detach") else loss)
        if step_evs:
            step_evs.append(torch.cuda.Event(enable_timing=True))
            step_evs[-1].record()
        # every tau-th step averages; a timed window shorter than tau still ends with one
        # average so the collective is always inside the measurement
        if (k + 1) % args.tau == 0 or (k == args.steps - 1 and not averaged):
            if comm is not None and dev.type == "cuda":
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
                trainer.average()
                ev[1].record()
                avg_events.append(ev)
            elif comm is not None:
                trainer.average()
                avg_events.append(None)
            averaged = True
    if comm is not None:
        comm.barrier()
    sync()
    elapsed_rank = time.perf_counter() - t0
    elapsed = elapsed_rank
    if step_evs:
        ms = [step_evs[i].elapsed_time(step_evs[i + 1]) for i in range(len(step_evs) - 1)]
        print(f"rank {rank} step ms: " + " ".join(f"{v:.2f}" for v in ms), file=sys.stderr, flush=True)
    if trace:
        print(f"rank {rank} losses: " + " ".join(repr(float(v)) for v in trace), file=sys.stderr, flush=True)
    per_rank_ms = [round(1000.0 * elapsed_rank / args.steps, 3)]
    avg_ms = [e[0].elapsed_time(e[1]) for e in avg_events if e is not None]
    comm_info = avg_check = bucket_ms = numa_all = None
    if comm is not None:
        elapsed = comm.max_over_ranks(elapsed_rank)
        per_rank_ms = [round(1000.0 * v / args.steps, 3) for v in comm.allgather_float(elapsed_rank)]
        avg_check = None
        if args.verify_average:  # untimed: average once more so the window's last step is averaged
            trainer.average()
            avg_check = verify_average(comm, net, dev, sync)
        comm_info = comm_bench(comm, net.flat_data, dev, sync, iters=1 if args.share_gpu else 4)
        bucket_ms = diag.timed_bucket_allreduce(comm, net.flat_data, comm.average_bucket_bytes, sync)
        numa_all = comm.allgather_int(int(numa))
    final_loss = float(loss) if loss is not None else float("nan")

    ms = 1000.0 * elapsed / args.steps
    img_s = world * B * args.steps / elapsed
    if rank == 0:
        out = {
            "metric": ("images/sec AlexNet training (227x227) at 1/2/4/8 MI355X; scaling efficiency"
                       if args.model in HEADLINE else f"images/sec {args.model} training"),
            "value": round(img_s, 1),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / BASELINE_IMG_S, 2) if args.model in HEADLINE else None,
            "dtype": "fp8" if n_fp8 else ("fp32-cpu" if dev.type == "cpu" else ("fp32" if fp32 else "bf16")),
            "data": f"synthetic (uint8 {HW}x{HW} -> on-device random crop/mirror/mean), random-init weights",
            "config": {
                "model": f"{args.model} (bvlc_reference_caffenet / AlexNet)" if args.model == "caffenet"
                else args.model,
                "global_batch": B * world,
                "per_gpu_batch": B,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "algorithm": f"local SGD, tau={args.tau}, RCCL all-reduce weight averaging",
                "hipgraph": trainer.use_graph, "streams": args.streams, "feed_group": feeder.group, "fused_input_fold": fused_fold, "fp8_layers": n_fp8, "fp8_dgrad": (args.fp8_dgrad_format if n_fp8 and args.fp8_dgrad else None), "fp8_wgrad": bool(n_fp8 and args.fp8_dgrad and args.fp8_wgrad),
                "final_loss": round(final_loss, 4),
            },
            "rccl_world": comm.world_size if comm is not None else 1,
            "comm_backend": comm.backend if comm is not None else None,
            "share_gpu": bool(args.share_gpu),
            "average_buckets": (len(comm.bucket_ranges(net.flat_data.numel(), comm.average_bucket_bytes))
                                if comm is not None else 0),
            "per_rank_ms_per_step": per_rank_ms,
            "averages_in_window": len(avg_events) if comm is not None else 0,
            "allreduce_ms_per_average": round(sum(avg_ms) / len(avg_ms), 3) if avg_ms else None,
            "avg_payload_mb": round(net.flat_data.numel() * 4 / 1e6, 1),
            "max_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2) if dev.type == "cuda" else None,
            "numa_node_rank0": numa,
            # GEMM products run on the cost model's choice (no tuning-database entry); 0 on the
            # zoo models' bench configurations (tests/test_tune_db_gpu.py)
            "tune_misses": len(G.tune_misses()) if dev.type == "cuda" else None,
            "autotune": bool(args.autotune),
        }
        if comm is not None:
            out["diag"] = {
                "rccl_version": diag.rccl_version() if comm.backend == "nccl" else None,
                "rccl_log_rank0": diag.read_rccl_logs(rccl_log),
                "bucket_allreduce_ms": bucket_ms,
                "numa_node_per_rank": numa_all,
                "step_spread_pct": round(100.0 * (max(per_rank_ms) / max(min(per_rank_ms), 1e-9) - 1.0), 2),
            }
        if comm_info is not None:
            out["comm_bench"] = comm_info
        if avg_check is not None:
            out["avg_check"] = avg_check
        print(json.dumps(out), flush=True)
    if args.host_profile and trainer.step_fn is not None:
        host_profile(trainer, dev)
    if args.save_tuned and rank == 0:
        from sparknet_amd.ops import gemm as G
        print(f"tuning database {args.save_tuned}: {G.save_tune_db(args.save_tuned)} entries", file=sys.stderr)
    if comm is not None:
        comm.close()
    return 0


def verify_average(comm, net, dev, sync):
    """The timed window ended with an average (bench loop): every rank must now hold the
    SAME fp32 masters bit for bit, and the bf16 compute shadow — the buffer the captured
    graph's next replay reads, at the pointer it was captured with — must be bf16(master)."""
    import torch
    sync()
    flat = net.flat_data.detach()
    words = flat.view(torch.int32).to(torch.int64)
    # order-sensitive 64-bit checksum of the bit patterns (exact integer arithmetic)
    idx = torch.arange(1, words.numel() + 1, device=words.device, dtype=torch.int64) % 1000003
    digest = [int(words.sum().item()), int((words * idx).sum().item())]
    shadow_ok = True
    if net.flat_compute is not net.flat_data:
        shadow_ok = bool(torch.equal(net.flat_compute, flat.to(net.flat_compute.dtype)))
    gathered = [comm.allgather_int(d) for d in digest]
    equal = all(len(set(g)) == 1 for g in gathered)
    ok_all = comm.allgather_int(int(shadow_ok))
    return {"masters_equal_across_ranks": equal, "shadow_is_bf16_master": all(ok_all),
            "digest_rank0": digest, "ranks": comm.world_size}


def comm_bench(comm, flat, dev, sync, bucket_mb=(256, 64, 16), iters=4):
    """After the timed window: all-reduce a scratch copy of the flat fp32 weight buffer at
    several bucket sizes and report the RCCL bus bandwidth (2(n-1)/n * bytes / time), so a
    multi-GPU run records how well the averaging collective uses the xGMI links."""
    scratch = flat.detach().clone()
    n = comm.world_size
    out = {}
    saved = comm.bucket_bytes
    for mb in bucket_mb:
        comm.bucket_bytes = mb << 20
        comm.allreduce_sum(scratch)
        sync()
        comm.barrier()
        t = time.perf_counter()
        for _ in range(iters):
            comm.allreduce_sum(scratch)
        sync()
        dt = comm.max_over_ranks((time.perf_counter() - t) / iters)
        nbytes = scratch.numel() * 4
        out[f"bucket_{mb}MB"] = {"ms": round(1000 * dt, 3), "busbw_GBps": round(2 * (n - 1) / n * nbytes / dt / 1e9, 1)}
    comm.bucket_bytes = saved
    del scratch
    return out


def host_profile(trainer, dev, n=200):
    """Host-side cost of each part of a graph step (feeder, hyper staging, replay) against
    the GPU time of the same steps: tells whether a small model is launch-bound."""
    import torch
    g, s = trainer.step_fn, trainer.solver
    parts = {"feeder": 0.0, "hyper": 0.0, "replay": 0.0}
    # replay() cost on an idle device vs back to back: a launch that waits for the previous
    # instance of the same graph shows up as ~one GPU step only in the back-to-back calls
    torch.cuda.synchronize(dev)
    idle = []
    for _ in range(3):
        g.pre()
        s.stage_hyper()
        a = time.perf_counter()
        g.graph.replay()
        idle.append(1e6 * (time.perf_counter() - a))
        s.iter += 1
        torch.cuda.synchronize(dev)
    print("replay us on an idle device: " + " ".join(f"{v:.0f}" for v in idle), file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        g.pre()
        b = time.perf_counter()
        s.stage_hyper()
        c = time.perf_counter()
        g.graph.replay()
        d = time.perf_counter()
        s.iter += 1
        parts["feeder"] += b - a
        parts["hyper"] += c - b
        parts["replay"] += d - c
    host = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    print("host us/step: " + " ".join(f"{k}={1e6 * v / n:.1f}" for k, v in parts.items()) +
          f" total={1e6 * host / n:.1f}; wall us/step={1e6 * wall / n:.1f}", file=sys.stderr, flush=True)
    f = trainer.feeder
    if f is None:
        return
    sub = {"stage": 0.0, "prefetch": 0.0}
    for _ in range(n):
        a = time.perf_counter()
        f.stage()
        b = time.perf_counter()
        f.prefetch()
        sub["stage"] += b - a
        sub["prefetch"] += time.perf_counter() - b
    torch.cuda.synchronize(dev)
    x, _ = f.source.next_batch()
    dx = f.slots[0][0]
    a = time.perf_counter()
    for _ in range(n):
        with torch.cuda.stream(f.copy_stream):
            dx.copy_(x, non_blocking=True)
    sub["h2d_copy_only"] = time.perf_counter() - a
    torch.cuda.synchronize(dev)
    print("feeder us/step: " + " ".join(f"{k}={1e6 * v / n:.1f}" for k, v in sub.items()) +
          f" pinned={x.is_pinned()}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    sys.exit(main())
