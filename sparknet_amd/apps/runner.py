"""Model-averaging training driver shared by CifarApp and ImageNetApp.

Per round (src/main/scala/apps/CifarApp.scala:95-136):
  1. (every ``test_every`` rounds, before training) test: each rank runs its test shard
     through the test net (weights shared with the train net), scores are all-reduced,
     accuracy = 100 * sum / #test minibatches  -> ``"%.2f% accuracy"``;
  2. every rank runs ``tau`` local solver steps on a random contiguous window of its
     shard (MinibatchSampler);
  3. weights are averaged with one RCCL all-reduce (no driver round trip).
Checkpoints at round boundaries (rank 0 writes the averaged .caffemodel, every rank its
own .solverstate since momentum is rank-local), resume, SIGINT/SIGHUP handling and a
fault-injection switch for resume tests.
"""
from __future__ import annotations

import os
import time

import torch

from .. import models
from ..core.solver import Solver
from ..data.prefetch import DeviceFeeder, HostBatchSource, SyntheticSource, WindowedSource
from ..engine import LocalSGDTrainer, fuse_relu
from ..parallel.comm import SyncSGDCallback
from ..utils.checkpoint import read_round_sidecar, save_caffemodel, write_round_sidecar
from ..utils.logging import TrainingLog
from .common import StopFlag, setup


class ListSource(HostBatchSource):
    def __init__(self, images, labels, batch, pin=True):
        self.images, self.labels, self.batch = images, labels.int(), batch
        self.n = images.shape[0] // batch
        self.i = 0
        self.pin = pin and torch.cuda.is_available()

    def next_batch(self):
        k = self.i % max(self.n, 1)
        self.i += 1
        sl = slice(k * self.batch, (k + 1) * self.batch)
        x, y = self.images[sl].contiguous(), self.labels[sl].contiguous()
        if self.pin:
            x, y = x.pin_memory(), y.pin_memory()
        return x, y


def evaluate(solver, feeder, n_batches: int, comm) -> tuple[list[float], list[str], int]:
    """SparkNet test(): per-rank sum of each output blob over its test batches, summed
    over ranks (CifarApp.scala:101-116, Solver::TestAndStoreResult)."""
    tn = solver.test_nets[0]
    acc = None
    from ..utils.trace import trace_range
    with trace_range("eval"):
        acc = _eval_batches(tn, feeder, n_batches)
    scores = acc.cpu().tolist() if acc is not None else [0.0] * len(tn.output_blobs)
    total = n_batches
    if comm is not None and comm.world_size > 1:
        scores = comm.allreduce_scores(scores + [float(n_batches)], device=solver.device
                                       if solver.device.type == "cuda" else None)
        total = int(scores.pop())
    return scores, [b.name for b in tn.output_blobs], total


def _eval_batches(tn, feeder, n_batches):
    acc = None
    for _ in range(n_batches):
        feeder.stage()
        feeder.prefetch()
        tn.forward()
        v = torch.stack([b.data.float().sum() for b in tn.output_blobs])
        acc = v if acc is None else acc + v
    return acc


def run(args, *, model: str, data_shape, crop: int, mean, scale: float, mirror: bool, classes: int,
        train_data=None, test_data=None, model_kw=None, log_name="training_log"):
    """``train_data`` / ``test_data``: (uint8 NCHW tensor, int labels) for THIS rank, or
    None for synthetic batches of ``data_shape`` (C, H, W)."""
    rank, world, dev, comm = setup(args)
    if callable(mean):  # e.g. a streamed, all-reduced mean image (ImageNetApp)
        mean = mean(comm)
    log = TrainingLog(args.log_dir, rank, name=log_name)
    C, H, W = data_shape
    kw = dict(train_batch=args.batch, test_batch=args.test_batch)
    kw.update(model_kw or {})
    sp = models.solver_for(model, **kw)
    if not len(sp.test_iter):
        sp.test_iter.append(1)
    solver = Solver(sp, device=dev, seed=args.seed + rank)
    if dev.type == "cuda":
        fuse_relu(solver.net)
        for tn in solver.test_nets:
            fuse_relu(tn)
        if getattr(args, "dtype", "bf16") == "fp8":
            from ..engine import enable_fp8
            log_fp8 = enable_fp8(solver.net)
        else:
            log_fp8 = 0
    if args.weights:
        solver.net.copy_trained_layers_from(args.weights)
    start_round = 0
    if args.resume:
        side = read_round_sidecar(args.resume + ".json")
        solver.restore(f"{args.resume}.rank{rank}.solverstate")
        start_round = side["round"]
        log.log(f"resumed from {args.resume} at round {start_round}")

    from ..data.native import NativeLoader
    if isinstance(train_data, (NativeLoader, HostBatchSource)):
        src = train_data  # native loader / streaming JPEG ring (data.stream)
    elif train_data is not None:
        src = WindowedSource(train_data[0], train_data[1], args.batch, args.tau, seed=args.seed * 101 + rank)
    else:
        src = SyntheticSource(args.batch, C, H, W, classes=classes, pool=4, seed=args.seed * 101 + rank)
    net = solver.net
    feeder = DeviceFeeder(src, net.blob_by_name("data"), net.blob_by_name("label"), crop=crop, mean=mean,
                          scale=scale, mirror=mirror, train=True, rng_state=net.ctx.rng_state, device=dev)
    tn = solver.test_nets[0]
    if isinstance(test_data, HostBatchSource):
        tsrc = test_data
        n_test = max(1, int(getattr(args, "test_batches", 0) or 10))
    elif test_data is not None:
        tsrc = ListSource(test_data[0], test_data[1], args.test_batch)
        n_test = tsrc.n
    else:
        tsrc = SyntheticSource(args.test_batch, C, H, W, classes=classes, pool=2, seed=10_000 + rank)
        n_test = 2
    tfeeder = DeviceFeeder(tsrc, tn.blob_by_name("data"), tn.blob_by_name("label"), crop=crop, mean=mean,
                           scale=scale, mirror=False, train=False, device=dev)
    if args.sync_sgd and comm is not None:
        solver.add_callback(SyncSGDCallback(comm, net))
    # sync SGD runs the eager step by default: the bucketed gradient all-reduces CAN be
    # captured with the iteration (engine.GraphStep runs the solver callbacks inside the
    # captured body; --sync-sgd-graph), but cross-rank collectives inside a replayed graph
    # have only been verified on a 1-rank RCCL group (tests/test_averaging_gpu.py)
    graph = dev.type == "cuda" and (not args.sync_sgd or getattr(args, "sync_sgd_graph", False))
    trainer = LocalSGDTrainer(solver, None if args.sync_sgd else comm, tau=args.tau, feeder=feeder,
                              use_graph=graph)
    if start_round == 0:
        trainer.broadcast_initial()
    trainer.round = start_round
    stop = StopFlag()
    log.log(f"{model}: {world} worker(s), batch {args.batch}, tau {args.tau}, device {dev}"
            + (f", fp8 forward in {log_fp8} layers" if dev.type == "cuda" and log_fp8 else ""))
    try:
        _rounds(args, solver, trainer, tfeeder, n_test, comm, log, stop, start_round, rank, world, dev)
    except BaseException:
        if comm is not None:
            comm.abort()  # peers exit now instead of waiting in the next collective
        raise
    log.close()
    if comm is not None:
        comm.close()
    return solver


def _rounds(args, solver, trainer, tfeeder, n_test, comm, log, stop, start_round, rank, world, dev):
    for r in range(start_round, args.rounds):
        if args.test_every and r % args.test_every == 0:
            scores, names, total = evaluate(solver, tfeeder, n_test, comm)
            for name, v in zip(names, scores):
                if "accuracy" in name or "top" in name:
                    log.log(f"{100.0 * v / max(total, 1):.2f}% accuracy ({name})", i=r)
            log.metric(event="test", round=r, **{n: v / max(total, 1) for n, v in zip(names, scores)})
        if r == args.fail_at_round and rank == getattr(args, "fail_rank", 0):
            log.log(f"fault injection: rank {rank} exits at round {r}")
            os._exit(3)
        t0 = time.perf_counter()
        log.log("training", i=r)
        loss = trainer.run_round()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        lv = float(loss) if loss is not None else float("nan")
        log.log(f"round done: loss {lv:.4f}, {world * args.batch * args.tau / dt:.1f} img/s", i=r)
        log.metric(event="round", round=r, loss=lv, seconds=dt, img_s=world * args.batch * args.tau / dt)
        req = stop.take()
        if (args.snapshot_every and (r + 1) % args.snapshot_every == 0) or req == "snapshot":
            checkpoint(solver, args.snapshot_prefix, r + 1, rank, comm)
            log.log(f"checkpoint at round {r + 1}")
        if req == "stop":
            log.log("stop requested")
            break


def checkpoint(solver, prefix: str, round_: int, rank: int, comm=None) -> None:
    """Round-boundary checkpoint: weights are identical on every rank after averaging, so
    rank 0 writes the .caffemodel; momentum is rank-local, so each rank writes its
    .solverstate; a JSON sidecar records the round counter."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    if rank == 0:
        save_caffemodel(solver.net, prefix + ".caffemodel")
    from .. import proto
    proto.write_binary(f"{prefix}.rank{rank}.solverstate", solver.solver_state(prefix + ".caffemodel"))
    if comm is not None:
        comm.barrier()
    if rank == 0:
        write_round_sidecar(prefix + ".json", round=round_, iter=solver.iter)
