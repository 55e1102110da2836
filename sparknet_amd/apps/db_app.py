"""DB-backed apps: CifarDBApp, ImageNetCreateDBApp and ImageNetRunDBApp
(src/main/scala/apps/CifarDBApp.scala:23-171, ImageNetCreateDBApp.scala:19-135,
ImageNetRunDBApp.scala:19-117).

``create`` — every rank writes its shard of the training and test data into its own
database (LevelDB by default, like the reference; ``--backend lmdb`` or ``sndb``), the
mean image is computed from per-rank partial sums plus one all-reduce and saved as
``mean.binaryproto``, and the per-rank test batch counts go to
``num_test_batches.txt`` (ImageNetCreateDBApp.scala:79-87).

``train`` — every rank builds the zoo model with Caffe ``Data`` layers reading its own
databases (transform: mean file, crop, mirror), optionally initialised from a
``.caffemodel`` (ImageNetRunDBApp.scala:75), then runs the model-averaging loop: test
every ``--test-every`` rounds, ``--tau`` local solver steps, one all-reduce average
(CifarDBApp.scala:127-167).

    python -m sparknet_amd.apps.db_app create --dataset cifar --data cifar-10-batches-bin --out dbs
    python -m sparknet_amd.apps.db_app train --dataset cifar --db dbs --rounds 20
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m sparknet_amd.apps.db_app create --dataset imagenet --synthetic --out dbs
"""
from __future__ import annotations

import argparse
import os
import time

import numpy as np
import torch

from .. import models, proto
from ..core.solver import Solver
from ..data.db import create_db
from ..data.loaders import compute_mean, write_mean_binaryproto
from ..data.sampler import shard_range
from ..utils.logging import TrainingLog
from .common import setup

DATASETS = {
    # name: (model, image C/H/W stored in the DB, crop, mirror, train batch, test batch, tau, classes)
    "cifar": ("cifar10_full", (3, 32, 32), 0, False, 100, 100, 10, 10),
    "imagenet": ("caffenet", (3, 256, 256), 227, True, 256, 50, 50, 1000),
}


def _db_paths(root: str, rank: int) -> tuple[str, str]:
    return os.path.join(root, f"train_db.rank{rank}"), os.path.join(root, f"test_db.rank{rank}")


def _load(args, rank: int, world: int):
    C, H, W = DATASETS[args.dataset][1]
    if args.synthetic or not args.data:
        g = np.random.default_rng(args.seed + 7 * rank)
        n_tr, n_te = args.synthetic_train, args.synthetic_test
        classes = DATASETS[args.dataset][7]
        return ((g.integers(0, 256, (n_tr, C, H, W), dtype=np.uint8), g.integers(0, classes, n_tr)),
                (g.integers(0, 256, (n_te, C, H, W), dtype=np.uint8), g.integers(0, classes, n_te)))
    if args.dataset == "cifar":
        from ..data.loaders import CifarLoader
        ld = CifarLoader(args.data, seed=args.seed)
        out = []
        for im, lab in ((ld.train_images, ld.train_labels), (ld.test_images, ld.test_labels)):
            a, b = shard_range(len(lab), rank, world)
            out.append((im[a:b], lab[a:b]))
        return tuple(out)
    from ..data.loaders import ImageNetLoader
    out = []
    for root, labels in ((args.data, args.labels), (args.val_data or args.data, args.val_labels or args.labels)):
        xs, ys = [], []
        for x, y in ImageNetLoader(root, labels).minibatches(1, (rank, world)):
            xs.append(x.numpy())
            ys.append(y.numpy())
        out.append((np.concatenate(xs), np.concatenate(ys)))
    return tuple(out)


def create(args) -> dict:
    rank, world, dev, comm = setup(args)
    log = TrainingLog(args.log_dir, rank, name="db_create_log")
    (tr_x, tr_y), (te_x, te_y) = _load(args, rank, world)
    os.makedirs(args.out, exist_ok=True)
    train_db, test_db = _db_paths(args.out, rank)
    t0 = time.perf_counter()
    log.log(f"write train data to DB ({len(tr_y)} images, {args.backend})")
    n_train = create_db(train_db, tr_x, tr_y, backend=args.backend, decimal_keys=args.decimal_keys)
    log.log(f"write test data to DB ({len(te_y)} images)")
    n_test = create_db(test_db, te_x, te_y, backend=args.backend, decimal_keys=args.decimal_keys)
    log.log("computing mean image")
    mean = compute_mean((tr_x[i:i + 256] for i in range(0, len(tr_x), 256)), comm)
    test_batch = DATASETS[args.dataset][5]
    counts = comm.allgather_int(n_test // test_batch) if comm is not None else [n_test // test_batch]
    if rank == 0:
        write_mean_binaryproto(mean, os.path.join(args.out, "mean.binaryproto"))
        with open(os.path.join(args.out, "num_test_batches.txt"), "w") as f:
            f.write("\n".join(str(c) for c in counts) + "\n")
    if comm is not None:
        comm.barrier()
    log.log(f"finished creating databases in {time.perf_counter() - t0:.1f}s")
    log.close()
    if comm is not None:
        comm.close()
    return {"train": train_db, "test": test_db, "n_train": n_train, "n_test": n_test}


def _data_layer(phase: int, source: str, batch: int, backend: str, mean_file: str, crop: int, mirror: bool):
    lp = proto.LayerParameter(name="data", type="Data", top=["data", "label"])
    lp.include.add().phase = phase
    lp.data_param.source = source
    lp.data_param.batch_size = batch
    lp.data_param.backend = 1 if backend == "lmdb" else 0
    lp.transform_param.mean_file = mean_file
    if crop:
        lp.transform_param.crop_size = crop
    lp.transform_param.mirror = bool(mirror and phase == proto.TRAIN)
    return lp


def db_solver(dataset: str, db_root: str, rank: int, backend: str, batch: int | None = None,
              test_batch: int | None = None):
    """Zoo solver whose JavaData inputs are replaced by Data layers over this rank's DBs."""
    model, chw, crop, mirror, b, tb, _, _ = DATASETS[dataset]
    batch, test_batch = batch or b, test_batch or tb
    kw = {"crop": crop} if crop else {}
    sp = models.solver_for(model, train_batch=batch, test_batch=test_batch, **kw)
    net = sp.net_param
    train_db, test_db = _db_paths(db_root, rank)
    mean_file = os.path.join(db_root, "mean.binaryproto")
    keep = [lp for lp in net.layer if lp.type not in ("JavaData", "RDD")]
    del net.layer[:]
    net.layer.add().CopyFrom(_data_layer(proto.TRAIN, train_db, batch, backend, mean_file, crop, mirror))
    net.layer.add().CopyFrom(_data_layer(proto.TEST, test_db, test_batch, backend, mean_file, crop, False))
    for lp in keep:
        net.layer.add().CopyFrom(lp)
    return sp


def train(args):
    rank, world, dev, comm = setup(args)
    log = TrainingLog(args.log_dir, rank, name="db_train_log")
    sp = db_solver(args.dataset, args.db, rank, args.backend, args.batch, args.test_batch)
    solver = Solver(sp, device=dev, seed=args.seed + rank)
    if args.weights:
        solver.net.copy_trained_layers_from(args.weights)
    counts_file = os.path.join(args.db, "num_test_batches.txt")
    with open(counts_file) as f:
        counts = [int(x) for x in f.read().split()]
    n_test = max(1, min(counts[rank] if rank < len(counts) else counts[-1], args.max_test_batches))
    if comm is not None:
        comm.broadcast_params(solver.net)
    tau = args.tau or DATASETS[args.dataset][6]
    log.log(f"{args.dataset}: {world} worker(s) on {args.backend} databases, tau {tau}, {n_test} test batches")
    history = []
    for r in range(args.rounds):
        if args.test_every and r % args.test_every == 0:
            scores = solver.test(0, n_test)
            names = [b.name for b in solver.test_nets[0].output_blobs]
            total = n_test
            if comm is not None:
                scores = comm.allreduce_scores(scores + [float(n_test)])
                total = int(scores.pop())
            acc = {n: 100.0 * v / total for n, v in zip(names, scores)}
            for n, v in acc.items():
                if "accuracy" in n:
                    log.log(f"{v:.2f}% accuracy", i=r)
            history.append((r, acc))
        log.log("training", i=r)
        solver.step(tau)
        if comm is not None:
            log.log("collecting weights", i=r)
            comm.average_params(solver.net)
    log.close()
    if comm is not None:
        comm.close()
    return solver, history


def main(argv=None):
    p = argparse.ArgumentParser(description="SparkNet DB apps (CifarDBApp / ImageNet{Create,Run}DBApp)")
    p.add_argument("command", choices=["create", "train"])
    p.add_argument("--dataset", choices=sorted(DATASETS), default="cifar")
    p.add_argument("--data", default=None)
    p.add_argument("--labels", default=None)
    p.add_argument("--val-data", default=None)
    p.add_argument("--val-labels", default=None)
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--synthetic-train", type=int, default=1000)
    p.add_argument("--synthetic-test", type=int, default=200)
    p.add_argument("--out", default="sparknet_dbs", help="create: output directory")
    p.add_argument("--db", default="sparknet_dbs", help="train: directory written by create")
    p.add_argument("--backend", choices=["leveldb", "lmdb", "sndb"], default="leveldb")
    p.add_argument("--decimal-keys", action="store_true", help="SparkNet's counter.toString keys")
    p.add_argument("--rounds", type=int, default=100)
    p.add_argument("--tau", type=int, default=0, help="local steps per round (0 = dataset default)")
    p.add_argument("--test-every", type=int, default=10)
    p.add_argument("--max-test-batches", type=int, default=1 << 30)
    p.add_argument("--batch", type=int, default=None)
    p.add_argument("--test-batch", type=int, default=None)
    p.add_argument("--weights", default=None, help=".caffemodel(.h5) to start from (ImageNetRunDBApp)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--log-dir", default=None)
    args = p.parse_args(argv)
    return create(args) if args.command == "create" else train(args)


if __name__ == "__main__":
    main()
