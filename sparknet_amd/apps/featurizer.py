"""FeaturizerApp — forward-only feature extraction (src/main/scala/apps/FeaturizerApp.scala:
88-103): run the TEST-phase net over every minibatch and collect one blob (default
``ip1``) per image.  Each rank featurizes its shard; rank-local ``.npy`` files.

    python -m sparknet_amd.apps.featurizer --data cifar-10-batches-bin --weights m.caffemodel \
        --blob ip1 --out features
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import models, proto
from ..core.net import Net
from ..data.loaders import CifarLoader
from ..data.prefetch import DeviceFeeder, SyntheticSource
from ..data.sampler import shard_range
from ..engine import fuse_relu
from .common import base_parser, setup
from .runner import ListSource


def featurize(net: Net, feeder, n_batches: int, blob: str) -> np.ndarray:
    out = []
    with torch.no_grad():
        for _ in range(n_batches):
            feeder.stage()
            feeder.prefetch()
            net.forward()
            out.append(net.blob_by_name(blob).nchw().float().cpu().numpy().copy())
    return np.concatenate(out) if out else np.zeros((0,))


def main(argv=None):
    p = base_parser("SparkNet FeaturizerApp", model="cifar10_full", batch=100, test_batch=100)
    p.add_argument("--blob", default="ip1")
    p.add_argument("--out", default="features")
    p.add_argument("--max-batches", type=int, default=0)
    args = p.parse_args(argv)
    rank, world, dev, comm = setup(args)
    netp = models.build(args.model, train_batch=args.batch, test_batch=args.test_batch)
    net = Net(netp, phase=proto.TEST, device=dev)
    if dev.type == "cuda":
        fuse_relu(net)
    if args.weights:
        net.copy_trained_layers_from(args.weights)
    if args.data and not args.synthetic:
        ld = CifarLoader(args.data, shuffle=False)
        x, y = ld.tensors(train=False)
        a, b = shard_range(x.shape[0], rank, world)
        src = ListSource(x[a:b], y[a:b], args.test_batch)
        n = src.n
        mean = ld.mean_image()
    else:
        src = SyntheticSource(args.test_batch, 3, 32, 32, classes=10, pool=2, seed=rank)
        n = 2
        mean = [125.3, 123.0, 113.9]
    if args.max_batches:
        n = min(n, args.max_batches)
    feeder = DeviceFeeder(src, net.blob_by_name("data"), net.blob_by_name("label"), crop=32, mean=mean,
                          train=False, device=dev)
    feats = featurize(net, feeder, n, args.blob)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    path = f"{args.out}.rank{rank}.npy"
    np.save(path, feats)
    if rank == 0:
        print(f"wrote {path}: {feats.shape}")
    if comm is not None:
        comm.close()
    return feats


if __name__ == "__main__":
    main()
