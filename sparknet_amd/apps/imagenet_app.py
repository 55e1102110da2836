"""ImageNetApp — CaffeNet model averaging (src/main/scala/apps/ImageNetApp.scala:19-192).

Reference constants: batch 256 train / 50 test, images resized to 256x256, random 227
crops (+ mirror) with mean subtraction, tau = 50.  Deliberate divergences:
the crop offset is drawn from 0..29 (Caffe's range, the reference used nextInt(29)) and
mean subtraction is actually applied (the reference's loop was a no-op).

    python -m sparknet_amd.apps.imagenet_app --synthetic --rounds 5
    python -m sparknet_amd.apps.imagenet_app --data /imagenet/train_tars --labels train.txt
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

from ..data.loaders import ImageNetLoader
from . import runner
from .common import base_parser, maybe_launch


def main(argv=None):
    p = base_parser("SparkNet ImageNetApp on MI355X", model="caffenet", tau=50, rounds=100, test_every=10,
                    batch=256, test_batch=50)
    p.add_argument("--labels", default=None)
    p.add_argument("--val-data", default=None)
    p.add_argument("--val-labels", default=None)
    p.add_argument("--max-images", type=int, default=0)
    args = p.parse_args(argv)
    rc = maybe_launch(args, "sparknet_amd.apps.imagenet_app", argv)
    if rc is not None:
        return rc
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    train = test = None
    mean = [104.0, 117.0, 123.0]
    if args.data and not args.synthetic:
        def load(root, labels, batch):
            xs, ys = [], []
            for x, y in ImageNetLoader(root, labels).minibatches(batch, (rank, world)):
                xs.append(x)
                ys.append(y)
                if args.max_images and len(xs) * batch >= args.max_images:
                    break
            return torch.cat(xs), torch.cat(ys)
        train = load(args.data, args.labels, args.batch)
        mean = train[0].float().mean(dim=(0,)).numpy().astype(np.float32)
        if args.val_data:
            test = load(args.val_data, args.val_labels, args.test_batch)
    crop = 227 if args.model in ("caffenet", "alexnet") else 224
    return runner.run(args, model=args.model, data_shape=(3, 256, 256), crop=crop, mean=mean, scale=1.0,
                      mirror=True, classes=1000, train_data=train, test_data=test,
                      model_kw={"crop": crop}, log_name="imagenet_log")


if __name__ == "__main__":
    _r = main()
    sys.exit(_r if isinstance(_r, int) else 0)
