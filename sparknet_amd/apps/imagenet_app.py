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

from ..data.loaders import ImageNetLoader
from . import runner
from .common import base_parser, bind_device, maybe_launch


def main(argv=None):
    p = base_parser("SparkNet ImageNetApp on MI355X", model="caffenet", tau=50, rounds=100, test_every=10,
                    batch=256, test_batch=50)
    p.add_argument("--labels", default=None)
    p.add_argument("--val-data", default=None)
    p.add_argument("--val-labels", default=None)
    p.add_argument("--max-images", type=int, default=0, help="cap on this rank's training images per epoch")
    p.add_argument("--mean-images", type=int, default=0,
                   help="images of this rank's shard used for the mean (0: the whole shard, as the reference)")
    p.add_argument("--decode-workers", type=int, default=8, help="JPEG decode threads per rank")
    p.add_argument("--ring-slots", type=int, default=4, help="pinned minibatch buffers per rank")
    p.add_argument("--shuffle-buffer", type=int, default=2048, help="compressed records in the shuffle buffer")
    p.add_argument("--test-batches", type=int, default=10, help="validation minibatches per evaluation")
    args = p.parse_args(argv)
    rc = maybe_launch(args, "sparknet_amd.apps.imagenet_app", argv)
    if rc is not None:
        return rc
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    train = test = None
    mean = [104.0, 117.0, 123.0]
    if args.data and not args.synthetic:
        bind_device(args)  # the pinned rings below allocate on the current device
        # bounded-memory streaming ingest (data.stream): compressed records -> decode pool ->
        # ring of pinned minibatches; the mean is one streamed pass over the shard
        from ..data.stream import StreamingJpegSource, streamed_mean
        loader = ImageNetLoader(args.data, args.labels)

        def mean(comm):  # resolved by runner.run once the process group exists
            return streamed_mean(loader, args.batch, (rank, world), comm=comm,
                                 max_images=args.mean_images or args.max_images, workers=args.decode_workers)
        train = StreamingJpegSource(loader, args.batch, (rank, world), slots=args.ring_slots,
                                    workers=args.decode_workers, shuffle_buffer=args.shuffle_buffer,
                                    seed=args.seed, max_images=args.max_images)
        if args.val_data:
            test = StreamingJpegSource(ImageNetLoader(args.val_data, args.val_labels), args.test_batch,
                                       (rank, world), slots=2, workers=args.decode_workers)
    crop = 227 if args.model in ("caffenet", "alexnet") else 224
    try:
        return runner.run(args, model=args.model, data_shape=(3, 256, 256), crop=crop, mean=mean, scale=1.0,
                          mirror=True, classes=1000, train_data=train, test_data=test,
                          model_kw={"crop": crop}, log_name="imagenet_log")
    finally:
        for src in (train, test):
            if src is not None:
                src.close()


if __name__ == "__main__":
    _r = main()
    sys.exit(_r if isinstance(_r, int) else 0)
