"""CifarApp — CIFAR-10 model averaging (src/main/scala/apps/CifarApp.scala:14-140).

Reference constants: batch 100 train / 100 test, tau = 10, test every 10 rounds, model
cifar10_full with JavaData inputs, mean-subtracted planar float input.

    python -m sparknet_amd.apps.cifar_app --data /path/to/cifar-10-batches-bin --rounds 50
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m sparknet_amd.apps.cifar_app --synthetic --rounds 20
"""
from __future__ import annotations

import os
import sys

from ..data.loaders import CifarLoader
from ..data.sampler import shard_range
from . import runner
from .common import base_parser, bind_device, maybe_launch


def main(argv=None):
    p = base_parser("SparkNet CifarApp on MI355X", model="cifar10_full", tau=10, rounds=100, test_every=10,
                    batch=100, test_batch=100)
    args = p.parse_args(argv)
    rc = maybe_launch(args, "sparknet_amd.apps.cifar_app", argv)
    if rc is not None:
        return rc
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    train = test = None
    mean = [125.3, 123.0, 113.9]
    if args.data and not args.synthetic:
        bind_device(args)  # pinned rings below allocate on the current device
        ld = CifarLoader(args.data, seed=args.seed)
        mean = ld.mean_image()  # full mean image (the reference computed it, then ignored it)
        files = [os.path.join(args.data, f"data_batch_{i}.bin") for i in range(1, 6)]
        files = [f for f in files if os.path.exists(f)]
        if args.native_loader and files:
            # native pipeline: mmap'd records, SparkNet window sampler, worker threads,
            # pinned ring (csrc/runtime/loader.cpp); sharding is done by the loader
            from ..data.native import SAMPLER_WINDOW, NativeLoader
            first = 0
            if args.resume:  # continue the batch stream where the checkpointed run stopped
                from ..utils.checkpoint import read_round_sidecar
                first = read_round_sidecar(args.resume + ".json")["round"] * args.tau
            train = NativeLoader.cifar10(files, args.batch, sampler=SAMPLER_WINDOW, tau=args.tau, rank=rank,
                                         world=world, seed=args.seed * 101 + rank, threads=2, first_batch=first)
        else:
            ti, tl = ld.tensors(train=True)
            a, b = shard_range(ti.shape[0], rank, world)
            train = (ti[a:b], tl[a:b])
        vi, vl = ld.tensors(train=False)
        a, b = shard_range(vi.shape[0], rank, world)
        test = (vi[a:b], vl[a:b])
    return runner.run(args, model=args.model, data_shape=(3, 32, 32), crop=32, mean=mean, scale=1.0,
                      mirror=False, classes=10, train_data=train, test_data=test, log_name="cifar_log")


if __name__ == "__main__":
    _r = main()
    sys.exit(_r if isinstance(_r, int) else 0)
