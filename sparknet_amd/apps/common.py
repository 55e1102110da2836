"""Shared plumbing of the training entry points (one process per GPU).

Launch: ``python -m sparknet_amd.apps.<app> ...`` on one GPU, or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 -m
sparknet_amd.apps.<app> ...`` for N GPUs (replaces ``spark-submit --class apps.X jar N``,
README.md:26).  Ranks map 1:1 to GPUs.
"""
from __future__ import annotations

import argparse
import os
import signal

import torch


def base_parser(desc: str, **defaults) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=desc)
    p.add_argument("--data", default=None, help="dataset directory (omit for --synthetic)")
    p.add_argument("--synthetic", action="store_true", help="synthetic data of the dataset's shape")
    p.add_argument("--model", default=defaults.get("model"))
    p.add_argument("--tau", type=int, default=defaults.get("tau", 10), help="local SGD steps per round")
    p.add_argument("--rounds", type=int, default=defaults.get("rounds", 100))
    p.add_argument("--test-every", type=int, default=defaults.get("test_every", 10))
    p.add_argument("--batch", type=int, default=defaults.get("batch", 100))
    p.add_argument("--test-batch", type=int, default=defaults.get("test_batch", 100))
    p.add_argument("--weights", default=None, help=".caffemodel to initialise from")
    p.add_argument("--resume", default=None, help="checkpoint prefix to resume from")
    p.add_argument("--snapshot-every", type=int, default=0, help="checkpoint every k rounds (0 = off)")
    p.add_argument("--snapshot-prefix", default="sparknet")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--cpu", action="store_true", help="run the fp32 reference path on the CPU")
    p.add_argument("--sync-sgd", action="store_true", help="all-reduce gradients every step (tau=1 semantics)")
    p.add_argument("--sync-sgd-graph", action="store_true",
                   help="--sync-sgd inside the captured hipGraph (bucketed RCCL all-reduces as graph nodes); "
                        "verified bitwise on a 1-rank group only, so the eager step is the default")
    p.add_argument("--log-dir", default=None)
    p.add_argument("--fail-at-round", type=int, default=-1, help="fault injection: a rank exits at round r")
    p.add_argument("--fail-rank", type=int, default=0, help="fault injection: the rank that exits")
    p.add_argument("--nproc", type=int, default=1,
                   help="start this many ranks on this node (one per GPU) unless already launched "
                        "by torch.distributed.run")
    p.add_argument("--pg-timeout", type=float, default=300.0,
                   help="collective timeout in seconds (a dead peer is detected sooner by the watchdog)")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                   help="GPU compute: bf16, or fp8 (e4m3 forward products, bf16 backward, fp32 masters)")
    p.add_argument("--native-loader", action=argparse.BooleanOptionalAction, default=True,
                   help="file-backed datasets go through the C++ loader (csrc/runtime/loader.cpp)")
    return p


def share_gpu() -> bool:
    """SN_SHARE_GPU=1: rehearse an N-rank job on ONE GPU — every rank on device 0, collectives
    over gloo (RCCL refuses two ranks on one device).  For tests on 1-GPU boxes."""
    return os.environ.get("SN_SHARE_GPU", "0") == "1"


def bind_device(args) -> torch.device:
    """Make this rank's GPU (LOCAL_RANK) the current device.  Call it before anything that
    starts HIP — pinning host memory (``pin_memory``) opens a context on the CURRENT device,
    so a source built before the bind would put every rank's pinned ring (and a context)
    on GPU 0."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if share_gpu():
        local = 0
    if args.cpu or not torch.cuda.is_available():
        return torch.device("cpu")
    torch.cuda.set_device(local)
    return torch.device("cuda", local)


def setup(args):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = bind_device(args)
    if dev.type == "cuda":
        from ..ops import _lib
        _lib.kernels()
    from ..parallel import Comm
    # a CPU job (--cpu) runs gloo even where RCCL is available: nccl has no CPU tensors
    comm = (Comm(backend="gloo" if (share_gpu() or dev.type != "cuda") else None,
                 device=dev if dev.type == "cuda" else None,
                 timeout_s=getattr(args, "pg_timeout", 300.0), watchdog=True) if world > 1 else None)
    return rank, world, dev, comm


def maybe_launch(args, module: str, argv=None):
    """``--nproc N`` outside a launcher: start N ranks of ``python -m module argv`` on this
    node (parallel.launch.spawn_local, before any GPU call) and return the job's exit code;
    otherwise None (this process is a rank, or the job is single-process)."""
    from ..parallel.launch import launched_world, spawn_local
    if args.nproc <= 1 or launched_world() is not None:
        return None
    import sys
    rest = list(sys.argv[1:] if argv is None else argv)
    return spawn_local(args.nproc, ["-m", module] + rest)


class StopFlag:
    """SIGINT -> stop, SIGHUP -> snapshot at the next round boundary
    (caffe/src/caffe/util/signal_handler.cpp:14-115 semantics)."""

    def __init__(self):
        self.request = "none"
        try:
            signal.signal(signal.SIGINT, self._stop)
            signal.signal(signal.SIGHUP, self._snap)
        except ValueError:  # not in the main thread
            pass

    def _stop(self, *a):
        self.request = "stop"

    def _snap(self, *a):
        self.request = "snapshot"

    def take(self) -> str:
        r, self.request = self.request, "none"
        return r
