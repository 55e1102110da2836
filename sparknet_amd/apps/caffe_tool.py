"""``caffe``-tool equivalent (caffe/tools/caffe.cpp:28-376): train / test / time /
device_query, driven by prototxt solver / net files.

    python -m sparknet_amd.apps.caffe_tool train --solver solver.prototxt [--weights w.caffemodel]
                                                 [--snapshot s.solverstate] [--iterations N]
    python -m sparknet_amd.apps.caffe_tool test --model net.prototxt --weights w.caffemodel --iterations 50
    python -m sparknet_amd.apps.caffe_tool time --model net.prototxt --iterations 20 [--phase TRAIN]
    python -m sparknet_amd.apps.caffe_tool time --zoo caffenet --batch 256
    python -m sparknet_amd.apps.caffe_tool device_query

``time`` reports per-layer forward/backward milliseconds measured with HIP events
(reference: Timer on cudaEvents, caffe/src/caffe/util/benchmark.cpp), in the reference
output shape ("<layer>\\tforward: <ms> ms." / "backward: ...", "Average Forward pass").
Nets whose inputs are file-backed Data layers should be run with --zoo (JavaData inputs,
synthetic batches).
"""
from __future__ import annotations

import argparse
import sys
import time

import torch

from .. import models, proto
from ..core.net import Net
from ..core.solver import Solver
from ..engine import fuse_relu


def _device(args):
    if args.cpu or not torch.cuda.is_available():
        return torch.device("cpu")
    torch.cuda.set_device(args.gpu)
    from ..ops import _lib
    _lib.kernels()
    return torch.device("cuda", args.gpu)


def _fill_inputs(net: Net, seed=0):
    g = torch.Generator().manual_seed(seed)
    for layer in net.layers:
        if layer.type_name in ("JavaData", "Input", "MemoryData"):
            for t in getattr(layer, "_tops", []):
                if len(t.shape) == 4:
                    t.set_nchw(torch.randn(t.shape, generator=g) * 50)
                else:
                    t.data.copy_(torch.randint(0, 10, tuple(t.data.shape), generator=g).float())


class _Timer:
    def __init__(self, dev):
        self.dev = dev
        self.cuda = dev.type == "cuda"

    def __enter__(self):
        if self.cuda:
            self.a = torch.cuda.Event(enable_timing=True)
            self.b = torch.cuda.Event(enable_timing=True)
            self.a.record()
        else:
            self.t = time.perf_counter()
        return self

    def __exit__(self, *e):
        if self.cuda:
            self.b.record()

    def ms(self) -> float:
        if self.cuda:
            self.b.synchronize()
            return self.a.elapsed_time(self.b)
        return (time.perf_counter() - self.t) * 1000


def cmd_time(args):
    dev = _device(args)
    if args.zoo:
        netp = models.build(args.zoo, train_batch=args.batch, test_batch=args.batch)
    else:
        netp = proto.read_net(args.model)
    phase = proto.TRAIN if args.phase.upper() == "TRAIN" else proto.TEST
    net = Net(netp, phase=phase, device=dev)
    if dev.type == "cuda":
        fuse_relu(net)
    _fill_inputs(net)
    L = len(net.layers)
    fwd = [0.0] * L
    bwd = [0.0] * L
    net.forward()
    net.backward()
    t_all = _Timer(dev)
    with t_all:
        for _ in range(args.iterations):
            for li in range(L):
                with _Timer(dev) as t:
                    net.layers[li].forward(net.bottom_vecs[li], net.top_vecs[li])
                fwd[li] += t.ms()
            net.prefill_loss_diffs()
            for li in range(L - 1, -1, -1):
                if net.layer_need_backward[li]:
                    with _Timer(dev) as t:
                        net.layers[li].backward(net.top_vecs[li], net.bottom_need_backward[li], net.bottom_vecs[li])
                    bwd[li] += t.ms()
    total = t_all.ms()
    n = args.iterations
    print(f"Average time per layer ({dev}):")
    for li, name in enumerate(net.layer_names):
        print(f"{name:>24}\tforward: {fwd[li] / n:.4f} ms.")
        print(f"{name:>24}\tbackward: {bwd[li] / n:.4f} ms.")
    print(f"Average Forward pass: {sum(fwd) / n:.4f} ms.")
    print(f"Average Backward pass: {sum(bwd) / n:.4f} ms.")
    print(f"Average Forward-Backward: {total / n:.4f} ms.")
    print(f"Total Time: {total:.4f} ms.")
    return fwd, bwd


def cmd_train(args):
    dev = _device(args)
    sp = proto.read_solver(args.solver)
    solver = Solver(sp, device=dev)
    if dev.type == "cuda":
        fuse_relu(solver.net)
    if args.snapshot:
        solver.restore(args.snapshot)
    elif args.weights:
        for w in args.weights.split(","):
            solver.net.copy_trained_layers_from(w)
    if args.iterations:
        solver.step(args.iterations)
    else:
        solver.solve()
    print(f"Optimization done at iter {solver.iter}")


def cmd_test(args):
    dev = _device(args)
    net = Net(proto.read_net(args.model), phase=proto.TEST, device=dev)
    if args.weights:
        net.copy_trained_layers_from(args.weights)
    sums = None
    for i in range(args.iterations):
        net.forward()
        v = [float(b.data.float().mean()) for b in net.output_blobs]
        sums = v if sums is None else [a + b for a, b in zip(sums, v)]
    for b, s in zip(net.output_blobs, sums or []):
        print(f"{b.name} = {s / args.iterations:g}")


def cmd_device_query(args):
    if not torch.cuda.is_available():
        print("no ROCm device")
        return
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        print(f"Device id: {i}\n  Name: {p.name}\n  Total global memory: {p.total_memory}\n"
              f"  Compute units: {p.multi_processor_count}\n  Arch: {getattr(p, 'gcnArchName', '?')}")


def main(argv=None):
    p = argparse.ArgumentParser(prog="caffe")
    p.add_argument("command", choices=["train", "test", "time", "device_query"])
    p.add_argument("--solver")
    p.add_argument("--model")
    p.add_argument("--zoo")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--weights")
    p.add_argument("--snapshot")
    p.add_argument("--iterations", type=int, default=50)
    p.add_argument("--phase", default="TRAIN")
    p.add_argument("--gpu", type=int, default=0)
    p.add_argument("--cpu", action="store_true")
    args = p.parse_args(argv)
    return {"train": cmd_train, "test": cmd_test, "time": cmd_time, "device_query": cmd_device_query}[
        args.command](args)


if __name__ == "__main__":
    sys.exit(main() and 0)
