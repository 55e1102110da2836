"""GPU half of SparkNet's weight averaging (reference CifarApp.scala:133-134:
``workers.map(getWeights).reduce(add)`` then ``scalarDivide(N)``) inside one process.

A LocalSGDTrainer runs CaffeNet with the whole iteration captured in a hipGraph and a
fake 2-rank Comm whose all-reduce adds a known second weight vector.  After tau captured
steps and an average, the fp32 masters must be the exact mean, the bf16 compute shadow
must be bf16(master) (hip.scale_shadow), and the NEXT graph replay must read the averaged
weights — its forward (through the per-step S2D conv1 weight fold, the dgrad weight flips
and the fused-FC epilogues) equals an eager forward on the averaged weights."""
import pytest
import torch

from sparknet_amd import models

pytestmark = pytest.mark.gpu


class FakeComm:
    """world_size = 2; the 'other rank' holds ``other`` (fp32, same layout as flat_data)."""

    def __init__(self, other, bucket_bytes=64 << 20):
        from sparknet_amd.parallel.comm import Comm
        self.other = other
        self.world_size, self.rank = 2, 0
        self.active = True  # Comm.active: collectives run (world > 1)
        self.bucket_bytes = self.average_bucket_bytes = bucket_bytes
        self.bucket_ranges = Comm.bucket_ranges.__get__(self)
        self._avg = Comm.average_params.__get__(self)

    def allreduce_sum(self, flat, async_op=False):
        o = flat.storage_offset()  # flat is a bucket view of net.flat_data (offset 0)
        flat.add_(self.other[o:o + flat.numel()])

    def average_params(self, net):
        self._avg(net)

    def broadcast_params(self, net):
        pass


def _caffenet_solver(dev, batch=4, crop=99):
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.engine import fuse_relu
    n = models.caffenet(train_batch=batch, test_batch=batch, crop=crop, classes=10)
    for l in n.layer:
        if l.type == "Dropout":
            l.dropout_param.dropout_ratio = 0.0  # deterministic forward for the eager comparison
        if l.type == "InnerProduct" and l.name in ("fc6", "fc7"):
            l.inner_product_param.num_output = 256
    sp = models.zoo.caffenet_solver(n)
    sp.base_lr = 1e-3
    solver = Solver(sp, device=dev, seed=5, build_test_nets=False)
    fuse_relu(solver.net)
    g = torch.Generator().manual_seed(2)
    solver.net.blob_by_name("data").set_nchw(torch.randn(batch, 3, crop, crop, generator=g) * 30)
    solver.net.blob_by_name("label").set_nchw(torch.randint(0, 10, (batch, 1), generator=g).float())
    return solver


def test_graph_trainer_average_updates_masters_shadow_and_next_replay(gpu):
    from sparknet_amd.engine import LocalSGDTrainer
    solver = _caffenet_solver(gpu)
    net = solver.net
    g = torch.Generator(device="cpu").manual_seed(7)
    other = (net.flat_data.detach().cpu() * (1.0 + 0.5 * torch.randn(net.flat_data.numel(), generator=g))).to(gpu)
    comm = FakeComm(other, bucket_bytes=4 << 20)  # several buckets: per-bucket scale + shadow
    tr = LocalSGDTrainer(solver, comm, tau=3, use_graph=True)
    assert tr.step_fn is not None
    for _ in range(3):
        tr.local_step()  # the first call captures the graph (eager warmups + capture + replay)
    torch.cuda.synchronize()
    assert tr.step_fn.graph is not None

    fc8 = net.blob_by_name("fc8")
    net.forward()
    fc8_before = fc8.data.float().clone()
    before = net.flat_data.detach().clone()
    tr.average()
    torch.cuda.synchronize()
    expect = (before + other) * 0.5
    assert torch.equal(net.flat_data, expect), "masters must be the exact mean"
    if net.flat_compute is not net.flat_data:
        assert torch.equal(net.flat_compute, net.flat_data.to(net.flat_compute.dtype)), "shadow = bf16(master)"

    net.forward()  # eager forward on the averaged weights
    fc8_eager = fc8.data.float().clone()
    tr.local_step()  # graph replay: forward + backward + update
    torch.cuda.synchronize()
    fc8_graph = fc8.data.float()
    scale = fc8_eager.abs().max().item() + 1e-6
    assert (fc8_graph - fc8_eager).abs().max().item() <= 1e-3 * scale, "replay must read the averaged weights"
    assert (fc8_before - fc8_eager).abs().max().item() > 1e-2 * scale, "averaging must change the forward"
    assert torch.isfinite(net.flat_data).all()


def test_sync_sgd_bucketed_allreduce_captured_in_graph(gpu):
    """Sync-SGD mode keeps the hipGraph: the SyncSGDCallback's bucketed RCCL all-reduces
    (launched from backward hooks, overlapped with the remaining backward) are captured
    with the iteration.  On a 1-rank NCCL(RCCL) group the reduction is the identity, so
    4 captured steps end bitwise equal to 4 captured steps without the callback."""
    import socket

    import torch.distributed as dist

    from sparknet_amd.engine import GraphStep
    from sparknet_amd.parallel.comm import Comm, SyncSGDCallback, grad_buckets
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}",
                            device_id=torch.device(gpu))
    try:
        res = []
        for sync in (False, True):
            solver = _caffenet_solver(torch.device(gpu), batch=2, crop=67)
            if sync:
                cb = SyncSGDCallback(Comm(), solver.net)
                cb.plan, cb.late = grad_buckets(solver.net, 1 << 16)  # force the overlapped buckets
                solver.net.backward_hooks.append(cb._hook)
                solver.add_callback(cb)
                assert sum(len(v) for v in cb.plan.values()) >= 2
            g = torch.Generator().manual_seed(1)
            batches = iter([(torch.randn(2, 3, 67, 67, generator=g) * 20, torch.tensor([[1.0], [4.0]]))
                            for _ in range(6)])

            def pre():
                x, y = next(batches)
                solver.net.blob_by_name("data").set_nchw(x)
                solver.net.blob_by_name("label").set_nchw(y)
            step = GraphStep(solver, warmup=1, pre=pre, overlap=False, fuse_fc=False)
            for _ in range(4):
                step.step()
            torch.cuda.synchronize()
            assert step.graph is not None
            res.append(solver.net.flat_data.detach().clone())
        assert torch.equal(res[0], res[1])
    finally:
        dist.destroy_process_group()
