"""Multi-process (gloo, CPU) tests of the distributed layer — the reference had no SN
distributed test; Caffe's only one is the N-device == 1-device x N-batch solver test
(caffe/src/caffe/test/test_gradient_based_solver.cpp:455-490), reproduced here."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sparknet_amd import proto


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _lsq_solver(seed, batch=4, sync=False):
    from sparknet_amd.core.solver import Solver
    net = proto.parse_prototxt(f"""
      name: "lsq"
      layer {{ name: "data" type: "JavaData" top: "data" java_data_param {{ shape {{ dim: {batch} dim: 3 }} }} }}
      layer {{ name: "targets" type: "JavaData" top: "targets" java_data_param {{ shape {{ dim: {batch} dim: 1 }} }} }}
      layer {{ name: "ip" type: "InnerProduct" bottom: "data" top: "ip"
        inner_product_param {{ num_output: 1 weight_filler {{ type: "gaussian" std: 1.0 }}
                               bias_filler {{ type: "gaussian" std: 1.0 }} }} }}
      layer {{ name: "loss" type: "EuclideanLoss" bottom: "ip" bottom: "targets" top: "loss" }}
    """)
    sp = proto.SolverParameter(base_lr=0.05, lr_policy="fixed", momentum=0.9, weight_decay=0.01)
    sp.net_param.CopyFrom(net)
    return Solver(sp, device="cpu", seed=seed)


def _data(step, lo, hi):
    g = torch.Generator().manual_seed(100 + step)
    X = torch.randn(8, 3, generator=g)
    Y = torch.randn(8, 1, generator=g)
    return X[lo:hi], Y[lo:hi]


def _worker_average(rank, world, port, q):
    _init(rank, world, port)
    from sparknet_amd.parallel import Comm
    from sparknet_amd.engine import LocalSGDTrainer
    comm = Comm()
    s = _lsq_solver(seed=rank)
    tr = LocalSGDTrainer(s, comm, tau=3, use_graph=False)
    tr.broadcast_initial()
    w0 = s.net.flat_data.clone()
    gathered = [torch.zeros_like(w0) for _ in range(world)]
    dist.all_gather(gathered, w0)
    same_start = all(torch.equal(g, w0) for g in gathered)
    layer_d, layer_t = s.net.layer_by_name("data"), s.net.layer_by_name("targets")
    for step in range(3):
        X, Y = _data(step * world + rank, 0, 4)
        layer_d.feed(X)
        layer_t.feed(Y)
        tr.local_step()
    before = s.net.flat_data.clone()
    allb = [torch.zeros_like(before) for _ in range(world)]
    dist.all_gather(allb, before)
    tr.average()
    after = s.net.flat_data.clone()
    manual = torch.stack(allb).mean(0)
    q.put((rank, same_start, bool(torch.allclose(after, manual, atol=1e-6)),
           bool(not torch.equal(allb[0], allb[1])), after.tolist()))
    comm.close()


def _worker_sync(rank, world, port, q):
    _init(rank, world, port)
    from sparknet_amd.parallel import Comm, SyncSGDCallback
    comm = Comm()
    s = _lsq_solver(seed=0, batch=4)
    s.add_callback(SyncSGDCallback(comm, s.net))
    lo, hi = rank * 4, rank * 4 + 4
    for step in range(4):
        X, Y = _data(step, lo, hi)
        s.net.layer_by_name("data").feed(X)
        s.net.layer_by_name("targets").feed(Y)
        s.step(1)
    q.put((rank, s.net.flat_data.tolist()))
    comm.close()


def _wrapped(fn, rank, world, port, q):
    """Run a worker, then leave the gloo group together: a rank that exits while its peer
    still has async collectives / the gloo transport open can abort the peer (SIGABRT)."""
    fn(rank, world, port, q)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wrapped, args=(fn, r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


def test_model_averaging_gloo():
    res = _run(_worker_average)
    for rank, same_start, avg_ok, diverged, _ in res:
        assert same_start, "ranks must start from rank 0's weights"
        assert diverged, "local steps on different data must diverge"
        assert avg_ok, "averaged weights must equal the manual mean"
    assert res[0][4] == res[1][4], "all ranks hold identical weights after averaging"


def test_sync_sgd_equals_single_large_batch():
    res = _run(_worker_sync)
    single = _lsq_solver(seed=0, batch=8)
    for step in range(4):
        X, Y = _data(step, 0, 8)
        single.net.layer_by_name("data").feed(X)
        single.net.layer_by_name("targets").feed(Y)
        single.step(1)
    for _, w in res:
        assert torch.allclose(torch.tensor(w), single.net.flat_data, atol=1e-5), (w[:8], single.net.flat_data[:8])


def _worker_misc(rank, world, port, q):
    _init(rank, world, port)
    from sparknet_amd.parallel import Comm
    comm = Comm()
    s = comm.allreduce_scores([1.0 + rank, 10.0])
    g = comm.allgather_int(rank * 5)
    m = comm.max_over_ranks(float(rank))
    q.put((rank, s, g, m))
    comm.close()


def test_collective_helpers():
    for rank, s, g, m in _run(_worker_misc):
        assert s == [3.0, 20.0] and g == [0, 5] and m == 1.0


def _multilayer_solver(seed):
    from sparknet_amd.core.solver import Solver
    net = proto.parse_prototxt("""
      name: "ml"
      layer { name: "data" type: "JavaData" top: "data" java_data_param { shape { dim: 4 dim: 3 dim: 6 dim: 6 } } }
      layer { name: "label" type: "JavaData" top: "label" java_data_param { shape { dim: 4 dim: 1 } } }
      layer { name: "conv" type: "Convolution" bottom: "data" top: "conv"
        param { lr_mult: 0 } param { lr_mult: 0 }
        convolution_param { num_output: 4 kernel_size: 3 weight_filler { type: "gaussian" std: 0.3 } } }
      layer { name: "ip1" type: "InnerProduct" bottom: "conv" top: "ip1"
        inner_product_param { num_output: 8 weight_filler { type: "gaussian" std: 0.3 } } }
      layer { name: "relu" type: "ReLU" bottom: "ip1" top: "ip1" }
      layer { name: "ip2" type: "InnerProduct" bottom: "ip1" top: "ip2"
        inner_product_param { num_output: 3 weight_filler { type: "gaussian" std: 0.3 } } }
      layer { name: "loss" type: "SoftmaxWithLoss" bottom: "ip2" bottom: "label" top: "loss" }
    """)
    sp = proto.SolverParameter(base_lr=0.1, lr_policy="fixed", momentum=0.9, weight_decay=0.001)
    sp.net_param.CopyFrom(net)
    return Solver(sp, device="cpu", seed=seed)


def _worker_bucketed(rank, world, port, q):
    _init(rank, world, port)
    from sparknet_amd.parallel import Comm, SyncSGDCallback
    from sparknet_amd.parallel.comm import grad_buckets
    comm = Comm()
    out = []
    for overlap in (False, True):
        s = _multilayer_solver(seed=0)
        cb = SyncSGDCallback(comm, s.net, overlap=overlap, bucket_bytes=64)
        s.add_callback(cb)
        for step in range(3):
            g = torch.Generator().manual_seed(1000 + 10 * step + rank)
            s.net.layer_by_name("data").feed(torch.randn(4, 3, 6, 6, generator=g))
            s.net.layer_by_name("label").feed(torch.randint(0, 3, (4, 1), generator=g).float())
            s.step(1)
        out.append(s.net.flat_data.tolist())
    plan, late = grad_buckets(s.net, 64)
    q.put((rank, out, sum(len(v) for v in plan.values()), len(late)))
    comm.close()


def test_bucketed_overlapped_grad_allreduce_matches_flat():
    res = _run(_worker_bucketed)
    for rank, (flat, bucketed), nb, nlate in res:
        assert nb >= 3 and nlate == 2, (nb, nlate)  # ip2 w/b, ip1 w/b buckets; frozen conv w/b late
        assert flat == bucketed
    assert res[0][1][1] == res[1][1][1]
