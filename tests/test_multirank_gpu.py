"""The N-rank production path on a real GPU inside a 1-GPU lease.

The driver's scaling run (bench.py at N = 2/4/8, one rank per GPU over RCCL) must not be
the first time this code holds device tensors in a multi-rank group.  On a 1-GPU box two
ranks share device 0 (SN_SHARE_GPU / ``--share-gpu``) and the collectives go over gloo —
RCCL refuses two ranks on one device — while everything else is the production path:
spawn_local before any GPU call, per-rank hipGraph capture, the grouped H2D feeder,
bucketed ``average_params`` + ``scale_shadow``, ``comm_bench`` on device tensors, the
watchdog thread and the per-rank JSON.  Reference algorithm: τ local steps then
collect-and-average (src/main/scala/apps/ImageNetApp.scala:151,185-186;
CifarApp.scala:133-134)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "SN_SHARE_GPU"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "4"
    return env


@pytest.mark.timeout(300)
def test_bench_two_ranks_share_gpu(gpu):
    r = subprocess.run([sys.executable, "-u", "bench.py", "--gpus", "2", "--share-gpu", "--verify-average",
                        "--steps", "6", "--warmup", "3", "--tau", "3"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == out["rccl_world"] == 2 and out["share_gpu"] and out["comm_backend"] == "gloo"
    assert out["config"]["hipgraph"] and out["config"]["feed_group"] >= 1
    assert out["averages_in_window"] == 2 and out["allreduce_ms_per_average"] is not None
    assert out["average_buckets"] == 4  # 244 MB in 64 MB buckets
    chk = out["avg_check"]
    assert chk["masters_equal_across_ranks"] and chk["shadow_is_bf16_master"] and chk["ranks"] == 2
    assert set(out["comm_bench"]) == {"bucket_256MB", "bucket_64MB", "bucket_16MB"}
    assert len(out["per_rank_ms_per_step"]) == 2 and out["config"]["final_loss"] == out["config"]["final_loss"]


@pytest.mark.timeout(300)
def test_cifar_app_two_ranks_share_gpu(gpu, tmp_path):
    """apps/runner.py on 2 ranks: per-round test score all-reduce on device tensors, graph
    local steps, averaging, rank-0 checkpoint + per-rank solverstate."""
    env = _env()
    env["SN_SHARE_GPU"] = "1"
    prefix = str(tmp_path / "ck" / "cifar")
    r = subprocess.run([sys.executable, "-u", "-m", "sparknet_amd.apps.cifar_app", "--nproc", "2", "--synthetic",
                        "--rounds", "2", "--tau", "3", "--test-every", "1", "--snapshot-every", "2",
                        "--snapshot-prefix", prefix, "--log-dir", str(tmp_path / "logs")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    assert os.path.exists(prefix + ".caffemodel")
    assert os.path.exists(prefix + ".rank0.solverstate") and os.path.exists(prefix + ".rank1.solverstate")


@pytest.mark.timeout(420)
def test_bench_eight_ranks_share_gpu(gpu):
    """The driver's N = 8 scaling run rehearsed on one GPU: 8 ranks started by spawn_local,
    8 graph captures on one device, gloo collectives on device tensors, bitwise-equal
    averaged masters on all 8 ranks, and the self-diagnosis block of the N > 1 JSON."""
    env = _env()
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, "-u", "bench.py", "--gpus", "8", "--share-gpu", "--verify-average",
                        "--steps", "4", "--warmup", "2", "--tau", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == out["rccl_world"] == 8 and out["share_gpu"]
    assert out["averages_in_window"] == 2 and len(out["per_rank_ms_per_step"]) == 8
    chk = out["avg_check"]
    assert chk["masters_equal_across_ranks"] and chk["shadow_is_bf16_master"] and chk["ranks"] == 8
    d = out["diag"]
    assert len(d["bucket_allreduce_ms"]) == 4 and len(d["numa_node_per_rank"]) == 8


def _sync_worker(rank, world, port, q, steps, batch, seed):
    import torch
    import torch.distributed as dist
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      SN_GEMM_AUTOTUNE="0")
    try:
        torch.cuda.set_device(0)
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from sparknet_amd.parallel import Comm, SyncSGDCallback
        s = _sync_solver(seed, batch)
        comm = Comm() if world > 1 else None
        if comm is not None:
            s.add_callback(SyncSGDCallback(comm, s.net, overlap=True, bucket_bytes=4096))
        for step in range(steps):
            x, y = _sync_batch(step, world * batch)
            lo = rank * batch
            s.net.layer_by_name("data").feed(x[lo:lo + batch])
            s.net.layer_by_name("label").feed(y[lo:lo + batch])
            s.step(1)
        torch.cuda.synchronize()
        # numpy, pickled by value: a torch tensor would travel as a shared-memory fd that the
        # parent cannot open once this process has exited
        q.put((rank, s.net.flat_data.detach().float().cpu().numpy().copy(), None))
        if comm is not None:
            comm.close()
    except BaseException as e:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _sync_solver(seed, batch):
    import torch
    from sparknet_amd import proto
    from sparknet_amd.core.solver import Solver
    net = proto.parse_prototxt("""
      name: "sync"
      layer { name: "data" type: "JavaData" top: "data" java_data_param { shape { dim: BATCH dim: 8 dim: 8 dim: 8 } } }
      layer { name: "label" type: "JavaData" top: "label" java_data_param { shape { dim: BATCH dim: 1 } } }
      layer { name: "conv" type: "Convolution" bottom: "data" top: "conv"
        convolution_param { num_output: 16 kernel_size: 3 weight_filler { type: "gaussian" std: 0.2 } } }
      layer { name: "relu0" type: "ReLU" bottom: "conv" top: "conv" }
      layer { name: "ip1" type: "InnerProduct" bottom: "conv" top: "ip1"
        inner_product_param { num_output: 32 weight_filler { type: "gaussian" std: 0.05 } } }
      layer { name: "relu" type: "ReLU" bottom: "ip1" top: "ip1" }
      layer { name: "ip2" type: "InnerProduct" bottom: "ip1" top: "ip2"
        inner_product_param { num_output: 8 weight_filler { type: "gaussian" std: 0.1 } } }
      layer { name: "loss" type: "SoftmaxWithLoss" bottom: "ip2" bottom: "label" top: "loss" }
    """.replace("BATCH", str(batch)))
    sp = proto.SolverParameter(base_lr=0.01, lr_policy="fixed", momentum=0.9, weight_decay=0.001)
    sp.net_param.CopyFrom(net)
    return Solver(sp, device=torch.device("cuda", 0), seed=seed, build_test_nets=False)


def _sync_batch(step, n):
    import torch
    g = torch.Generator().manual_seed(500 + step)
    return torch.randn(n, 8, 8, 8, generator=g), torch.randint(0, 8, (n, 1), generator=g).float()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_sync_sgd_share_gpu_matches_single_rank_large_batch(gpu, world):
    """Caffe P2PSync semantics (test_gradient_based_solver.cpp:455-490) on GPU-resident
    ranks: N ranks x batch B with the bucketed, backward-overlapped gradient all-reduce
    (SyncSGDCallback) == 1 rank x batch N*B, and the N ranks hold bitwise-equal masters."""
    import multiprocessing as mp
    import socket
    import torch
    batch, steps = 4, 4
    ctx = mp.get_context("spawn")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]

    def launch(n, b):
        q = ctx.Queue()
        procs = [ctx.Process(target=_sync_worker, args=(r, n, port + (0 if n > 1 else 1), q, steps, b, 7))
                 for r in range(n)]
        for p in procs:
            p.start()
        res = [q.get(timeout=240) for _ in range(n)]
        for p in procs:
            p.join(timeout=60)
        for _, _, err in res:
            assert err is None, err
        return [torch.from_numpy(w) for _, w, _ in sorted(res, key=lambda t: t[0])]

    multi = launch(world, batch)
    single = launch(1, world * batch)[0]
    for w in multi[1:]:
        assert torch.equal(w, multi[0]), "ranks must hold bitwise-identical masters"
    err = (multi[0] - single).abs().max().item()
    assert err < 1e-5, err
