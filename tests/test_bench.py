"""bench.py contract on the CPU: `--gpus N` outside a launcher starts N ranks through
parallel.launch.spawn_local (the path the 8-GPU run takes with `python bench.py --gpus 8`),
every rank joins one process group, and rank 0 prints ONE JSON line for the whole job."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--cpu", "--model", "cifar10_quick", "--batch", "4", "--steps", "3", "--warmup", "1", "--tau", "2"]


def _clean_env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_bench_spawns_n_ranks_and_reports_job_json():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=ROOT, env=_clean_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rccl_world"] == 2
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 8
    assert len(out["per_rank_ms_per_step"]) == 2
    assert out["steps"] == 3 and out["averages_in_window"] >= 1
    assert out["ms_per_step"] >= max(out["per_rank_ms_per_step"]) - 1e-3  # slowest rank's clock
    assert set(out["comm_bench"]) == {"bucket_256MB", "bucket_64MB", "bucket_16MB"}
    d = out["diag"]  # self-diagnosis block of every N > 1 run (parallel/diag.py)
    assert len(d["bucket_allreduce_ms"]) >= 1 and all(v >= 0 for v in d["bucket_allreduce_ms"])
    assert len(d["numa_node_per_rank"]) == 2 and d["step_spread_pct"] >= 0


def test_bench_refuses_world_mismatch():
    env = _clean_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "--gpus 2" in r.stderr


def test_bench_verify_average_cpu():
    """--verify-average on the gloo CPU path: post-average masters bitwise equal on both ranks."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--verify-average", *ARGS], cwd=ROOT,
                       env=_clean_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["avg_check"]["masters_equal_across_ranks"] and out["avg_check"]["shadow_is_bf16_master"]
    assert out["comm_backend"] == "gloo" and out["average_buckets"] >= 1


def test_bench_under_torchrun_like_the_driver():
    """The driver's multi-GPU form: `python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...` (ranks
    from the launcher's env, no self-spawn), here on the gloo CPU path."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", *ARGS],
                       cwd=ROOT, env=_clean_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the job line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rccl_world"] == 2 and out["config"]["parallelism"] == "dp2"


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_bench_forced_comm_at_world_one():
    """SN_COMM_FORCE=1 under a one-process torch.distributed.run: the process group, the
    initial broadcast, every averaging all-reduce and the post-window diagnostics run at world
    1 (on a GPU box this is the RCCL rehearsal of the scaling path, scripts/gpu_r5ap.sh)."""
    env = _clean_env()
    env["SN_COMM_FORCE"] = "1"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
                        "--verify-average", *ARGS], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["rccl_world"] == 1 and out["comm_backend"] == "gloo"
    assert out["averages_in_window"] >= 1 and out["average_buckets"] >= 1
    assert out["avg_check"]["masters_equal_across_ranks"] and out["avg_check"]["shadow_is_bf16_master"]
    assert set(out["comm_bench"]) == {"bucket_256MB", "bucket_64MB", "bucket_16MB"}


def test_comm_inactive_at_world_one_without_force():
    from sparknet_amd.parallel.comm import Comm
    c = Comm()
    assert c.world_size == 1 and not c.active


def test_gemm_autotune_off_by_default_and_rank_sync_cpu():
    """Kernel selection is fixed by the committed database + cost model unless asked for
    (VERDICT r5 #6): a fresh process imports gemm with first-call tuning OFF, bench.py does
    not turn it on without --autotune, and sync_tuned adopts rank 0's choices over gloo."""
    code = r'''
import os, sys
os.environ.pop("SN_GEMM_AUTOTUNE", None)
sys.path.insert(0, ".")
from sparknet_amd.ops import gemm as G
assert G._AUTOTUNE is False
import bench
sys.argv = ["bench.py"]
assert bench.parse().autotune is False
'''
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=_clean_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


def _sync_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from sparknet_amd.ops import gemm as G
    from sparknet_amd.parallel import Comm
    import torch
    comm = Comm(backend="gloo")
    key = (1, 2, 3, 1, 0, 0, 0, 0, 0, False, False, False, (8,), (8,), torch.bfloat16)
    G._TUNED[key] = (rank, 1, 64)  # every rank "tuned" a different tile
    n = G.sync_tuned(comm)
    q.put((rank, G._TUNED[key], n))
    dist.destroy_process_group()


def test_sync_tuned_adopts_rank0_choices_gloo():
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sync_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert [r[1] for r in res] == [(0, 1, 64), (0, 1, 64)], res
    assert all(r[2] >= 1 for r in res)
