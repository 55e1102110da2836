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
