"""Training entry points end to end on the CPU (fp32 reference path): CifarApp over
CIFAR-format binary files through the native loader, round-boundary checkpoint + resume
(bitwise continuation) and the fault-injection switch.  Reference: CifarApp.scala:14-140
(no test in the reference; SURVEY §5.3-5.4 asks for resume / fault tests)."""
import os
import subprocess
import sys

import pytest
import torch

from sparknet_amd.apps import cifar_app
from sparknet_amd.data.loaders import write_synthetic_cifar

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def cifar_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("cifar_app")
    write_synthetic_cifar(str(d), n_train=200, n_test=40, seed=1)
    return str(d)


def _args(d, *extra):
    return ["--cpu", "--data", d, "--model", "cifar10_quick", "--batch", "10", "--test-batch", "10",
            "--tau", "2", "--test-every", "0", *extra]


@pytest.mark.parametrize("native", [True, False])
def test_cifar_app_runs(cifar_dir, native):
    s = cifar_app.main(_args(cifar_dir, "--rounds", "2", "--native-loader" if native else "--no-native-loader"))
    assert s.iter == 4
    assert torch.isfinite(s.net.flat_data).all()


def test_checkpoint_resume_is_exact(cifar_dir, tmp_path):
    """2 rounds + checkpoint + resume for 1 round == 3 uninterrupted rounds (weights,
    momentum, LR-schedule iteration and the data stream all continue)."""
    full = cifar_app.main(_args(cifar_dir, "--rounds", "3"))
    pre = str(tmp_path / "ck" / "snap")
    cifar_app.main(_args(cifar_dir, "--rounds", "2", "--snapshot-every", "2", "--snapshot-prefix", pre))
    assert os.path.exists(pre + ".caffemodel") and os.path.exists(pre + ".rank0.solverstate")
    resumed = cifar_app.main(_args(cifar_dir, "--rounds", "3", "--resume", pre))
    assert resumed.iter == full.iter == 6
    assert torch.equal(resumed.net.flat_data, full.net.flat_data)
    assert all(torch.equal(a, b) for a, b in zip(resumed.history, full.history))


def test_fault_injection_exits_and_resume_recovers(cifar_dir, tmp_path):
    pre = str(tmp_path / "f" / "snap")
    cmd = [sys.executable, "-m", "sparknet_amd.apps.cifar_app", *_args(cifar_dir, "--rounds", "4",
           "--snapshot-every", "1", "--snapshot-prefix", pre, "--fail-at-round", "2")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, r.stderr[-2000:]
    assert os.path.exists(pre + ".json")
    s = cifar_app.main(_args(cifar_dir, "--rounds", "4", "--resume", pre))
    assert s.iter == 8


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_multirank_app_via_launcher(cifar_dir):
    """--nproc 2 starts two gloo ranks through parallel.launch.spawn_local; a clean run
    exits 0 (watchdogs marked done, no false failure at shutdown)."""
    cmd = [sys.executable, "-m", "sparknet_amd.apps.cifar_app", *_args(cifar_dir, "--rounds", "2", "--nproc", "2")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


def test_launcher_fails_fast_when_a_rank_dies(cifar_dir):
    import time
    cmd = [sys.executable, "-m", "sparknet_amd.apps.cifar_app",
           *_args(cifar_dir, "--rounds", "50", "--nproc", "2", "--fail-at-round", "1", "--fail-rank", "1")]
    t = time.time()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, r.stderr[-3000:]
    assert time.time() - t < 120


def test_watchdog_ends_surviving_rank_within_seconds(cifar_dir):
    """Ranks started WITHOUT a supervising launcher (each its own process): rank 1 dies
    mid-run with os._exit; rank 0 must notice through its heartbeat watchdog and exit
    non-zero within 30 s of the death instead of hanging in the next all-reduce."""
    import time
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SN_WATCHDOG_TIMEOUT="5")
        cmd = [sys.executable, "-m", "sparknet_amd.apps.cifar_app",
               *_args(cifar_dir, "--rounds", "1000", "--fail-at-round", "2", "--fail-rank", "1")]
        procs.append(subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                      text=True))
    try:
        assert procs[1].wait(timeout=240) == 3
        t_dead = time.time()
        rc0 = procs[0].wait(timeout=60)
        assert time.time() - t_dead < 30
        assert rc0 != 0
        err = procs[0].stderr.read()
        assert "watchdog" in err or rc0 != 0, err[-2000:]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
