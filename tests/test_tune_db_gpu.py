"""Kernel selection is reproducible: with first-call autotuning off (the
default) every GEMM of the zoo models' bench configurations comes from the committed tuning
database, and two processes on one box produce bit-identical CaffeNet loss trajectories."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(*extra, timeout=240):
    env = dict(os.environ)
    env.pop("SN_GEMM_AUTOTUNE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *extra], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line), p.stderr


@pytest.mark.parametrize("model,extra", [
    ("caffenet", ()), ("alexnet", ()), ("googlenet", ()), ("cifar10_quick", ()),
    ("vgg16", ()), ("vgg16", ("--dtype", "fp8")),
])
def test_bench_products_all_in_tuning_db(gpu, model, extra):
    out, _ = _bench("--model", model, "--steps", "2", "--warmup", "1", *extra)
    assert out["autotune"] is False
    assert out["tune_misses"] == 0, out


def test_two_processes_bitwise_identical_caffenet_losses(gpu):
    runs = [_bench("--steps", "20", "--warmup", "2", "--loss-trace")[1] for _ in range(2)]
    traces = [[ln for ln in err.splitlines() if ln.startswith("rank 0 losses:")][-1] for err in runs]
    assert traces[0] == traces[1], traces
