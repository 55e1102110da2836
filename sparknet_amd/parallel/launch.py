"""Single-node process launcher: one rank per GPU, started BEFORE any GPU call.

SparkNet starts one JVM executor per worker through ``spark-submit`` (reference
README.md:26, ``ec2/spark_ec2.py``); on one MI355X node the equivalent is one Python
process per GPU.  ``torch.distributed.run`` is the usual way, but ``bench.py --gpus N`` and
the apps' ``--nproc N`` also start the ranks themselves through :func:`spawn_local`:

* the parent never touches HIP (no ``torch.cuda`` call, no kernel library load), so the
  children own their GPUs exclusively and nothing is re-exec'd from a GPU process;
* every child gets the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR =
  127.0.0.1, MASTER_PORT) and ``SN_LAUNCHED=1``;
* fail fast: when any child exits non-zero, the launcher terminates the others (exact PIDs
  it started) and returns that exit code — the role of Spark's ``spark.task.maxFailures=1``
  (reference src/main/scala/apps/CifarApp.scala:30).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launched_world() -> int | None:
    """WORLD_SIZE when this process was started by a launcher (torchrun or ours)."""
    w = os.environ.get("WORLD_SIZE")
    return int(w) if w is not None else None


def spawn_local(nprocs: int, argv: list[str], env: dict | None = None, port: int | None = None,
                grace_s: float = 10.0, poll_s: float = 0.2) -> int:
    """Run ``python <argv>`` as ``nprocs`` ranks on this node; returns the job's exit code
    (0, or the first non-zero child code; a child killed by a signal returns 128+sig)."""
    port = port or free_port()
    procs = []
    for r in range(nprocs):
        e = dict(os.environ if env is None else env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SN_LAUNCHED="1")
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (the only mode the host supports)
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    code = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and code == 0:
                    code = rc if rc > 0 else 128 - rc
                    print(f"[launch] rank {procs.index(p)} exited with {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    _terminate(live, grace_s)
                    live = []
                    break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        _terminate(procs, grace_s)
        code = code or 130
    return code


def _terminate(procs, grace_s: float) -> None:
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t = time.time() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.0, t - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
