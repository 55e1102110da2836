"""Training logs in SparkNet's format plus a JSONL metrics stream.

The reference driver wrote wall-clock-stamped lines ``"<sec>: msg"`` and
``"<sec>, i = k: msg"`` to ``$SPARKNET_HOME/training_log_<ts>.txt``
(src/main/scala/apps/CifarApp.scala:36-46) and accuracy as ``"%.2f% accuracy"``.
This logger keeps that human format and adds one JSON object per event
(img/s, all-reduce ms, loss, accuracy) for machine consumption.
"""
from __future__ import annotations

import json
import os
import sys
import time


class TrainingLog:
    def __init__(self, directory: str | None = None, rank: int = 0, name: str = "training_log", echo: bool = True):
        self.t0 = time.time()
        self.rank = rank
        self.echo = echo and rank == 0
        self.f = self.jf = None
        if rank == 0:
            directory = directory or os.environ.get("SPARKNET_HOME", ".")
            os.makedirs(directory, exist_ok=True)
            ts = int(self.t0 * 1000)
            self.path = os.path.join(directory, f"{name}_{ts}.txt")
            self.f = open(self.path, "w")
            self.jf = open(os.path.join(directory, f"{name}_{ts}.jsonl"), "w")

    def elapsed(self) -> float:
        return time.time() - self.t0

    def log(self, message: str, i: int | None = None) -> None:
        if self.rank != 0:
            return
        t = self.elapsed()
        line = f"{t:.3f}: {message}" if i is None else f"{t:.3f}, i = {i}: {message}"
        self.f.write(line + "\n")
        self.f.flush()
        if self.echo:
            print(line, file=sys.stdout, flush=True)

    def metric(self, **kv) -> None:
        if self.rank != 0:
            return
        kv.setdefault("t", round(self.elapsed(), 4))
        self.jf.write(json.dumps(kv) + "\n")
        self.jf.flush()

    def close(self) -> None:
        for f in (self.f, self.jf):
            if f:
                f.close()
