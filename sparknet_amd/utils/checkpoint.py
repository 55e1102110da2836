"""Checkpoint IO in Caffe formats (.caffemodel = NetParameter with per-layer blobs,
.solverstate = SolverState), bit-compatible with the reference
(caffe/src/caffe/solver.cpp:447-519, net.cpp:805-923).  Masters are fp32 regardless
of the bf16 compute dtype; blobs are written in Caffe's canonical layout.
"""
from __future__ import annotations

import json
import os

from .. import proto


def save_caffemodel(net, path: str, write_diff: bool = False) -> None:
    proto.write_binary(path, net.to_proto(write_diff=write_diff))


def load_caffemodel(net, path: str) -> None:
    net.copy_trained_layers_from(proto.read_net(path))


def write_round_sidecar(path: str, **info) -> None:
    """Round counter / metadata for model-averaging resume (JSON next to the model)."""
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(info, f)
    os.replace(tmp, path)


def read_round_sidecar(path: str) -> dict:
    with open(path) as f:
        return json.load(f)
