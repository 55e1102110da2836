"""Trace ranges for rocprofv3 / roctracer timelines (ranges around the round
phases — data, compute, all-reduce, eval — so a trace shows which MFMA kernels belong to
which phase).  ``torch.cuda.nvtx`` emits roctx markers on ROCm builds.  Off unless
``SN_TRACE=1`` (a marker costs a host call per range)."""
from __future__ import annotations

import contextlib
import os

import torch

ENABLED = os.environ.get("SN_TRACE", "0") == "1"


@contextlib.contextmanager
def trace_range(name: str):
    if not ENABLED or not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()
