"""Self-diagnosis of a multi-rank run (bench.py at N > 1).

The first RCCL run on an 8-GPU node must explain itself if it is slow: which RCCL
library, how many channels the communicator built, which transport each peer pair uses
(P2P/IPC over xGMI vs SHM through host memory), how long each averaging bucket took on
the GPU, how evenly the ranks stepped, and where each rank's feeder threads live (NUMA).

RCCL reports channels and transports only in its debug log; :func:`rccl_debug_env` points
that log at a per-process file before the communicator exists and :func:`parse_rccl_log`
reads the facts back out of it.
"""
from __future__ import annotations

import glob
import os
import re

_LOG_DIR_ENV = "SN_RCCL_LOG_DIR"


def rccl_debug_env(log_dir: str | None = None) -> str | None:
    """Route RCCL's INIT/GRAPH debug lines of THIS process to a file (before the process
    group initialises; an explicit user NCCL_DEBUG setting is left alone).  Returns the
    file pattern, or None when the user already chose a debug destination."""
    if os.environ.get("NCCL_DEBUG_FILE"):
        return None
    log_dir = log_dir or os.environ.get(_LOG_DIR_ENV) or "/tmp"
    os.makedirs(log_dir, exist_ok=True)
    os.environ.setdefault("NCCL_DEBUG", "INFO")
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH")
    pattern = os.path.join(log_dir, f"sn_rccl.{os.getpid()}.%h.%p.log")
    os.environ["NCCL_DEBUG_FILE"] = pattern
    return pattern


_CHANNEL = re.compile(r"Channel\s+(\d+)\s*/\s*(\d+)")
_VIA = re.compile(r"\bvia\s+([A-Za-z0-9_]+(?:/[A-Za-z0-9_]+)?)")
_VERSION = re.compile(r"\b(?:RCCL|NCCL)\s+version\s+([0-9][0-9A-Za-z.+\-_]*)")
_NCHANNELS = re.compile(r"(\d+)\s+coll channels")


def parse_rccl_log(text: str) -> dict:
    """Facts of one rank's RCCL debug log: library version, channel count (the largest
    'Channel xx/NN' denominator, or 'NN coll channels'), the transports seen ('via P2P/IPC',
    'via SHM', 'via NET/...') with their connection counts, and the number of lines read."""
    version = None
    channels = 0
    transports: dict[str, int] = {}
    lines = text.splitlines()
    for line in lines:
        if version is None:
            m = _VERSION.search(line)
            if m:
                version = m.group(1)
        for m in _CHANNEL.finditer(line):
            channels = max(channels, int(m.group(2)))
        m = _NCHANNELS.search(line)
        if m:
            channels = max(channels, int(m.group(1)))
        for m in _VIA.finditer(line):
            t = m.group(1)
            transports[t] = transports.get(t, 0) + 1
    return {"version": version, "channels": channels or None, "transports": transports, "lines": len(lines)}


def read_rccl_logs(pattern: str | None) -> dict | None:
    """Parse every file this process's RCCL wrote (the %h / %p placeholders expanded)."""
    if not pattern:
        return None
    files = sorted(glob.glob(pattern.replace("%h", "*").replace("%p", "*")))
    if not files:
        return {"version": None, "channels": None, "transports": {}, "lines": 0, "files": 0}
    text = ""
    for f in files:
        try:
            with open(f, errors="replace") as fh:
                text += fh.read()
        except OSError:
            pass
    out = parse_rccl_log(text)
    out["files"] = len(files)
    return out


def rccl_version() -> str | None:
    """torch's view of the collective library version (RCCL on ROCm)."""
    try:
        import torch
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 - no nccl in this build
        return None


def timed_bucket_allreduce(comm, flat, bucket_bytes: int, sync) -> list[float]:
    """GPU-timed all-reduce of each averaging bucket of a scratch copy of ``flat``: one
    hipEvent pair per bucket on the current stream (the collective is issued synchronously,
    so each pair brackets exactly one bucket).  Returns ms per bucket (max over ranks)."""
    import torch
    import torch.distributed as dist
    scratch = flat.detach().clone()
    out = []
    sync()
    comm.barrier()
    for s, e in comm.bucket_ranges(scratch.numel(), bucket_bytes):
        if scratch.is_cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dist.all_reduce(scratch[s:e], op=dist.ReduceOp.SUM)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
        else:
            import time
            t = time.perf_counter()
            dist.all_reduce(scratch[s:e], op=dist.ReduceOp.SUM)
            ms = 1e3 * (time.perf_counter() - t)
        out.append(round(comm.max_over_ranks(ms), 3))
    del scratch
    return out


def check_placement(comm, n_gpus: int, share_gpu: bool, device_index: int, local_rank: int) -> str | None:
    """The failure conditions a scaling run must refuse: a communicator smaller or larger
    than the GPUs asked for, or a rank not on the GPU of its LOCAL_RANK (two ranks on one
    device would silently halve that device's throughput).  Returns an error or None."""
    world = comm.world_size if comm is not None else 1
    if world != n_gpus:
        return f"collective world {world} != --gpus {n_gpus}"
    if not share_gpu and device_index != local_rank:
        return f"rank on cuda:{device_index} but LOCAL_RANK={local_rank}"
    if comm is not None and world > 1:
        devs = comm.allgather_int(device_index)
        if not share_gpu and len(set(devs)) != len(devs):
            return f"ranks share devices: {devs}"
    return None
