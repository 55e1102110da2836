"""Node topology helpers for one-process-per-GPU jobs.

An 8x MI355X node hangs its GPUs off (typically) two CPU sockets.  Each rank copies a
full uint8 ImageNet minibatch host->device every step (CaffeNet: 50 MB per 2.7 ms step per
GPU), so the pinned staging ring should live in the memory of the socket the GPU's PCIe
root port belongs to.  :func:`bind_to_gpu_numa` restricts the calling process to that
node's CPUs BEFORE the pinned buffers are allocated (first-touch placement), using only
sysfs (no libnuma in the image).  Best effort: where sysfs does not report a node (VMs,
containers) nothing changes.
"""
from __future__ import annotations

import os


def _parse_cpulist(s: str) -> set[int]:
    out: set[int] = set()
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def gpu_numa_node(device_index: int) -> int:
    """NUMA node of a GPU's PCIe function (-1 when unknown)."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        addr = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{addr}/numa_node") as f:
            return int(f.read().strip())
    except Exception:
        return -1


def bind_to_gpu_numa(device_index: int) -> int:
    """Pin this process to the CPUs of its GPU's NUMA node; returns the node or -1."""
    node = gpu_numa_node(device_index)
    if node < 0 or not hasattr(os, "sched_setaffinity"):
        return -1
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _parse_cpulist(f.read())
        allowed = os.sched_getaffinity(0) & cpus
        if not allowed:
            return -1
        os.sched_setaffinity(0, allowed)
        return node
    except OSError:
        return -1
