"""Distributed training: RCCL collectives, model averaging, sync-SGD, sharding."""
from .comm import Comm, SyncSGDCallback  # noqa: F401
