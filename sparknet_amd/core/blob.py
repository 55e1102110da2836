"""Blob: the unit of data exchanged between layers (Caffe ``Blob<Dtype>``,
caffe/include/caffe/blob.hpp, caffe/src/caffe/blob.cpp).

Differences from the reference, by design:

* No implicit host/device state machine (SyncedMemory, caffe/src/caffe/syncedmem.cpp:25-77):
  a blob's storage lives on exactly one device; moves are explicit.
* ``shape`` is the *logical* Caffe shape (N, C, H, W for images) but 4-D activations are
  stored channels-last: ``data`` has physical shape (N, H, W, C).  Every kernel in
  ``csrc/kernels`` is written for that layout (contiguous channels feed the implicit-GEMM
  conv and vectorised pooling / LRN).  ``nchw()`` gives the logical view.
* Activations use the net's compute dtype (bf16 on MI355X, fp32 on the CPU reference
  path); learnable parameters are ``Param`` objects with an fp32 master.
"""
from __future__ import annotations

import math

import torch


def physical_shape(shape: tuple) -> tuple:
    if len(shape) == 4:
        n, c, h, w = shape
        return (n, h, w, c)
    return tuple(shape)


class Blob:
    __slots__ = ("name", "shape", "dtype", "device", "_data", "_diff")

    def __init__(self, name: str = "", shape=(), dtype=torch.float32, device="cpu"):
        self.name = name
        self.shape = tuple(int(s) for s in shape)
        self.dtype = dtype
        self.device = torch.device(device)
        self._data = None
        self._diff = None

    # -- shape -----------------------------------------------------------------------
    def reshape(self, shape, dtype=None) -> "Blob":
        shape = tuple(int(s) for s in shape)
        dtype = dtype or self.dtype
        if shape != self.shape or dtype != self.dtype:
            self.shape, self.dtype = shape, dtype
            self._data = None
            self._diff = None
        return self

    def reshape_like(self, other: "Blob") -> "Blob":
        return self.reshape(other.shape, other.dtype)

    @property
    def count(self) -> int:
        return int(math.prod(self.shape)) if self.shape else 1

    def num_axes(self) -> int:
        return len(self.shape)

    def canonical_axis(self, axis: int) -> int:
        return axis + len(self.shape) if axis < 0 else axis

    def count_range(self, start: int, end: int | None = None) -> int:
        end = len(self.shape) if end is None else end
        return int(math.prod(self.shape[start:end]))

    @property
    def is_image(self) -> bool:
        return len(self.shape) == 4

    # -- storage ---------------------------------------------------------------------
    @property
    def data(self) -> torch.Tensor:
        if self._data is None:
            self._data = torch.zeros(physical_shape(self.shape), dtype=self.dtype, device=self.device)
        return self._data

    @data.setter
    def data(self, t: torch.Tensor) -> None:
        assert tuple(t.shape) == physical_shape(self.shape), (self.name, t.shape, self.shape)
        self._data = t

    @property
    def diff(self) -> torch.Tensor:
        if self._diff is None:
            self._diff = torch.zeros(physical_shape(self.shape), dtype=self.dtype, device=self.device)
        return self._diff

    @diff.setter
    def diff(self, t: torch.Tensor) -> None:
        assert tuple(t.shape) == physical_shape(self.shape), (self.name, t.shape, self.shape)
        self._diff = t

    def has_diff(self) -> bool:
        return self._diff is not None

    def share_data(self, other: "Blob") -> None:
        assert self.count == other.count
        self._data = other.data.view(physical_shape(self.shape))

    def share_diff(self, other: "Blob") -> None:
        assert self.count == other.count
        self._diff = other.diff.view(physical_shape(self.shape))

    # -- logical views ---------------------------------------------------------------
    def nchw(self, diff: bool = False) -> torch.Tensor:
        t = self.diff if diff else self.data
        return t.permute(0, 3, 1, 2) if self.is_image else t

    def set_nchw(self, t: torch.Tensor, diff: bool = False) -> None:
        """Copy a logical-layout tensor into the blob (converting dtype/layout)."""
        t = t.to(self.device)
        if self.is_image:
            t = t.permute(0, 2, 3, 1)
        dst = self.diff if diff else self.data
        dst.copy_(t.reshape(dst.shape))

    def asum_data(self) -> float:
        return float(self.data.float().abs().sum())

    def __repr__(self) -> str:
        return f"Blob({self.name!r}, shape={self.shape}, dtype={self.dtype}, device={self.device})"
