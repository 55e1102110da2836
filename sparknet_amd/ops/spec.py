"""Geometry records shared by the reference (CPU/PyTorch) and HIP implementations."""
from __future__ import annotations

import math
from dataclasses import dataclass


@dataclass(frozen=True)
class ConvSpec:
    N: int
    H: int
    W: int
    C: int          # input channels
    K: int          # output channels (num_output)
    R: int
    S: int
    sh: int = 1
    sw: int = 1
    ph: int = 0
    pw: int = 0
    dh: int = 1
    dw: int = 1
    groups: int = 1

    @property
    def P(self) -> int:
        return (self.H + 2 * self.ph - (self.dh * (self.R - 1) + 1)) // self.sh + 1

    @property
    def Q(self) -> int:
        return (self.W + 2 * self.pw - (self.dw * (self.S - 1) + 1)) // self.sw + 1

    @property
    def Cg(self) -> int:
        return self.C // self.groups

    @property
    def Kg(self) -> int:
        return self.K // self.groups

    def with_batch(self, n: int) -> "ConvSpec":
        return ConvSpec(n, self.H, self.W, self.C, self.K, self.R, self.S, self.sh, self.sw,
                        self.ph, self.pw, self.dh, self.dw, self.groups)


@dataclass(frozen=True)
class ConvNdSpec:
    """N-d convolution over a logical [num][C][D_0..D_{n-1}] blob (Caffe's general path:
    base_conv_layer.cpp:16-40 — every axis before the channel axis is batch, every axis
    after it spatial; no dilation in this Caffe)."""
    num: int
    C: int
    K: int
    ins: tuple
    ks: tuple
    st: tuple
    pd: tuple
    groups: int = 1

    @property
    def nd(self) -> int:
        return len(self.ins)

    @property
    def outs(self) -> tuple:
        return tuple((i + 2 * p - k) // s + 1 for i, k, s, p in zip(self.ins, self.ks, self.st, self.pd))

    @property
    def Cg(self) -> int:
        return self.C // self.groups

    @property
    def Kg(self) -> int:
        return self.K // self.groups

    @property
    def T(self) -> int:
        return math.prod(self.ks)

    @property
    def P(self) -> int:
        return math.prod(self.outs)

    @property
    def Sin(self) -> int:
        return math.prod(self.ins)


POOL_MAX, POOL_AVE, POOL_STOCHASTIC = 0, 1, 2


@dataclass(frozen=True)
class PoolSpec:
    N: int
    H: int
    W: int
    C: int
    kh: int
    kw: int
    sh: int = 1
    sw: int = 1
    ph: int = 0
    pw: int = 0
    method: int = POOL_MAX

    @property
    def P(self) -> int:
        # Caffe ceil-mode output size with the "last window starts inside" clip
        # (caffe/src/caffe/layers/pooling_layer.cpp:90-103)
        p = int(math.ceil((self.H + 2 * self.ph - self.kh) / self.sh)) + 1
        if self.ph and (p - 1) * self.sh >= self.H + self.ph:
            p -= 1
        return p

    @property
    def Q(self) -> int:
        q = int(math.ceil((self.W + 2 * self.pw - self.kw) / self.sw)) + 1
        if self.pw and (q - 1) * self.sw >= self.W + self.pw:
            q -= 1
        return q
