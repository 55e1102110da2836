"""Layer base class, learnable ``Param`` and the type-string registry.

Reference: ``Layer<Dtype>`` (caffe/include/caffe/layer.hpp:67-514) and
``LayerRegistry`` (caffe/include/caffe/layer_factory.hpp:74-137).

A layer implements ``setup`` (LayerSetUp + first Reshape), ``reshape``, ``forward`` and
``backward`` over lists of :class:`Blob`.  There is one implementation per layer; it
calls the device-dispatching ops in :mod:`sparknet_amd.ops`, which run hand-written HIP
kernels on an MI355X and PyTorch fp32 reference code on the CPU.

Parameters: every learnable blob is a :class:`Param` with an fp32 master (a view into
the net's single flat parameter buffer, like Caffe's ``Params``/``GPUParams``,
caffe/src/caffe/parallel.cpp:69-115), an fp32 gradient (view into the flat gradient
buffer) and a compute copy (bf16 view of the flat compute buffer on GPU).  A param's
*internal* layout is the one the kernels want (e.g. conv weights [Cout][R][S][Cin/g]);
``to_caffe`` / ``from_caffe`` convert to the canonical Caffe layout used by fillers,
``.caffemodel`` files and the get/set-weights API.
"""
from __future__ import annotations

import math
from typing import Callable

import torch

from .blob import Blob


class Param:
    def __init__(self, caffe_shape, shape=None, to_caffe: Callable | None = None,
                 from_caffe: Callable | None = None, filler=None, name: str = ""):
        self.caffe_shape = tuple(int(s) for s in caffe_shape)
        self.shape = tuple(int(s) for s in (shape if shape is not None else caffe_shape))
        self._to_caffe = to_caffe
        self._from_caffe = from_caffe
        self.filler = filler
        self.name = name
        self.lr_mult = 1.0
        self.decay_mult = 1.0
        self.owner: Param | None = None  # set when shared by ParamSpec.name
        self.data = torch.zeros(self.shape, dtype=torch.float32)  # replaced by flat views
        self.diff: torch.Tensor | None = None
        self.compute: torch.Tensor | None = None
        self.offset = -1  # element offset in the flat buffers
        self.version = 0  # bumped whenever master changes outside the solver

    @property
    def count(self) -> int:
        return int(math.prod(self.shape))

    @property
    def caffe_count(self) -> int:
        return int(math.prod(self.caffe_shape))

    def to_caffe(self, t: torch.Tensor | None = None) -> torch.Tensor:
        t = self.data if t is None else t
        t = t.detach().float()
        return (self._to_caffe(t) if self._to_caffe else t).reshape(self.caffe_shape)

    def from_caffe(self, t: torch.Tensor) -> torch.Tensor:
        t = t.reshape(self.caffe_shape).float()
        out = self._from_caffe(t) if self._from_caffe else t
        return out.reshape(self.shape)

    def set_caffe(self, t: torch.Tensor) -> None:
        self.data.copy_(self.from_caffe(t.to(self.data.device)))

    def root(self) -> "Param":
        p = self
        while p.owner is not None:
            p = p.owner
        return p

    def __repr__(self):
        return f"Param({self.name!r}, caffe={self.caffe_shape}, internal={self.shape})"


class Layer:
    type_name = "Layer"
    # arity constraints (Layer::ExactNumBottomBlobs & co.); -1 = unchecked
    exact_bottoms = -1
    min_bottoms = -1
    max_bottoms = -1
    exact_tops = -1
    min_tops = -1
    max_tops = -1
    auto_top_blobs = False
    is_loss = False
    is_data = False

    def __init__(self, lp, ctx):
        self.lp = lp
        self.ctx = ctx  # NetContext: device, compute dtype, phase, rng
        self.name = lp.name
        self.phase = lp.phase
        self.params: list[Param] = []
        self.param_propagate_down: list[bool] = []
        self.loss_weights: list[float] = []

    # -- helpers ---------------------------------------------------------------------
    @property
    def device(self) -> torch.device:
        return self.ctx.device

    @property
    def dtype(self) -> torch.dtype:
        return self.ctx.dtype

    def add_param(self, caffe_shape, shape=None, to_caffe=None, from_caffe=None, filler=None) -> Param:
        p = Param(caffe_shape, shape, to_caffe, from_caffe, filler, name=f"{self.name}/{len(self.params)}")
        self.params.append(p)
        return p

    def check_blob_counts(self, bottoms, tops) -> None:
        nb, nt = len(bottoms), len(tops)
        def chk(cond, msg):
            if not cond:
                raise ValueError(f"{self.type_name} layer {self.name!r}: {msg}")
        if self.exact_bottoms >= 0:
            chk(nb == self.exact_bottoms, f"takes {self.exact_bottoms} bottom blob(s), got {nb}")
        if self.min_bottoms >= 0:
            chk(nb >= self.min_bottoms, f"takes at least {self.min_bottoms} bottom blob(s)")
        if self.max_bottoms >= 0:
            chk(nb <= self.max_bottoms, f"takes at most {self.max_bottoms} bottom blob(s)")
        if self.exact_tops >= 0:
            chk(nt == self.exact_tops, f"produces {self.exact_tops} top blob(s), got {nt}")
        if self.min_tops >= 0:
            chk(nt >= self.min_tops, f"produces at least {self.min_tops} top blob(s)")
        if self.max_tops >= 0:
            chk(nt <= self.max_tops, f"produces at most {self.max_tops} top blob(s)")

    def needed_tops(self) -> int:
        return max(self.min_tops, self.exact_tops)

    # -- lifecycle (Layer::SetUp, layer.hpp:67-80) -------------------------------------
    def setup(self, bottoms: list[Blob], tops: list[Blob]) -> None:
        self.check_blob_counts(bottoms, tops)
        self.layer_setup(bottoms, tops)
        self.reshape(bottoms, tops)
        self.set_loss_weights(tops)

    def layer_setup(self, bottoms, tops) -> None:
        pass

    def reshape(self, bottoms, tops) -> None:
        raise NotImplementedError

    def set_loss_weights(self, tops) -> None:
        """Layer::SetLossWeights (layer.hpp:414-428): loss layers default to weight 1
        on top 0; explicit ``loss_weight`` entries override."""
        n = len(tops)
        lw = list(self.lp.loss_weight)
        if not lw and self.is_loss and n > 0:
            lw = [1.0] + [0.0] * (n - 1)
        if lw and len(lw) != n:
            raise ValueError(f"layer {self.name!r}: loss_weight must be unspecified or given per top")
        self.loss_weights = lw + [0.0] * (n - len(lw))

    def loss(self, top_id: int) -> float:
        return self.loss_weights[top_id] if top_id < len(self.loss_weights) else 0.0

    def forward(self, bottoms, tops) -> None:
        raise NotImplementedError

    def backward(self, tops, propagate_down, bottoms) -> None:
        pass

    def allow_force_backward(self, bottom_id: int) -> bool:
        return True

    def param_grads_needed(self, i: int) -> bool:
        return i < len(self.param_propagate_down) and self.param_propagate_down[i]

    supports_grad_overwrite = False  # backward honours grad_overwrite() (see Net.clear_param_diffs)

    def grad_overwrite(self, i: int) -> bool:
        """True when param i's gradient buffer was lazily cleared and this is its first
        write of the pass: the caller must store, not accumulate."""
        st = self.ctx.stale_diffs
        if not st:
            return False
        off = self.params[i].offset
        if off in st:
            st.discard(off)
            return True
        return False

    def __repr__(self):
        return f"<{self.type_name} {self.name!r}>"


_REGISTRY: dict[str, type] = {}


def register(*names: str):
    def deco(cls):
        for n in names:
            if n in _REGISTRY:
                raise ValueError(f"layer type {n!r} registered twice")
            _REGISTRY[n] = cls
        cls.type_name = names[0]
        return cls
    return deco


def create_layer(lp, ctx) -> Layer:
    """LayerRegistry::CreateLayer (layer_factory.hpp:74-83)."""
    from .. import layers  # noqa: F401  (populates the registry)
    t = lp.type
    if t not in _REGISTRY:
        raise KeyError(f"Unknown layer type: {t!r} (known: {', '.join(sorted(_REGISTRY))})")
    return _REGISTRY[t](lp, ctx)


def layer_types() -> list[str]:
    from .. import layers  # noqa: F401
    return sorted(_REGISTRY)
