"""Data-entry layers.

* ``JavaData`` (SparkNet's RDD feed, caffe/src/caffe/layers/java_data_layer.cpp:10-47,
  proto field java_data_param=149) and ``Input`` / ``MemoryData``: externally fed.
  The reference called back into the JVM for every minibatch and then did a
  synchronous H2D copy; here the layer owns a device top blob that a feeder writes into
  (``set_source``): typically the device-side augment kernel reading a pinned uint8
  ring slot that was copied on a side stream (see :mod:`sparknet_amd.data.prefetch`).
* ``DummyData`` (dummy_data_layer.cpp): filler-generated blobs — the synthetic-data
  backend of tests and benchmarks.
* ``Data``: Datum records from an on-disk DB (our ``SNDB`` record file; LMDB/LevelDB
  are not available in this environment) with the DataTransformer semantics
  (crop / mirror / mean / scale).
* ``ImageData``: image list file decoded with PIL.
"""
from __future__ import annotations

from typing import Callable

import torch

from ..core.filler import fill
from ..core.layer import Layer, register


class ExternalDataLayer(Layer):
    """Top blobs are written by an external feeder: ``source(top_tensors)`` or a plain
    tensor copy (``feed``)."""
    is_data = True
    min_tops = 1

    def layer_setup(self, bottoms, tops):
        self.source: Callable | None = None

    def set_source(self, fn: Callable | None) -> None:
        """``fn(layer, tops)`` fills ``tops[i].data`` in place (device side)."""
        self.source = fn

    def feed(self, *tensors: torch.Tensor) -> None:
        """Copy logical-layout (NCHW) tensors into the tops (convenience API)."""
        for t, x in zip(self._tops, tensors):
            t.set_nchw(torch.as_tensor(x).to(t.dtype))

    def reshape(self, bottoms, tops):
        self._tops = tops

    def forward(self, bottoms, tops):
        if self.source is not None:
            self.source(self, tops)

    def backward(self, tops, propagate_down, bottoms):
        pass


@register("JavaData", "RDD")
class JavaDataLayer(ExternalDataLayer):
    exact_tops = 1

    def reshape(self, bottoms, tops):
        super().reshape(bottoms, tops)
        shape = tuple(self.lp.java_data_param.shape.dim)
        if not shape:
            raise ValueError(f"JavaData layer {self.name!r} needs java_data_param.shape")
        tops[0].reshape(shape, self.dtype if len(shape) == 4 else torch.float32)


@register("Input")
class InputLayer(ExternalDataLayer):
    """Caffe's newer ``Input`` layer: shapes from ``java_data_param.shape`` entries (the
    schema has no input_param; one shape per top is taken from ``net.input_shape``-like
    dims stored in java_data_param for compatibility)."""

    def reshape(self, bottoms, tops):
        super().reshape(bottoms, tops)
        shape = tuple(self.lp.java_data_param.shape.dim)
        for t in tops:
            t.reshape(shape, self.dtype if len(shape) == 4 else torch.float32)


@register("MemoryData")
class MemoryDataLayer(ExternalDataLayer):
    exact_tops = 2

    def layer_setup(self, bottoms, tops):
        super().layer_setup(bottoms, tops)
        p = self.lp.memory_data_param
        self.batch = int(p.batch_size)
        self.chw = (int(p.channels), int(p.height), int(p.width))
        self.data = None
        self.labels = None
        self.pos = 0

    def reshape(self, bottoms, tops):
        super().reshape(bottoms, tops)
        tops[0].reshape((self.batch,) + self.chw, self.dtype)
        tops[1].reshape((self.batch,), torch.float32)

    def reset(self, data, labels) -> None:
        """MemoryDataLayer::Reset: arrays of N x C x H x W and N labels."""
        data = torch.as_tensor(data)
        labels = torch.as_tensor(labels)
        if data.shape[0] % self.batch:
            raise ValueError("MemoryData: number of samples must be a multiple of batch_size")
        self.data, self.labels, self.pos = data, labels, 0

    def forward(self, bottoms, tops):
        if self.source is not None:
            self.source(self, tops)
            return
        if self.data is None:
            raise RuntimeError("MemoryData layer used before reset()")
        sl = slice(self.pos, self.pos + self.batch)
        tops[0].set_nchw(self.data[sl].to(self.dtype))
        tops[1].data.copy_(self.labels[sl].float().to(self.device))
        self.pos = (self.pos + self.batch) % self.data.shape[0]


@register("DummyData")
class DummyDataLayer(Layer):
    is_data = True
    min_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.dummy_data_param
        n = len(tops)
        if len(p.shape):
            shapes = [tuple(s.dim) for s in p.shape]
        else:
            shapes = [(p.num[i if len(p.num) > 1 else 0], p.channels[i if len(p.channels) > 1 else 0],
                       p.height[i if len(p.height) > 1 else 0], p.width[i if len(p.width) > 1 else 0])
                      for i in range(n)]
        if len(shapes) == 1 and n > 1:
            shapes = shapes * n
        fillers = list(p.data_filler)
        if not fillers:
            fillers = [None] * n
        elif len(fillers) == 1:
            fillers = fillers * n
        self.shapes, self.fillers = shapes, fillers
        # constant fillers are filled once; others refill every forward (dummy_data_layer.cpp)
        self.refill = [f is not None and f.type != "constant" for f in fillers]

    def reshape(self, bottoms, tops):
        for t, s in zip(tops, self.shapes):
            t.reshape(s, self.dtype if len(s) == 4 else torch.float32)
        self._filled = False

    def _fill(self, t, f):
        v = fill(f, t.shape, self.ctx.gen)
        t.set_nchw(v)

    def forward(self, bottoms, tops):
        for i, t in enumerate(tops):
            if self.refill[i] or not self._filled:
                self._fill(t, self.fillers[i])
        self._filled = True


@register("Data")
class DataLayer(ExternalDataLayer):
    """DB-backed data layer: reads ``Datum`` records from an SNDB file (see
    :mod:`sparknet_amd.data.db`) and applies the transform_param on the host."""
    exact_tops = -1
    min_tops = 1
    max_tops = 2

    def layer_setup(self, bottoms, tops):
        super().layer_setup(bottoms, tops)
        from ..data.db import DatumReader
        p = self.lp.data_param
        self.reader = DatumReader(p.source)
        self.batch = int(p.batch_size)
        self.tp = self.lp.transform_param
        d = self.reader.peek()
        crop = self.tp.crop_size or p.crop_size
        self.chw = (d.channels, crop or d.height, crop or d.width)
        from ..data.transform import DataTransformer
        self.transformer = DataTransformer(self.tp, self.phase, seed=self.ctx.seed)

    def reshape(self, bottoms, tops):
        super().reshape(bottoms, tops)
        tops[0].reshape((self.batch,) + self.chw, self.dtype)
        if len(tops) > 1:
            tops[1].reshape((self.batch,), torch.float32)

    def forward(self, bottoms, tops):
        if self.source is not None:
            self.source(self, tops)
            return
        imgs, labels = [], []
        for _ in range(self.batch):
            d = self.reader.next()
            imgs.append(self.transformer.transform_datum(d))
            labels.append(d.label)
        tops[0].set_nchw(torch.stack(imgs))
        if len(tops) > 1:
            tops[1].data.copy_(torch.tensor(labels, dtype=torch.float32))


@register("ImageData")
class ImageDataLayer(ExternalDataLayer):
    """image_data_layer.cpp: ``source`` lists "path label" lines; PIL decode + resize."""
    exact_tops = 2

    def layer_setup(self, bottoms, tops):
        super().layer_setup(bottoms, tops)
        import os
        p = self.lp.image_data_param
        with open(p.source) as f:
            self.lines = [(ln.rsplit(None, 1)[0], int(ln.rsplit(None, 1)[1])) for ln in f if ln.strip()]
        self.root = p.root_folder
        self.batch = int(p.batch_size)
        self.new_hw = (int(p.new_height), int(p.new_width))
        self.color = p.is_color
        self.pos = 0
        if p.shuffle:
            g = torch.Generator().manual_seed(self.ctx.seed)
            perm = torch.randperm(len(self.lines), generator=g).tolist()
            self.lines = [self.lines[i] for i in perm]
        first = self._load(os.path.join(self.root, self.lines[0][0]))
        crop = self.lp.transform_param.crop_size
        self.chw = (first.shape[0], crop or first.shape[1], crop or first.shape[2])
        from ..data.transform import DataTransformer
        self.transformer = DataTransformer(self.lp.transform_param, self.phase, seed=self.ctx.seed)

    def _load(self, path):
        from PIL import Image
        import numpy as np
        im = Image.open(path).convert("RGB" if self.color else "L")
        if self.new_hw[0] and self.new_hw[1]:
            im = im.resize((self.new_hw[1], self.new_hw[0]))
        a = np.asarray(im, dtype=np.uint8)
        if a.ndim == 2:
            a = a[:, :, None]
        a = a[:, :, ::-1].copy() if self.color else a  # Caffe/OpenCV order is BGR
        return torch.from_numpy(a).permute(2, 0, 1).contiguous()

    def reshape(self, bottoms, tops):
        super().reshape(bottoms, tops)
        tops[0].reshape((self.batch,) + self.chw, self.dtype)
        tops[1].reshape((self.batch,), torch.float32)

    def forward(self, bottoms, tops):
        import os
        imgs, labels = [], []
        for _ in range(self.batch):
            path, lab = self.lines[self.pos]
            self.pos = (self.pos + 1) % len(self.lines)
            imgs.append(self.transformer.transform_chw(self._load(os.path.join(self.root, path))))
            labels.append(lab)
        tops[0].set_nchw(torch.stack(imgs))
        tops[1].data.copy_(torch.tensor(labels, dtype=torch.float32))
