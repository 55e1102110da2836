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
* ``HDF5Data`` / ``HDF5Output``: HDF5 files through the built-in codec
  (:mod:`sparknet_amd.utils.hdf5`).
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


@register("WindowData")
class WindowDataLayer(ExternalDataLayer):
    """R-CNN window sampler (caffe/src/caffe/layers/window_data_layer.cpp:33-468), PIL
    instead of OpenCV. The window file repeats ``# idx / path / C H W / n / n x (label
    overlap x1 y1 x2 y2)``; windows with overlap >= fg_threshold are foreground, those
    below bg_threshold background (label forced to 0). Each batch draws
    ``batch - int(batch * fg_fraction)`` background windows and then the foreground ones,
    crops them with optional context padding (``warp`` or ``square`` mode), resizes
    bilinearly to crop_size, mirrors, and writes (pixel - mean) * scale into a zeroed
    batch — the padded border stays 0, as in the reference."""
    exact_tops = 2

    def layer_setup(self, bottoms, tops):
        super().layer_setup(bottoms, tops)
        import numpy as np
        p = self.lp.window_data_param
        tp = self.lp.transform_param
        self.p, self.crop, self.mirror = p, int(tp.crop_size), bool(tp.mirror)
        if self.crop <= 0:
            raise ValueError(f"WindowData layer {self.name!r} needs transform_param.crop_size > 0")
        self.images, self.fg, self.bg = [], [], []
        with open(p.source) as f:
            tok = f.read().split()
        i = 0
        while i < len(tok):
            if tok[i] != "#":
                raise ValueError(f"window file {p.source!r}: expected '#' at token {i}")
            idx, path = int(tok[i + 1]), p.root_folder + tok[i + 2]
            c, h, w, n = (int(t) for t in tok[i + 3:i + 7])
            i += 7
            while len(self.images) <= idx:
                self.images.append(None)
            self.images[idx] = (path, (c, h, w))
            for _ in range(n):
                lab, ov = int(tok[i]), float(tok[i + 1])
                x1, y1, x2, y2 = (int(t) for t in tok[i + 2:i + 6])
                i += 6
                if ov >= p.fg_threshold:
                    if lab <= 0:
                        raise ValueError("foreground windows need a positive label")
                    self.fg.append((idx, lab, ov, x1, y1, x2, y2))
                elif ov < p.bg_threshold:
                    self.bg.append((idx, 0, 0.0, x1, y1, x2, y2))
        if not self.images:
            raise ValueError(f"window file {p.source!r} is empty")
        self.channels = self.images[0][1][0]
        self.mean = self.mean_values = None
        if tp.mean_file:
            if len(tp.mean_value):
                raise ValueError("Cannot specify mean_file and mean_value at the same time")
            from ..data.loaders import read_mean_binaryproto
            self.mean = np.asarray(read_mean_binaryproto(tp.mean_file), np.float32)
        elif len(tp.mean_value):
            mv = list(tp.mean_value)
            self.mean_values = np.asarray(mv if len(mv) > 1 else mv * self.channels, np.float32)
        self.rng = np.random.default_rng(self.ctx.seed)
        self.cache = {}

    def reshape(self, bottoms, tops):
        super().reshape(bottoms, tops)
        b = int(self.p.batch_size)
        tops[0].reshape((b, self.channels, self.crop, self.crop), self.dtype)
        tops[1].reshape((b,), torch.float32)

    def _image(self, idx):
        import numpy as np
        from PIL import Image
        if idx in self.cache:
            return self.cache[idx]
        a = np.asarray(Image.open(self.images[idx][0]).convert("RGB"), np.uint8)[:, :, ::-1]  # BGR
        if self.p.cache_images:
            self.cache[idx] = a
        return a

    def _window(self, win, mirror):
        """One cropped window: (HWC uint8 patch, pad_h, pad_w)."""
        import numpy as np
        from PIL import Image
        img = self._image(win[0])
        rows, cols = img.shape[:2]
        crop, ctx_pad = self.crop, int(self.p.context_pad)
        x1, y1, x2, y2 = win[3:]
        out_w = out_h = crop
        pad_h = pad_w = 0
        if ctx_pad > 0 or self.p.crop_mode == "square":
            cscale = crop / (crop - 2 * ctx_pad)
            hh, hw = (y2 - y1 + 1) / 2.0, (x2 - x1 + 1) / 2.0
            cx, cy = x1 + hw, y1 + hh
            if self.p.crop_mode == "square":
                hh = hw = max(hh, hw)
            x1, x2 = int(round(cx - hw * cscale)), int(round(cx + hw * cscale))
            y1, y2 = int(round(cy - hh * cscale)), int(round(cy + hh * cscale))
            uh, uw = y2 - y1 + 1, x2 - x1 + 1
            px1, py1 = max(0, -x1), max(0, -y1)
            px2, py2 = max(0, x2 - cols + 1), max(0, y2 - rows + 1)
            x1, x2, y1, y2 = x1 + px1, x2 - px2, y1 + py1, y2 - py2
            sx, sy = crop / uw, crop / uh
            out_w = int(round((x2 - x1 + 1) * sx))
            out_h = int(round((y2 - y1 + 1) * sy))
            px1, px2 = int(round(px1 * sx)), int(round(px2 * sx))
            py1 = int(round(py1 * sy))
            pad_h, pad_w = py1, (px2 if mirror else px1)
            out_h, out_w = min(out_h, crop - pad_h), min(out_w, crop - pad_w)
        roi = np.ascontiguousarray(img[y1:y2 + 1, x1:x2 + 1])
        patch = np.asarray(Image.fromarray(roi).resize((out_w, out_h), Image.BILINEAR), np.uint8)
        if mirror:
            patch = patch[:, ::-1]
        return patch, pad_h, pad_w

    def next_batch(self):
        """Host batch: (N x C x crop x crop float32, N labels)."""
        import numpy as np
        b, crop = int(self.p.batch_size), self.crop
        data = np.zeros((b, self.channels, crop, crop), np.float32)
        labels = np.zeros((b,), np.float32)
        n_fg = int(b * self.p.fg_fraction)
        item = 0
        for pool, count in ((self.bg, b - n_fg), (self.fg, n_fg)):
            for _ in range(count):
                win = pool[int(self.rng.integers(len(pool)))]
                mirror = self.mirror and bool(self.rng.integers(2))
                patch, ph, pw = self._window(win, mirror)
                h, w = patch.shape[:2]
                px = patch.transpose(2, 0, 1).astype(np.float32)
                if self.mean is not None:
                    off = (self.mean.shape[2] - crop) // 2
                    px = px - self.mean[:, off + ph:off + ph + h, off + pw:off + pw + w]
                elif self.mean_values is not None:
                    px = px - self.mean_values[:, None, None]
                data[item, :, ph:ph + h, pw:pw + w] = px * self.p.scale
                labels[item] = win[1]
                item += 1
        return data, labels

    def forward(self, bottoms, tops):
        if self.source is not None:
            self.source(self, tops)
            return
        data, labels = self.next_batch()
        tops[0].set_nchw(torch.from_numpy(data).to(self.dtype))
        tops[1].data.copy_(torch.from_numpy(labels))


def _resolve_listed(path: str, list_file: str) -> str:
    """File names in a list file are taken relative to the working directory (as Caffe
    does); failing that, relative to the list file's directory, then its basename there."""
    import os
    if os.path.exists(path):
        return path
    base = os.path.dirname(os.path.abspath(list_file))
    for cand in (os.path.join(base, path), os.path.join(base, os.path.basename(path))):
        if os.path.exists(cand):
            return cand
    raise FileNotFoundError(f"HDF5 file {path!r} listed in {list_file!r} not found")


@register("HDF5Data")
class HDF5DataLayer(Layer):
    """hdf5_data_layer.cpp:26-160: ``source`` lists HDF5 files; top i is the dataset
    named like the top; rows are served in order (or shuffled, per file and per pass) and
    files advance when one is exhausted.  Rows are gathered on the host and copied once
    per batch."""
    is_data = True
    min_tops = 1

    def layer_setup(self, bottoms, tops):
        if self.lp.HasField("transform_param"):
            raise ValueError(f"{self.type_name} does not transform data.")
        p = self.lp.hdf5_data_param
        with open(p.source) as f:
            self.files = [_resolve_listed(tok, p.source) for tok in f.read().split()]
        if not self.files:
            raise ValueError(f"Must have at least 1 HDF5 filename listed in {p.source}")
        self.batch = int(p.batch_size)
        self.shuffle = bool(p.shuffle)
        self.gen = torch.Generator().manual_seed(int(self.ctx.seed))
        self.file_perm = self._perm(len(self.files))
        self.cur_file = 0
        self._load(self.files[self.file_perm[0]])
        self.row = 0

    def _perm(self, n):
        return torch.randperm(n, generator=self.gen).tolist() if self.shuffle else list(range(n))

    def _load(self, path):
        from ..utils import hdf5
        f = hdf5.File(path)
        self.arrays = []
        for name in self.lp.top:
            a = f[name].read()
            if a.ndim < 1:
                raise ValueError(f"HDF5Data: dataset {name!r} must have at least 1 axis")
            self.arrays.append(torch.from_numpy(a.astype("float32")))
        n = self.arrays[0].shape[0]
        for a in self.arrays[1:]:
            if a.shape[0] != n:
                raise ValueError("HDF5Data: all datasets must have the same number of rows")
        self.data_perm = self._perm(n)

    def reshape(self, bottoms, tops):
        for t, a in zip(tops, self.arrays):
            shape = (self.batch,) + tuple(a.shape[1:])
            t.reshape(shape, self.dtype if len(shape) == 4 else torch.float32)

    def forward(self, bottoms, tops):
        parts = [[] for _ in tops]
        for _ in range(self.batch):
            if self.row == self.arrays[0].shape[0]:
                if len(self.files) > 1:
                    self.cur_file += 1
                    if self.cur_file == len(self.files):
                        self.cur_file = 0
                        if self.shuffle:
                            self.file_perm = self._perm(len(self.files))
                    self._load(self.files[self.file_perm[self.cur_file]])
                self.row = 0
                if self.shuffle:
                    self.data_perm = self._perm(self.arrays[0].shape[0])
            r = self.data_perm[self.row]
            for j in range(len(tops)):
                parts[j].append(self.arrays[j][r])
            self.row += 1
        for t, rows in zip(tops, parts):
            t.set_nchw(torch.stack(rows))

    def backward(self, tops, propagate_down, bottoms):
        pass


@register("HDF5Output")
class HDF5OutputLayer(Layer):
    """hdf5_output_layer.cpp:15-60: writes bottom 0 as ``data`` and bottom 1 as ``label``
    to ``file_name`` on every forward (the file holds the latest batch)."""
    exact_bottoms = 2
    exact_tops = 0

    def layer_setup(self, bottoms, tops):
        self.file_name = self.lp.hdf5_output_param.file_name

    def reshape(self, bottoms, tops):
        if bottoms[0].shape[0] != bottoms[1].shape[0]:
            raise ValueError("data blob and label blob must have the same batch size")

    def forward(self, bottoms, tops):
        from ..utils import hdf5
        arrs = [b.nchw().float().cpu().numpy() for b in bottoms]
        hdf5.write(self.file_name, {"data": arrs[0], "label": arrs[1]})

    def backward(self, tops, propagate_down, bottoms):
        pass
