"""Host-side DataTransformer (caffe/src/caffe/data_transformer.cpp:17-130) for the Data /
ImageData layers: crop (random in TRAIN, centre in TEST), mirror, mean (file or
per-channel values), scale.  The hot training path uses the fused device kernel
(``csrc/kernels/augment.hip``) instead; this one serves the DB-backed apps and tests.
"""
from __future__ import annotations

import numpy as np
import torch


class DataTransformer:
    def __init__(self, tp, phase: int, seed: int = 0):
        self.scale = float(tp.scale)
        self.mirror = bool(tp.mirror)
        self.crop = int(tp.crop_size)
        self.phase = phase
        self.rng = np.random.default_rng(seed)
        self.mean = None
        if tp.mean_file:
            from .loaders import read_mean_binaryproto
            self.mean = torch.from_numpy(read_mean_binaryproto(tp.mean_file)).float()
        elif len(tp.mean_value):
            self.mean = torch.tensor(list(tp.mean_value), dtype=torch.float32).view(-1, 1, 1)

    def transform_chw(self, x: torch.Tensor) -> torch.Tensor:
        x = x.float()
        C, H, W = x.shape
        if self.mean is not None:
            m = self.mean
            if m.dim() == 3 and m.shape[1] > 1:
                x = x - m[:, :H, :W]
            else:
                m = m.reshape(-1, 1, 1)
                x = x - (m if m.shape[0] == C else m[:1])
        if self.crop:
            if self.phase == 0:
                h0 = int(self.rng.integers(0, H - self.crop + 1))
                w0 = int(self.rng.integers(0, W - self.crop + 1))
            else:
                h0, w0 = (H - self.crop) // 2, (W - self.crop) // 2
            x = x[:, h0:h0 + self.crop, w0:w0 + self.crop]
        if self.mirror and self.phase == 0 and self.rng.integers(0, 2):
            x = x.flip(-1)
        return x * self.scale

    def transform_datum(self, d) -> torch.Tensor:
        from .db import datum_to_array
        return self.transform_chw(torch.from_numpy(datum_to_array(d).copy()))
