"""Weight fillers (caffe/include/caffe/filler.hpp:19-295).

Fillers run on the host in the *Caffe* layout of a parameter (fan-in/fan-out are
derived from it exactly as Caffe does: fan_in = count / shape[0], fan_out =
count / shape[1]) using a seeded torch Generator, so initialisation is reproducible
and independent of the internal kernel layout.  The default filler is ``constant 0``
(FillerParameter.type default), which matters for DSL-built nets.
"""
from __future__ import annotations

import math

import torch


def fill(filler, shape, gen: torch.Generator) -> torch.Tensor:
    shape = tuple(shape)
    count = math.prod(shape) if shape else 1
    t = torch.empty(shape, dtype=torch.float32)
    typ = filler.type if filler is not None else "constant"
    if typ == "constant":
        t.fill_(filler.value if filler is not None else 0.0)
    elif typ == "uniform":
        t.uniform_(filler.min, filler.max, generator=gen)
    elif typ == "gaussian":
        t.normal_(filler.mean, filler.std, generator=gen)
        if filler.sparse >= 0:
            num_outputs = shape[0]
            p = filler.sparse / float(num_outputs)
            mask = torch.bernoulli(torch.full(shape, p), generator=gen)
            t.mul_(mask)
    elif typ == "positive_unitball":
        t.uniform_(0, 1, generator=gen)
        num = shape[0]
        t2 = t.view(num, -1)
        t2.div_(t2.sum(dim=1, keepdim=True))
    elif typ in ("xavier", "msra"):
        fan_in = count // shape[0]
        fan_out = count // shape[1] if len(shape) > 1 else count
        vn = filler.variance_norm
        n = {0: fan_in, 1: fan_out, 2: (fan_in + fan_out) / 2.0}[int(vn)]
        if typ == "xavier":
            scale = math.sqrt(3.0 / n)
            t.uniform_(-scale, scale, generator=gen)
        else:
            t.normal_(0.0, math.sqrt(2.0 / n), generator=gen)
    elif typ == "bilinear":
        if len(shape) != 4 or shape[2] != shape[3]:
            raise ValueError("bilinear filler needs a square 4-D blob")
        k = shape[3]
        f = math.ceil(k / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        idx = torch.arange(count)
        x = (idx % k).float()
        y = ((idx // k) % k).float()
        t.view(-1).copy_((1 - (x / f - c).abs()) * (1 - (y / f - c).abs()))
    else:
        raise ValueError(f"Unknown filler type {typ!r}")
    return t
