#!/usr/bin/env python3
"""Which fp32 device-mode kernels move the CaffeNet one-step updates away from the fp32 CPU
engine: the test's comparison with the pooling / LRN passes on the HIP fp32 kernels or on the
reference formulas (ops.ref on device tensors)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import test_bench_fidelity_gpu as fid  # noqa: E402
import test_fp32_device_gpu as t32  # noqa: E402
from sparknet_amd.ops import f32dev, ref  # noqa: E402

x, y = fid._data(n=2 * fid.B)
w0 = fid._initial_weights()
uc = fid._one_step_updates(torch.device("cpu"), w0, x, y)
orig = {k: getattr(f32dev, k) for k in ("pool_forward_aux", "pool_backward", "lrn_forward", "lrn_backward")}
ref_pool = {"pool_forward_aux": lambda x, s, gate=False: (ref.pool_forward(x, s), None),
            "pool_backward": lambda dy, x, s, aux=None, y=None, gate=False: ref.pool_backward(dy, x, s, gate)}
ref_lrn = {"lrn_forward": ref.lrn_forward,
           "lrn_backward": lambda dy, x, size, alpha, beta, k, within=False, y=None: ref.lrn_backward(dy, x, size, alpha, beta, k, within)}
for name, patch in (("kernels", {}), ("ref pool", ref_pool), ("ref lrn", ref_lrn), ("ref pool + lrn", {**ref_pool, **ref_lrn})):
    for k, v in orig.items():
        setattr(f32dev, k, patch.get(k, v))
    ug = t32._fp32_gpu_updates(fid, "cuda:0", w0, x, y)
    e = fid._errs(ug, uc)
    print(name, {k: (round(a, 5), round(b, 5)) for k, (a, b) in e.items() if k.startswith(("conv1", "conv2", "fc8"))}, flush=True)
