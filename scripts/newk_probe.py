"""Launch the round-4 kernels at CaffeNet b256 shapes, 5 times each, for rocprofv3 --pmc passes:
the tap-packed conv1 (conv_packed_kernel), the fused pool+LRN forward / backward."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sparknet_amd.ops import hip  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec, PoolSpec  # noqa: E402

s = ConvSpec(256, 57, 57, 48, 96, 3, 3, 1, 1, 0, 0, 1, 1, 1)
assert hip.packed_conv_ok(s)
x = (torch.randn(256, 57, 57, 48, device="cuda")).to(torch.bfloat16)
w = (torch.randn(96, 3, 3, 48, device="cuda") * 0.05).to(torch.bfloat16)
b = torch.randn(96, device="cuda")
for _ in range(5):
    hip.conv_forward(x, w, b, s, relu=True)
ps = PoolSpec(256, 55, 55, 96, 3, 3, 2, 2)
xp = torch.relu(torch.randn(256, 55, 55, 96, device="cuda")).to(torch.bfloat16)
for _ in range(5):
    pooled, mask, y = hip.pool_lrn_forward(xp, ps, False, 5, 1e-4, 0.75, 1.0)
dy = torch.randn_like(y)
for _ in range(5):
    hip.lrn_pool_backward(dy, pooled, mask, ps, 5, 1e-4, 0.75, 1.0)
torch.cuda.synchronize()
print("ok")
