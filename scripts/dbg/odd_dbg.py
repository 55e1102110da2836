import os, sys
sys.path.insert(0, os.getcwd())
import torch
from sparknet_amd.ops import layers_hip as lh, _lib, hip
from sparknet_amd import ops
_lib.kernels()
print("libs", _lib.loaded_libraries())
g = torch.Generator().manual_seed(0)
for shp, C_, inner in [((5, 7), 7, 1), ((2, 6, 5, 3), 3, 1), ((4, 9), 9, 1)]:
    x = torch.randn(shp, generator=g); dy = torch.randn(shp, generator=g); a = torch.randn(C_, generator=g) * 0.5
    ref_dx = dy * torch.where(x > 0, torch.ones_like(x), a)
    xc, dyc, ac = x.cuda().bfloat16(), dy.cuda().bfloat16(), a.cuda()
    dx = lh.prelu_bwd(xc, dyc, ac, C_, inner)
    torch.cuda.synchronize()
    print(shp, "dx err", (dx.float().cpu() - ref_dx).abs().max().item())
    print(" x ", xc.float().cpu().reshape(-1)[:12]); print(" dy", dyc.float().cpu().reshape(-1)[:12]); print(" dx", dx.float().cpu().reshape(-1)[:12]); print(" rf", ref_dx.reshape(-1)[:12])
rng = torch.zeros(2, dtype=torch.int64, device="cuda"); rng[0] = 123
for n in (21, 16, 35, 64):
    x = torch.ones(n, dtype=torch.bfloat16, device="cuda")
    y = hip.dropout_forward(x, 0.5, rng, 1); torch.cuda.synchronize()
    print("dropout", n, sorted(set(y.float().cpu().tolist())), y.float().cpu().tolist())
x = torch.randn(6, 5, generator=g)
y = ops.softmax_forward(x.cuda().bfloat16()); torch.cuda.synchronize()
print("softmax rows5 err", (y.float().cpu() - torch.softmax(x, 1)).abs().max().item())
