import torch
from sparknet_amd.ops import layers_hip as lh, _lib
_lib.kernels()
g = torch.Generator().manual_seed(0)
for shp, C_, inner in [((5, 7), 7, 1), ((2, 6, 5, 3), 3, 1), ((4, 9), 9, 1)]:
    x = torch.randn(shp, generator=g)
    dy = torch.randn(shp, generator=g)
    a = torch.randn(C_, generator=g) * 0.5
    ref_y = torch.where(x > 0, x, x * a)
    ref_dx = dy * torch.where(x > 0, torch.ones_like(x), a)
    xc, dyc, ac = x.cuda().bfloat16(), dy.cuda().bfloat16(), a.cuda()
    y = lh.prelu_fwd(xc, ac, C_, inner)
    dx = lh.prelu_bwd(xc, dyc, ac, C_, inner)
    print(shp, "y err", (y.float().cpu() - ref_y).abs().max().item(), "dx err", (dx.float().cpu() - ref_dx).abs().max().item())
    sd = torch.zeros(C_, device="cuda")
    lh.axis_reduce(lh.RED_PRELU, dyc, xc, 1, x.numel() // C_, C_, inner, out=sd, acc=True)
    print("  slope grad err", (sd.cpu() - (dy * x * (x <= 0)).reshape(-1, C_).sum(0)).abs().max().item())
    print("  dx after reduce err", (dx.float().cpu() - ref_dx).abs().max().item())
