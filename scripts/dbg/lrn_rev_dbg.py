"""Where pool_lrn_bwd_rev (gate on) differs from pool_bwd_k3s2 + lrn_across_bwd."""
import torch
from sparknet_amd.ops import hip
from sparknet_amd.ops.spec import PoolSpec

for (N, H, W, C, pad, size) in [(4, 55, 55, 96, 0, 5), (3, 14, 15, 40, 1, 3), (2, 13, 13, 8, 0, 9)]:
    for gate in (False, True):
        s = PoolSpec(N, H, W, C, 3, 3, 2, 2, pad, pad)
        alpha, beta, k = 1e-4 * 50, 0.75, 1.0
        g = torch.Generator().manual_seed(5)
        x = (torch.randn(N, H, W, C, generator=g) * 2.0).to(torch.bfloat16).cuda()
        if gate:
            x = x.clamp_min(0)
        y = hip.lrn_forward(x, size, alpha, beta, k)
        _, mask = hip.pool_forward_mask(y, s, False)
        g = torch.Generator().manual_seed(6)
        dy = (torch.randn(N, s.P, s.Q, C, generator=g) * 2.0).to(torch.bfloat16).cuda()
        dl = hip.pool_backward(dy, y, s, mask)
        dx_ref = hip.lrn_backward(dl, x, size, alpha, beta, k, gate=gate)
        dx_ng = hip.lrn_backward(dl, x, size, alpha, beta, k, gate=False)
        dx = hip.pool_lrn_backward_rev(dy, mask, x, s, size, alpha, beta, k, gate)
        dx0 = hip.pool_lrn_backward_rev(dy, mask, x, s, size, alpha, beta, k, False)
        torch.cuda.synchronize()
        bad = (dx.float() != dx_ref.float()) | (dx.isnan() != dx_ref.isnan())
        bad0 = dx0.float() != dx_ng.float()
        print(f"case {(N, H, W, C, pad, size)} gate {gate}: mismatches {int(bad.sum())} (ungated kernel vs ungated ref {int(bad0.sum())}), "
              f"nan ref {int(dx_ref.isnan().sum())} nan fused {int(dx.isnan().sum())}")
        idx = bad.nonzero()[:8]
        for i in idx.tolist():
            n, h, w, c = i
            print("   ", i, "fused", float(dx[n, h, w, c]), "ref", float(dx_ref[n, h, w, c]), "ungated ref", float(dx_ng[n, h, w, c]),
                  "x", float(x[n, h, w, c]), "dl", float(dl[n, h, w, c]))
