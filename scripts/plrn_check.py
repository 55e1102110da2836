"""Fused LRN -> pool backward vs the two unfused launches at CaffeNet's production shapes (b256),
for the argmax mask read from global memory (SN_PLRN_MASK_LDS=0) and staged in LDS (=1)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sparknet_amd.ops import hip  # noqa: E402
from sparknet_amd.ops.spec import PoolSpec  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
for name, s in {"pool1/norm1": PoolSpec(N, 55, 55, 96, 3, 3, 2, 2), "pool2/norm2": PoolSpec(N, 27, 27, 256, 3, 3, 2, 2)}.items():
    for gate in (False, True):
        torch.manual_seed(0)
        x = torch.randn(s.N, s.H, s.W, s.C, device="cuda").to(torch.bfloat16)
        if gate:
            x = x.clamp_min(0)
        pooled, mask, y = hip.pool_lrn_forward(x, s, gate, 5, 1e-4, 0.75, 1.0)
        p_ref, m_ref = hip.pool_forward_mask(x, s, gate)
        fwd_ok = torch.equal(pooled, p_ref) and torch.equal(mask, m_ref)
        dy = torch.randn_like(y)
        dp = hip.lrn_backward(dy, p_ref, 5, 1e-4, 0.75, 1.0)
        dx_ref = hip.pool_backward(dp, x, s, m_ref, gate=gate)
        for mlds in ("0", "1"):
            os.environ["SN_PLRN_MASK_LDS"] = mlds
            dx = hip.lrn_pool_backward(dy, pooled, mask, s, 5, 1e-4, 0.75, 1.0)
            bad = (dx != dx_ref)
            nb = int(bad.sum())
            where = ""
            if nb:
                idx = bad.nonzero()[:5].tolist()
                where = f" first {idx}"
            print(f"{name} N={N} gate={gate} fwd_equal={fwd_ok} mask_lds={mlds}: {nb} mismatches of {dx.numel()}{where}",
                  flush=True)
        os.environ.pop("SN_PLRN_MASK_LDS")

# the tile sweep of scripts/plrn_probe.py (which flagged a mismatch once): every (mask_lds, LDS budget, group)
# config against the unfused reference, in one process
if len(sys.argv) > 2 and sys.argv[2] == "sweep":
    s = PoolSpec(N, 27, 27, 256, 3, 3, 2, 2)
    x = torch.relu(torch.randn(s.N, s.H, s.W, s.C, device="cuda")).to(torch.bfloat16)
    pooled, mask, y = hip.pool_lrn_forward(x, s, False, 5, 1e-4, 0.75, 1.0)
    dy = torch.randn_like(y)
    dp = hip.lrn_backward(dy, pooled, 5, 1e-4, 0.75, 1.0)
    dx_ref = hip.pool_backward(dp, x, s, mask)
    for rep in range(2):
        for mlds in ("0", "1"):
            os.environ["SN_PLRN_MASK_LDS"] = mlds
            for cg in (None, 4, 8, 16, 32):
                for b in (32768, 49152, 65536, 98304):
                    os.environ["SN_PLRN_LDS"] = str(b)
                    if cg is None:
                        os.environ.pop("SN_PLRN_CG", None)
                    else:
                        os.environ["SN_PLRN_CG"] = str(cg)
                    try:
                        dx = hip.lrn_pool_backward(dy, pooled, mask, s, 5, 1e-4, 0.75, 1.0)
                    except RuntimeError:
                        continue
                    nb = int((dx != dx_ref).sum())
                    if nb:
                        idx = (dx != dx_ref).nonzero()[:3].tolist()
                        print(f"rep {rep} mask_lds {mlds} cg {cg} budget {b}: {nb} mismatches, first {idx}", flush=True)
    print("sweep done", flush=True)
