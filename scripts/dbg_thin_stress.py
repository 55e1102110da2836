"""Repeat cifar10_quick's conv1 weight gradient (M 32, N 201 with the bias column, K 102400)
on one tile / split-K config many times and compare every result with the fp32 reference
and with the first launch (intermittent-race check for VERDICT r4 weak #3).

python scripts/dbg_thin_stress.py <tile> <splits> [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from sparknet_amd.ops import gemm as G, hip, ref  # noqa: E402
from sparknet_amd.ops.spec import ConvSpec  # noqa: E402

tile, splits = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
G._FORCE_TILE = tile
kchunk = -(-(-(-102400 // splits)) // 64) * 64
G.choose_splits = lambda *a, **k: (-(-102400 // kchunk), kchunk)
dev = torch.device("cuda:0")
s = ConvSpec(100, 32, 32, 8, 32, 5, 5, 1, 1, 2, 2, 1, 1, 1)
g = torch.Generator(device="cpu").manual_seed(0)
x = (torch.randn(100, 32, 32, 8, generator=g) * 40).to(torch.bfloat16)
x[..., 3:] = 0  # the padded input channels of the real net
dy = (torch.randn(100, 32, 32, 32, generator=g) * 1e-3).to(torch.bfloat16)
dy[torch.rand(dy.shape, generator=g) < 0.5] = 0  # ReLU-gated
w = (torch.randn(32, 5, 5, 8, generator=g) * 0.1).to(torch.bfloat16)
dw_r, db_r = torch.zeros(32, 5, 5, 8), torch.zeros(32)
ref.conv_backward(dy.float(), x.float(), w.float(), s, False, dw_r, db_r)
xd, dyd, wd = x.to(dev), dy.to(dev), w.to(dev)
first = None
bad = 0
for i in range(reps):
    dw, db = torch.zeros(32, 5, 5, 8, device=dev), torch.zeros(32, device=dev)
    hip.conv_backward(dyd, xd, wd, s, False, dw, db)
    torch.cuda.synchronize()
    cur = torch.cat([dw.flatten(), db]).cpu()
    if first is None:
        first = cur
        r = torch.cat([dw_r.flatten(), db_r])
        err = ((cur - r).abs().max() / r.abs().max()).item()
        print(f"tile {tile} splits {splits}: rel max err vs fp32 {err:.2e}", flush=True)
    elif not torch.equal(cur, first):
        bad += 1
        d = (cur - first).abs()
        print(f"rep {i}: differs from rep 0, max |d| {d.max().item():.3e} at {int(d.argmax())}", flush=True)
print(f"tile {tile} splits {splits}: {bad} of {reps - 1} repeats differ from the first", flush=True)
