import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
import test_layers_gpu as T
from sparknet_amd.ops import layers_hip as lh
orig = lh.prelu_bwd
def wrapped(x, dy, slope, C_, inner):
    out = orig(x, dy, slope, C_, inner)
    torch.cuda.synchronize()
    ref = dy.float() * torch.where(x.float() > 0, torch.ones_like(x.float()), slope.float().reshape(-1))
    print("prelu_bwd args", x.shape, x.dtype, x.stride(), dy.shape, dy.dtype, dy.stride(), slope.shape, slope.dtype, C_, inner,
          "err", (out.float() - ref).abs().max().item(), "x ptr", x.data_ptr() % 256, dy.data_ptr() % 256, out.data_ptr() % 256)
    return out
lh.prelu_bwd = wrapped
for case in ("prelu_2d", "softmax_axis1_3d"):
    txt, bottoms, kw = T.CASES[case]
    try:
        T.run_both(txt, bottoms, **kw); print(case, "OK")
    except AssertionError as e:
        print(case, "FAIL", str(e)[:300])
net = T._net('layer { name: "L" type: "Dropout" bottom: "x" top: "y" dropout_param { dropout_ratio: 0.5 } }', {"x": (3, 7)}, "cuda")
xb = net.blob_by_name("x"); xb.set_nchw(torch.ones(3, 7))
print("x before", xb.data.float().cpu().tolist())
net.forward()
print("x after", net.blob_by_name("x").data.float().cpu().tolist())
print("y", net.blob_by_name("y").data.float().cpu().tolist(), [l.type_name for l in net.layers])
