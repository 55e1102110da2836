import os, sys
sys.path.insert(0, os.getcwd())
os.environ["SN_GEMM_TUNE_DB"] = "0"; os.environ["SN_GEMM_TUNE_LOG"] = "1"
import torch
from sparknet_amd.ops import _lib, gemm, hip
from sparknet_amd.ops.spec import ConvSpec
_lib.kernels()
s = ConvSpec(int(os.environ.get("PN", "64")), int(os.environ.get("PH", "56")), int(os.environ.get("PH", "56")), int(os.environ.get("PC", "128")), int(os.environ.get("PK", "256")), 3, 3, 1, 1, 1, 1)
x = torch.randn(s.N, s.H, s.W, s.C, device="cuda").to(torch.bfloat16)
w = (torch.randn(s.K, 3, 3, s.C, device="cuda") * 0.05).to(torch.bfloat16)
sc = hip.Fp8Scales(2, x.device)
xq, wq = hip.quant_fp8(x, sc.slot(0)), hip.quant_fp8(w, sc.slot(1))
y = hip.conv_forward_fp8(xq, wq, None, s, sc.deq(0), sc.deq(1))
torch.cuda.synchronize(); print("ok", y.shape)
