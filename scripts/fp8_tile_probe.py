"""e4m3 forward GEMM tiles (0 = 128x128, 11 = 256x256, 16 = 192x128) against the bf16
engine's best tiles on VGG-16 conv shapes (dense equivalents, M = pixels at batch 256)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm, hip  # noqa: E402

_lib.kernels()


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for name, M, N, K in [("conv2_2", 3211264, 128, 1152), ("conv3_2", 802816, 256, 2304),
                      ("conv4_2", 200704, 512, 4608), ("conv5_2", 50176, 512, 4608)]:
    x = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.1).to(torch.bfloat16)
    sc = hip.Fp8Scales(2, x.device)
    xq, wq = hip.quant_fp8(x, sc.slot(0)), hip.quant_fp8(w, sc.slot(1))
    sc.update()
    xq, wq = hip.quant_fp8(x, sc.slot(0)), hip.quant_fp8(w, sc.slot(1))
    fl = 2.0 * M * N * K
    row = []
    for t in (0, 11, 16):
        gemm._FORCE_TILE = t
        row.append(f"fp8 t{t}:{fl / timeit(lambda: hip.linear_forward_fp8(xq, wq, None, sc.deq(0), sc.deq(1))) / 1e6:.0f}")
        row.append(f"bf16 t{t}:{fl / timeit(lambda: gemm.linear_fwd(x, w)) / 1e6:.0f}")
    gemm._FORCE_TILE = -1
    print(f"{name} M={M} N={N} K={K} TF/s:", " ".join(row), flush=True)
    del x, w, xq, wq
