"""Dense bf16 GEMM ceiling check: our MFMA GEMM (ops.gemm.linear_fwd, tuned tile) against
torch.matmul (hipBLASLt) on the dense equivalents of CaffeNet / VGG conv GEMM shapes
(M = pixels, N = filters, K = taps x channels), x @ w^T with both operands K-contiguous."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm  # noqa: E402

_lib.kernels()
gemm.load_tune_db()


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


SHAPES = [("caffenet conv3 fwd", 43264, 384, 2304), ("caffenet conv2 fwd/g", 186624, 128, 1200),
          ("caffenet conv5 fwd/g", 43264, 128, 1728), ("vgg conv3_2 fwd", 802816, 256, 2304),
          ("vgg conv4_2 fwd", 200704, 512, 4608), ("fc6 fwd b256", 256, 4096, 9216),
          ("square 8192", 8192, 8192, 8192)]
print(f"{'shape':24s} {'M':>7} {'N':>5} {'K':>5}  {'ours us':>8} {'TF/s':>6}  {'blas us':>8} {'TF/s':>6}")
for name, M, N, K in SHAPES:
    x = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.1).to(torch.bfloat16)
    fl = 2.0 * M * N * K
    t_o = timeit(lambda: gemm.linear_fwd(x, w))
    t_b = timeit(lambda: torch.matmul(x, w.t()))
    print(f"{name:24s} {M:7d} {N:5d} {K:5d}  {t_o:8.1f} {fl / t_o / 1e6:6.0f}  {t_b:8.1f} {fl / t_b / 1e6:6.0f}")
    del x, w

# every tile on the large dense shapes (splits = 1)
if os.environ.get("TILE_SWEEP", "1") == "1":
    for name, M, N, K in [("vgg conv4_2 fwd", 200704, 512, 4608), ("square 8192", 8192, 8192, 8192),
                          ("caffenet conv3 fwd", 43264, 384, 2304)]:
        x = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.1).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        row = []
        for t in sorted(gemm.TILES):
            gemm._FORCE_TILE = t
            try:
                row.append(f"{t}:{fl / timeit(lambda: gemm.linear_fwd(x, w), 5) / 1e6:.0f}")
            except Exception as e:  # noqa: BLE001
                row.append(f"{t}:-")
        gemm._FORCE_TILE = -1
        print(name, "TF/s by tile:", " ".join(row))
        del x, w
