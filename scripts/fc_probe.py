"""Batch-256 InnerProduct GEMMs (CaffeNet fc6 / fc7 / fc8 forward and data gradient) by
tile and split-K factor, against torch.matmul (hipBLASLt).  Times include the split-K
reduce (the whole gemm() call)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sparknet_amd.ops import _lib, gemm  # noqa: E402
from sparknet_amd.ops.gemm import EPI_BF16, Dense  # noqa: E402

_lib.kernels()


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1 << 18)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


B = 256
for name, N, K in [("fc6", 4096, 9216), ("fc7", 4096, 4096), ("fc8", 1000, 4096)]:
    x = (torch.randn(B, K, device="cuda") * 0.1).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.1).to(torch.bfloat16)
    dy = (torch.randn(B, N, device="cuda") * 0.1).to(torch.bfloat16)
    y = torch.empty(B, N, dtype=torch.bfloat16, device="cuda")
    dx = torch.empty(B, K, dtype=torch.bfloat16, device="cuda")
    t_bf = timeit(lambda: torch.matmul(x, w.t()))
    t_bd = timeit(lambda: torch.matmul(dy, w))
    t_of = timeit(lambda: gemm.linear_fwd(x, w, out=y))
    t_od = timeit(lambda: gemm.linear_dgrad(dy, w, out=dx))
    print(f"{name}: fwd blas {t_bf:.1f} us, ours(tuned) {t_of:.1f} | dgrad blas {t_bd:.1f}, ours(tuned) {t_od:.1f}")
    for t in (0, 10, 19, 20, 21, 22):
        rf, rd = [], []
        for s in (1, 2, 4, 8, 16):
            gemm._FORCE_TILE = t
            try:
                rf.append(f"s{s}:{timeit(lambda: gemm.gemm(B, N, K, Dense(x, K, True), Dense(w, K, True), y, N, epi=EPI_BF16, splits=s)):.1f}")
            except Exception:  # noqa: BLE001
                rf.append(f"s{s}:-")
            try:
                rd.append(f"s{s}:{timeit(lambda: gemm.gemm(B, K, N, Dense(dy, N, True), Dense(w, K, False), dx, K, epi=EPI_BF16, splits=s)):.1f}")
            except Exception:  # noqa: BLE001
                rd.append(f"s{s}:-")
        gemm._FORCE_TILE = -1
        print(f"  tile {t:2d} fwd " + " ".join(rf) + " | dgrad " + " ".join(rd))
