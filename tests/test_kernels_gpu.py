"""HIP kernels vs the PyTorch fp32 reference (ops.ref) on identical bf16 inputs.

Mirrors the reference's per-layer GPU-vs-CPU tests (caffe/src/caffe/test/test_*_layer.cpp
run over {CPU, GPU} with the CPU as oracle).
"""
import pytest
import torch

from sparknet_amd.ops import ref
from sparknet_amd.ops.spec import POOL_AVE, POOL_MAX, ConvSpec, PoolSpec

pytestmark = pytest.mark.gpu


def rnd(*shape, scale=1.0, dev="cuda"):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def close(a, b, tol=2e-2, what=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err / scale < tol, f"{what}: rel err {err / scale:.3e} (abs {err:.3e}, scale {scale:.3e})"


CONV_CASES = [
    # N, H, W, C, K, R, S, stride, pad, groups
    (2, 13, 13, 16, 32, 3, 3, 1, 1, 1),
    (2, 27, 27, 48, 64, 5, 5, 1, 2, 2),      # AlexNet conv2-like (grouped)
    (2, 35, 35, 3, 16, 11, 11, 4, 0, 1),     # conv1-like (space-to-depth folded path)
    (2, 30, 30, 3, 16, 7, 7, 2, 3, 1),       # GoogLeNet conv1-like (s2d with channel pad 3->4)
    (2, 28, 28, 1, 20, 5, 5, 1, 0, 1),       # LeNet conv1 (explicit im2col path)
    (2, 16, 16, 32, 24, 1, 1, 1, 0, 1),      # 1x1
    (2, 15, 15, 16, 16, 3, 3, 2, 1, 1),      # stride 2 dgrad fallback
    (2, 12, 12, 20, 50, 5, 5, 1, 0, 1),      # LeNet conv2 (odd channels)
    (3, 9, 9, 64, 40, 3, 3, 1, 1, 2),
    (2, 35, 35, 3, 96, 11, 11, 4, 0, 1),     # conv1 with 96 filters: 128x96 tile on the folded input
    (2, 13, 13, 64, 384, 3, 3, 1, 1, 2),     # conv4-like: 192 filters per group -> 128x96 tile
    (3, 7, 7, 32, 288, 3, 3, 1, 1, 1),       # 3 x 96-wide N tiles, ragged M
    (2, 27, 27, 96, 64, 5, 5, 1, 2, 2),      # conv2-like: dgrad has 48 channels per group -> 256x48 tile
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv(gpu, case):
    from sparknet_amd.ops import hip
    N, H, W, Cc, K, R, S, st, pd, g = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    x = rnd(N, H, W, Cc)
    w = rnd(K, R, S, Cc // g, scale=0.2)
    b = torch.randn(K, device="cuda")
    y = hip.conv_forward(x, w, b, s, relu=True)
    close(y, ref.conv_forward(x, w, b, s, relu=True), what="fwd")
    dy = rnd(N, s.P, s.Q, K)
    dw = torch.zeros(K, R, S, Cc // g, device="cuda")
    db = torch.zeros(K, device="cuda")
    dx = hip.conv_backward(dy, x, w, s, True, dw, db)
    dw_r = torch.zeros_like(dw)
    db_r = torch.zeros_like(db)
    dx_r = ref.conv_backward(dy, x, w, s, True, dw_r, db_r)
    close(dx, dx_r, what="dgrad")
    close(dw, dw_r, what="wgrad")
    close(db, db_r, 1e-3, what="bias")


@pytest.mark.parametrize("case", [CONV_CASES[1], CONV_CASES[2], CONV_CASES[4], CONV_CASES[10]])
def test_conv_grad_overwrite(gpu, case):
    """dw_acc / db_acc False (lazily cleared gradients): both are overwritten, including
    the bias gradient produced by the wgrad GEMM's ones column."""
    from sparknet_amd.ops import hip
    N, H, W, Cc, K, R, S, st, pd, g = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    x = rnd(N, H, W, Cc)
    w = rnd(K, R, S, Cc // g, scale=0.2)
    dy = rnd(N, s.P, s.Q, K)
    dw = torch.full((K, R, S, Cc // g), 7.0, device="cuda")
    db = torch.full((K,), 7.0, device="cuda")
    hip.conv_backward(dy, x, w, s, False, dw, db, dw_acc=False, db_acc=False)
    dw_r, db_r = torch.zeros_like(dw), torch.zeros_like(db)
    ref.conv_backward(dy, x, w, s, False, dw_r, db_r)
    close(dw, dw_r, what="wgrad")
    close(db, db_r, 1e-3, what="bias")


def test_flip_batch_matches_single_flips(gpu):
    """One flip_weights_multi launch == the per-layer flip_weights kernel, incl. after a
    re-allocation of an input (descriptor table rebuilt)."""
    from sparknet_amd.ops import _lib, hip
    shapes = [(2, 128, 5, 5, 48), (1, 384, 3, 3, 256), (2, 192, 3, 3, 192), (1, 24, 1, 1, 32)]
    items, refs = [], []
    for G, Kg, R, S, Cg in shapes:
        w = rnd(G * Kg, R, S, Cg)
        wt = torch.empty((G, Cg, R, S, Kg), dtype=torch.bfloat16, device="cuda")
        r = torch.empty_like(wt)
        _lib.call("flip_weights", w, r, G, Kg, R, S, Cg)
        items.append((w, wt, G, Kg, R, S, Cg))
        refs.append(r)
    fb = hip.FlipBatch(items, "cuda")
    fb.run()
    for (_, wt, *_), r in zip(items, refs):
        assert torch.equal(wt, r)
    w2 = rnd(*items[0][0].shape)
    items[0] = (w2,) + items[0][1:]
    fb.items = items
    fb.run()
    r0 = torch.empty_like(refs[0])
    _lib.call("flip_weights", w2, r0, *shapes[0])
    assert torch.equal(items[0][1], r0)


def test_flip_batch_vector_and_scalar_paths(gpu):
    """The 16-byte form of flip_weights_multi (Kg, Cg multiples of 8, aligned tensors; partial
    64 x 64 tiles) and its 2-byte fallback (odd channel counts, a weight view 2 bytes off
    alignment) both equal the per-layer flip_weights kernel."""
    from sparknet_amd.ops import _lib, hip
    shapes = [(1, 72, 3, 3, 40), (2, 8, 5, 5, 136), (1, 20, 3, 3, 12), (1, 64, 3, 3, 64)]
    items, refs = [], []
    for i, (G, Kg, R, S, Cg) in enumerate(shapes):
        n = G * Kg * R * S * Cg
        base = rnd(n + 8)
        w = base[1:n + 1] if i == 3 else base[:n]  # shape 3: misaligned view
        wt = torch.empty((G, Cg, R, S, Kg), dtype=torch.bfloat16, device="cuda")
        r = torch.empty_like(wt)
        _lib.call("flip_weights", w.contiguous(), r, G, Kg, R, S, Cg)
        items.append((w, wt, G, Kg, R, S, Cg))
        refs.append(r)
    hip.FlipBatch(items, "cuda").run()
    for (_, wt, *_), r in zip(items, refs):
        assert torch.equal(wt, r)


@pytest.mark.parametrize("case", [CONV_CASES[0], CONV_CASES[1], CONV_CASES[8]])
def test_conv_dgrad_inplace_weights(gpu, case, monkeypatch):
    """dgrad reading W through the FLIPW operand (no flip pass) == the reference."""
    from sparknet_amd.ops import hip
    monkeypatch.setattr(hip, "DGRAD_INPLACE_WEIGHTS", True)
    N, H, W, Cc, K, R, S, st, pd, g = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    x = rnd(N, H, W, Cc)
    w = rnd(K, R, S, Cc // g, scale=0.2)
    dy = rnd(N, s.P, s.Q, K)
    close(hip.conv_backward(dy, x, w, s, True), ref.conv_backward(dy, x, w, s, True), what="dgrad")


@pytest.mark.parametrize("M,K,N", [(256, 9216, 4096), (64, 800, 500), (100, 64, 10)])
def test_linear(gpu, M, K, N):
    from sparknet_amd.ops import hip
    x, w = rnd(M, K), rnd(N, K, scale=0.05)
    b = torch.randn(N, device="cuda")
    close(hip.linear_forward(x, w, b, True), ref.linear_forward(x, w, b, True))
    dy = rnd(M, N)
    dw, db = torch.zeros(N, K, device="cuda"), torch.zeros(N, device="cuda")
    dwr, dbr = torch.zeros_like(dw), torch.zeros_like(db)
    dx = hip.linear_backward(dy, x, w, True, dw, db)
    dxr = ref.linear_backward(dy, x, w, True, dwr, dbr)
    close(dx, dxr)
    close(dw, dwr)
    close(db, dbr, 1e-3)


@pytest.mark.parametrize("method", [POOL_MAX, POOL_AVE])
@pytest.mark.parametrize("geo", [(2, 55, 55, 96, 3, 2, 0), (2, 32, 32, 32, 3, 2, 0), (2, 8, 8, 24, 3, 2, 1),
                                 (2, 7, 7, 16, 7, 1, 0), (2, 6, 6, 3, 2, 2, 0), (2, 9, 9, 16, 3, 1, 1),
                                 (2, 8, 8, 16, 2, 2, 0), (2, 13, 13, 32, 3, 2, 1), (2, 7, 9, 16, 2, 2, 0),
                                 (2, 8, 8, 16, 2, 2, 1), (2, 14, 14, 64, 5, 3, 0),
                                 (2, 14, 14, 480, 3, 1, 1), (3, 7, 7, 832, 3, 1, 1), (2, 28, 28, 40, 3, 1, 1),
                                 (2, 11, 13, 24, 3, 1, 0), (2, 6, 6, 8, 3, 1, 2)])
def test_pool(gpu, method, geo):
    from sparknet_amd.ops import hip
    N, H, W, Cc, k, st, pd = geo
    s = PoolSpec(N, H, W, Cc, k, k, st, st, pd, pd, method)
    x = rnd(N, H, W, Cc)
    y, mask = hip.pool_forward_mask(x, s)
    close(y, ref.pool_forward(x, s), 1e-2)
    dy = rnd(N, s.P, s.Q, Cc)
    close(hip.pool_backward(dy, x, s, mask), ref.pool_backward(dy, x, s), 1e-2)


@pytest.mark.parametrize("within", [False, True])
@pytest.mark.parametrize("geo", [(2, 13, 13, 96, 5), (2, 8, 8, 256, 5), (2, 6, 6, 20, 3), (2, 5, 5, 16, 9)])
def test_lrn(gpu, within, geo):
    from sparknet_amd.ops import hip
    N, H, W, Cc, size = geo
    x = rnd(N, H, W, Cc, scale=3.0)
    a, bta, k = (5e-5, 0.75, 1.0) if within else (1e-2, 0.75, 2.0)
    y = hip.lrn_forward(x, size, a, bta, k, within)
    close(y, ref.lrn_forward(x, size, a, bta, k, within))
    dy = rnd(N, H, W, Cc)
    close(hip.lrn_backward(dy, x, size, a, bta, k, within), ref.lrn_backward(dy, x, size, a, bta, k, within))
    # fused backward of the in-place ReLU that produced x (GoogLeNet conv2/3x3 -> relu -> norm2)
    xr = torch.relu(x)
    gated = ref.relu_backward(ref.lrn_backward(dy, xr, size, a, bta, k, within), xr)
    close(hip.lrn_backward(dy, xr, size, a, bta, k, within, gate=True), gated)


def test_relu_dropout(gpu):
    from sparknet_amd.ops import hip
    x = rnd(4, 4096)
    close(hip.relu_forward(x, 0.1), ref.relu_forward(x, 0.1), 1e-2)
    dy = rnd(4, 4096)
    close(hip.relu_backward(dy, x, 0.1), ref.relu_backward(dy, x, 0.1), 1e-2)
    rng = torch.tensor([1234567, 42], dtype=torch.int64, device="cuda")
    y = hip.dropout_forward(x, 0.5, rng, 3)
    yr = ref.dropout_forward(x.cpu(), 0.5, 1234567, 42, 3)
    close(y, yr, 1e-2)
    keep = (y != 0).float().mean().item()
    assert 0.45 < keep < 0.55
    # fused ReLU backward: gate = ReLU output (after in-place dropout)
    gate = hip.relu_forward(x, 0.0)
    dx = hip.dropout_backward(dy, 0.5, rng, 3, gate)
    close(dx, ref.dropout_backward(dy.cpu(), 0.5, 1234567, 42, 3, gate.cpu()), 1e-2)


@pytest.mark.parametrize("geo", [(2, 55, 55, 96, 3, 2, 0), (2, 13, 13, 256, 3, 2, 0), (2, 9, 9, 3, 2, 2, 0)])
def test_maxpool_relu_gate(gpu, geo):
    """Max pooling over a ReLU output with the ReLU backward folded into the argmax mask:
    windows whose max is 0 pass no gradient."""
    from sparknet_amd.ops import hip
    N, H, W, Cc, k, st, pd = geo
    s = PoolSpec(N, H, W, Cc, k, k, st, st, pd, pd, POOL_MAX)
    x = torch.relu(rnd(N, H, W, Cc).float() - 0.9).to(torch.bfloat16)  # many all-zero windows
    y, mask = hip.pool_forward_mask(x, s, gate=True)
    close(y, ref.pool_forward(x, s), 1e-2)
    dy = rnd(N, s.P, s.Q, Cc)
    close(hip.pool_backward(dy, x, s, mask, gate=True), ref.pool_backward(dy, x, s, gate=True), 1e-2)
    close(hip.pool_backward(dy, x, s, None, gate=True), ref.pool_backward(dy, x, s, gate=True), 1e-2)


@pytest.mark.parametrize("geo", [(4, 56, 56, 128, 2, 2, 0), (3, 7, 9, 16, 2, 2, 0), (2, 8, 8, 16, 2, 2, 1),
                                 (2, 28, 28, 192, 3, 1, 1), (3, 7, 9, 16, 3, 1, 1), (2, 9, 8, 16, 3, 1, 0),
                                 (2, 6, 6, 16, 3, 1, 2)])
def test_maxpool_k2s2_k3s1_gated_edges(gpu, geo):
    """VGG's 2x2 / stride-2 and GoogLeNet's 3x3 / stride-1 max pools (vectorised fixed-window
    kernels) against the fp32 reference, gated or not, ties (ReLU zeros), ragged and padded
    edges included."""
    from sparknet_amd.ops import hip
    N, H, W, Cc, k, st, pd = geo
    s = PoolSpec(N, H, W, Cc, k, k, st, st, pd, pd, POOL_MAX)
    x = torch.relu(rnd(N, H, W, Cc).float() - 0.5).to(torch.bfloat16)
    dy = rnd(N, s.P, s.Q, Cc)
    for gate in (False, True):
        y, mask = hip.pool_forward_mask(x, s, gate=gate)
        close(y, ref.pool_forward(x, s), 1e-2)
        close(hip.pool_backward(dy, x, s, mask, gate=gate), ref.pool_backward(dy, x, s, gate=gate), 1e-2)


@pytest.mark.parametrize("e5m2", [False, True])
@pytest.mark.parametrize("geo", [(2, 16, 16, 64, 2, 2, 0), (2, 14, 14, 32, 3, 1, 1)])
def test_pool_fp8_side_output(gpu, geo, e5m2):
    """The pooling kernels' fp8 side output (engine.fuse_fp8_quant: a pool's output as the
    next conv's fp8 input, its input gradient as the previous conv's fp8 output gradient)
    is byte-identical to quantising the bf16 result with the same (initialised) slot, and
    its block maxima fold into the slot's amax."""
    from sparknet_amd.ops import gemm as G, hip
    N, H, W, Cc, k, st, pd = geo
    s = PoolSpec(N, H, W, Cc, k, k, st, st, pd, pd, POOL_MAX)
    x = torch.relu(rnd(N, H, W, Cc).float()).to(torch.bfloat16)
    sc = hip.Fp8Scales(2, gpu)
    for i in range(2):
        if e5m2:
            sc.set_e5m2(i)
        sc.slots[i, 0], sc.slots[i, 2], sc.slots[i, 3] = 37.0, 1 / 37.0, 1.0  # initialised slots
    if hip.pool_side_ok(s, False):
        side = G.Fp8Side(torch.empty((N, s.P, s.Q, Cc), dtype=torch.bfloat16, device=gpu), sc.slot(0), e5m2)
        y, mask = hip.pool_forward_mask(x, s, gate=True, side=side)
        assert torch.equal(side.q, hip.quant_fp8(y, sc.slot(1), e5m2=e5m2))
        assert sc.slots[0, 1].item() == y.float().abs().max().item() and side.part.abs().sum().item() == 0
    else:
        y, mask = hip.pool_forward_mask(x, s, gate=True)
    if hip.pool_side_ok(s, True):
        sc.slots[:, 1] = 0
        dy = rnd(N, s.P, s.Q, Cc)
        side = G.Fp8Side(torch.empty((N, H, W, Cc), dtype=torch.bfloat16, device=gpu), sc.slot(0), e5m2)
        dx = hip.pool_backward(dy, x, s, mask, gate=True, side=side)
        close(dx, ref.pool_backward(dy, x, s, gate=True), 1e-2)
        assert torch.equal(side.q, hip.quant_fp8(dx, sc.slot(1), e5m2=e5m2))
        assert sc.slots[0, 1].item() == dx.float().abs().max().item()


@pytest.mark.parametrize("shape", [(2, 20, 37), (3, 16, 16), (1, 56, 56)])
def test_conv3x3_c64_direct(gpu, shape, monkeypatch):
    """The direct 64 -> 64-channel 3x3 conv (csrc/kernels/conv3x3.hip, VGG conv1_2): forward
    with bias + ReLU and the data gradient with the ReLU gate, against the fp32 reference
    and the implicit-GEMM path on the same bf16 inputs."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    N, H, W = shape
    s = ConvSpec(N, H, W, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    assert hip.direct_c64_ok(s)
    x = rnd(N, H, W, 64)
    w = rnd(64, 3, 3, 64, scale=0.1)
    b = torch.randn(64, device="cuda")
    dy = rnd(N, H, W, 64)
    gate = torch.relu(rnd(N, H, W, 64).float()).to(torch.bfloat16)
    y = hip.conv_forward(x, w, b, s, relu=True)
    dx = hip.conv_backward(dy, gate, w, s, True, gate=gate)
    ref = torch.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1))
    close(y, ref.permute(0, 2, 3, 1), 1e-2)
    dref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1)
    close(dx, (dref.permute(0, 2, 3, 1) * (gate.float() > 0)), 1e-2)
    monkeypatch.setattr(hip, "_DIRECT_C64", False)
    y2 = hip.conv_forward(x, w, b, s, relu=True)
    dx2 = hip.conv_backward(dy, gate, w, s, True, gate=gate)
    close(y, y2, 1e-2)
    close(dx, dx2, 1e-2)


@pytest.mark.parametrize("shape", [(2, 57, 57), (1, 20, 35)])
def test_conv3x3_k96_direct(gpu, shape, monkeypatch):
    """The 64-channel direct 3x3 kernel's 48 -> 96-channel, pad-0 instance (CaffeNet conv1
    after the space-to-depth fold, SN_CONV_PACKED=0) with bias + ReLU, against the fp32
    reference and the GEMM path."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    N, H, W = shape
    s = ConvSpec(N, H, W, 48, 96, 3, 3, 1, 1, 0, 0, 1, 1, 1)
    monkeypatch.setattr(hip, "_DIRECT_K96", True)
    monkeypatch.setattr(hip, "_PACKED", False)
    assert hip.direct_conv_ok(s) and not hip.packed_conv_ok(s)
    x = rnd(N, H, W, 48)
    w = rnd(96, 3, 3, 48, scale=0.1)
    b = torch.randn(96, device="cuda")
    y = hip.conv_forward(x, w, b, s, relu=True)
    ref = torch.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b))
    close(y, ref.permute(0, 2, 3, 1), 1e-2)
    monkeypatch.setattr(hip, "_DIRECT_K96", False)
    close(y, hip.conv_forward(x, w, b, s, relu=True), 1e-2)


@pytest.mark.parametrize("N,H,W,C", [(2, 57, 57, 48), (1, 20, 35, 48), (3, 9, 200, 16), (2, 3, 3, 8), (1, 4, 70, 40),
                                     (260, 57, 57, 48)])
@pytest.mark.parametrize("relu,bias", [(True, True), (False, False)])
def test_conv_packed_direct(gpu, N, H, W, C, relu, bias, monkeypatch):
    """The tap-packed direct conv (csrc/kernels/conv_packed.hip: k = tap * C + c, 192-pixel
    row-major tiles; CaffeNet conv1 after the fold is (N, 57, 57, 48)): ragged last tiles,
    a tile spanning many short rows (W = 3), wide rows (W = 200), C < 48 (zero-weight K tail),
    more tiles than CUs (N = 260: the persistent loop's cross-tile patch prefetch), against
    the fp32 reference and, at C = 48, the 64-channel direct kernel."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    monkeypatch.setattr(hip, "_PACKED", True)
    s = ConvSpec(N, H, W, C, 96, 3, 3, 1, 1, 0, 0, 1, 1, 1)
    assert hip.packed_conv_ok(s)
    x = rnd(N, H, W, C)
    w = rnd(96, 3, 3, C, scale=0.1)
    b = torch.randn(96, device="cuda") if bias else None
    y = hip.conv_forward(x, w, b, s, relu=relu)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b)
    if relu:
        ref = torch.relu(ref)
    close(y, ref.permute(0, 2, 3, 1), 1e-2)
    if C == 48:
        monkeypatch.setattr(hip, "_PACKED", False)
        close(y, hip.conv_forward(x, w, b, s, relu=relu), 1e-2)


def test_conv_packed_caffenet_conv1(gpu, monkeypatch):
    """CaffeNet conv1 (227 x 227 x 3, 11 x 11 / 4) through conv_forward: the space-to-depth
    fold feeds the packed kernel; against the fp32 reference of the unfolded conv."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    monkeypatch.setattr(hip, "_PACKED", True)
    s = ConvSpec(4, 227, 227, 3, 96, 11, 11, 4, 4, 0, 0, 1, 1, 1)
    plan = hip.s2d_plan(s)
    assert plan is not None and hip.packed_conv_ok(plan[4])
    x = rnd(4, 227, 227, 3)
    w = rnd(96, 11, 11, 3, scale=0.05)
    b = torch.randn(96, device="cuda")
    y = hip.conv_forward(x, w, b, s, relu=True)
    ref = torch.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, stride=4))
    close(y, ref.permute(0, 2, 3, 1), 1e-2)


@pytest.mark.parametrize("N,H,W,C", [(2, 115, 115, 16), (1, 20, 35, 16), (3, 9, 200, 8), (2, 4, 4, 16),
                                     (8, 115, 115, 16)])
@pytest.mark.parametrize("relu,bias", [(True, True), (False, False)])
def test_conv_packed44_direct(gpu, N, H, W, C, relu, bias, monkeypatch):
    """The tap-packed direct conv's <4 taps, 64 outputs> instance (GoogLeNet conv1 after the
    2x2 fold is (N, 115, 115, 16)): ragged last tiles, a 4 x 4 image (one output pixel), wide rows,
    C = 8 (zero-weight K tail), more tiles than CUs (N = 8: 528 tiles), against the fp32
    reference and the implicit-GEMM path."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    monkeypatch.setattr(hip, "_PACKED44", True)
    s = ConvSpec(N, H, W, C, 64, 4, 4, 1, 1, 0, 0, 1, 1, 1)
    assert hip.packed44_conv_ok(s)
    x = rnd(N, H, W, C)
    w = rnd(64, 4, 4, C, scale=0.1)
    b = torch.randn(64, device="cuda") if bias else None
    y = hip.conv_forward(x, w, b, s, relu=relu)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b)
    if relu:
        ref = torch.relu(ref)
    close(y, ref.permute(0, 2, 3, 1), 1e-2)
    monkeypatch.setattr(hip, "_PACKED44", False)
    close(y, hip.conv_forward(x, w, b, s, relu=relu), 1e-2)


@pytest.mark.parametrize("N,H,W,C,K", [(2, 20, 20, 64, 192), (1, 9, 37, 48, 288), (2, 56, 56, 64, 192),
                                       (3, 5, 5, 16, 192)])
@pytest.mark.parametrize("relu,bias", [(True, True), (False, False)])
def test_conv_direct96_split(gpu, N, H, W, C, K, relu, bias, monkeypatch):
    """3x3 / pad-1 convolutions with <= 64 inputs and a multiple of 96 outputs (GoogLeNet's
    conv2/3x3, 64 -> 192) run as 96-output direct launches into channel slices of the output:
    against the fp32 reference and the implicit-GEMM path."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    monkeypatch.setattr(hip, "_DIRECT96", True)
    s = ConvSpec(N, H, W, C, K, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    assert hip.direct96_split_ok(s)
    x = rnd(N, H, W, C)
    w = rnd(K, 3, 3, C, scale=0.1)
    b = torch.randn(K, device="cuda") if bias else None
    y = hip.conv_forward(x, w, b, s, relu=relu)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1)
    if relu:
        ref = torch.relu(ref)
    close(y, ref.permute(0, 2, 3, 1), 1e-2)
    monkeypatch.setattr(hip, "_DIRECT96", False)
    close(y, hip.conv_forward(x, w, b, s, relu=relu), 1e-2)


@pytest.mark.parametrize("N,H,W,C", [(2, 56, 56, 64), (1, 7, 57, 64), (3, 9, 5, 16), (2, 1, 1, 64)])
@pytest.mark.parametrize("relu,bias", [(True, True), (False, False)])
def test_conv_packed11(gpu, N, H, W, C, relu, bias, monkeypatch):
    """The tap-packed direct kernel's <1 tap, 64 outputs> instance (GoogLeNet conv2/3x3_reduce)
    against the fp32 reference and the implicit GEMM."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    monkeypatch.setattr(hip, "_PACKED11", True)
    s = ConvSpec(N, H, W, C, 64, 1, 1, 1, 1, 0, 0, 1, 1, 1)
    assert hip.packed11_conv_ok(s)
    x = rnd(N, H, W, C)
    w = rnd(64, 1, 1, C, scale=0.1)
    b = torch.randn(64, device="cuda") if bias else None
    y = hip.conv_forward(x, w, b, s, relu=relu)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b)
    if relu:
        ref = torch.relu(ref)
    close(y, ref.permute(0, 2, 3, 1), 1e-2)
    monkeypatch.setattr(hip, "_PACKED11", False)
    close(y, hip.conv_forward(x, w, b, s, relu=relu), 1e-2)


@pytest.mark.parametrize("N,H,W", [(2, 226, 226), (1, 20, 35), (3, 9, 200), (2, 3, 3), (300, 12, 12)])
@pytest.mark.parametrize("relu,bias", [(True, True), (False, False)])
def test_conv_packed3x3k64(gpu, N, H, W, relu, bias, monkeypatch):
    """The tap-packed direct kernel's <3 taps, 64 outputs> instance (VGG-16 conv1_1 after its
    fold is (N, 226, 226, 8)): ragged last tiles, a one-pixel image, wide rows, more tiles than
    CUs, against the fp32 reference and the implicit-GEMM path."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    monkeypatch.setattr(hip, "_PACKED_K64", True)
    s = ConvSpec(N, H, W, 8, 64, 3, 3, 1, 1, 0, 0, 1, 1, 1)
    assert hip.packed3x3k64_ok(s)
    x = rnd(N, H, W, 8)
    w = rnd(64, 3, 3, 8, scale=0.1)
    b = torch.randn(64, device="cuda") if bias else None
    y = hip.conv_forward(x, w, b, s, relu=relu)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b)
    if relu:
        ref = torch.relu(ref)
    close(y, ref.permute(0, 2, 3, 1), 1e-2)
    monkeypatch.setattr(hip, "_PACKED_K64", False)
    close(y, hip.conv_forward(x, w, b, s, relu=relu), 1e-2)


def test_conv_packed3x3k64_vgg_conv1_1(gpu, monkeypatch):
    """VGG-16 conv1_1 (224 x 224 x 3, 3x3, pad 1) through conv_forward: the fold (pad baked in,
    channels padded to 8) feeds the packed <3, 64> kernel; against the fp32 reference."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    monkeypatch.setattr(hip, "_PACKED_K64", True)
    s = ConvSpec(2, 224, 224, 3, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    plan = hip.s2d_plan(s)
    assert plan is not None and hip.packed3x3k64_ok(plan[4])
    x = rnd(2, 224, 224, 3)
    w = rnd(64, 3, 3, 3, scale=0.1)
    b = torch.randn(64, device="cuda")
    y = hip.conv_forward(x, w, b, s, relu=True)
    ref = torch.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1))
    close(y, ref.permute(0, 2, 3, 1), 1e-2)


def test_conv_packed44_googlenet_conv1(gpu, monkeypatch):
    """GoogLeNet conv1 (224 x 224 x 3, 7 x 7 / 2, pad 3) through conv_forward: the 2x2
    space-to-depth fold feeds the packed 4x4 kernel; against the fp32 reference."""
    from sparknet_amd.ops import hip
    import torch.nn.functional as F
    monkeypatch.setattr(hip, "_PACKED44", True)
    s = ConvSpec(2, 224, 224, 3, 64, 7, 7, 2, 2, 3, 3, 1, 1, 1)
    plan = hip.s2d_plan(s)
    assert plan is not None and hip.packed44_conv_ok(plan[4])
    x = rnd(2, 224, 224, 3)
    w = rnd(64, 7, 7, 3, scale=0.05)
    b = torch.randn(64, device="cuda")
    y = hip.conv_forward(x, w, b, s, relu=True)
    ref = torch.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, stride=2, padding=3))
    close(y, ref.permute(0, 2, 3, 1), 1e-2)


def test_softmax_loss_and_accuracy(gpu):
    from sparknet_amd.ops import hip
    x = rnd(256, 1000, scale=2.0)
    lab = torch.randint(0, 1000, (256,), device="cuda").float()
    loss, prob, norm = hip.softmax_loss_forward(x, lab, None, True, 256)
    lr, pr, nr = ref.softmax_loss_forward(x.cpu(), lab.cpu(), None, True, 256)
    assert abs(loss.item() - lr.item()) < 1e-3 * abs(lr.item())
    close(prob, pr, 1e-3)
    lw = torch.tensor([1.0], device="cuda")
    g = hip.softmax_loss_backward(prob, lab, lw, norm)
    gr = ref.softmax_loss_backward(pr, lab.cpu(), 1.0, nr)
    close(g, gr, 1e-2)
    # ignore label path
    lab2 = lab.clone()
    lab2[:10] = 7
    loss2, _, norm2 = hip.softmax_loss_forward(x, lab2, 7, True, 256)
    lr2, _, nr2 = ref.softmax_loss_forward(x.cpu(), lab2.cpu(), 7, True, 256)
    assert abs(loss2.item() - lr2.item()) < 1e-3 * abs(lr2.item())
    assert norm2.item() == nr2.item()
    for k in (1, 5):
        a = hip.accuracy(x, lab, k).item()
        ar = ref.accuracy(x.cpu(), lab.cpu(), k).item()
        assert abs(a - ar) < 1e-6
    close(hip.softmax_forward(x), ref.softmax_forward(x), 1e-2)
    y = hip.softmax_forward(x)
    dy = rnd(256, 1000)
    close(hip.softmax_backward(dy, y), ref.softmax_backward(dy, y), 2e-2)


@pytest.mark.parametrize("kind", range(6))
@pytest.mark.parametrize("l1,clip", [(False, False), (True, True)])
def test_solver_update(gpu, kind, l1, clip):
    from sparknet_amd.ops import hip
    from sparknet_amd.core.solver import N_HYPER
    total = 64 * 41
    segs = [(0, 1000, 1.0, 1.0), (1024, 600, 2.0, 0.0), (1664, 900, 0.5, 3.0)]
    w = torch.randn(total, device="cuda")
    g = torch.randn(total, device="cuda")
    hist = [torch.rand(total, device="cuda") for _ in range(2)]
    hyper = torch.zeros(N_HYPER, device="cuda")
    hyper[:9] = torch.tensor([0.01, 0.9, 5e-4, 5.0 if clip else -1, 0.5, 1e-8, 0.999, 0.98, 0.7])
    tabs = hip.solver_tables(segs, total, "cuda")
    wr, gr, hr = w.cpu().clone(), g.cpu().clone(), [h.cpu().clone() for h in hist]
    lr = torch.zeros(total)
    dc = torch.zeros(total)
    for off, cnt, lm, dm in segs:
        padded = -(-cnt // 64) * 64
        lr[off:off + padded] = lm
        dc[off:off + padded] = dm
    shadow = torch.empty(total, dtype=torch.bfloat16, device="cuda")
    hip.solver_update(kind, w, g, hist, shadow, tabs, hyper, l1, clip)
    ref.solver_update_ref(kind, wr, gr, hr, lr, dc, hyper.cpu().tolist(), l1, clip)
    close(w, wr, 1e-5)
    close(hist[0], hr[0], 1e-4)
    close(shadow, wr, 1e-2)


def test_cast_and_augment(gpu):
    from sparknet_amd.ops import hip
    src = torch.randn(1003, device="cuda")
    dst = torch.empty(1003, dtype=torch.bfloat16, device="cuda")
    hip.cast_f32_to_bf16(src, dst)
    assert torch.equal(dst, src.to(torch.bfloat16))
    img = torch.randint(0, 256, (4, 3, 40, 44), dtype=torch.uint8, device="cuda")
    mean = torch.tensor([100.0, 110.0, 120.0], device="cuda")
    out = torch.empty((4, 32, 32, 3), dtype=torch.bfloat16, device="cuda")
    offs = torch.zeros((4, 3), dtype=torch.int32, device="cuda")
    rng = torch.tensor([7, 3], dtype=torch.int64, device="cuda")
    hip.augment(img, out, 32, mean, 1, 0.5, rng, True, True, offs)
    for n in range(4):
        ho, wo, mir = offs[n].tolist()
        crop = img[n, :, ho:ho + 32, wo:wo + 32].float()
        if mir:
            crop = crop.flip(-1)
        expect = ((crop - mean.view(3, 1, 1)) * 0.5).permute(1, 2, 0)
        close(out[n], expect, 1e-2)


@pytest.mark.parametrize("src_hw", [(40, 44), (39, 41), (256, 256)])
@pytest.mark.parametrize("mean_mode", [1, 2])
@pytest.mark.parametrize("ksp", [(11, 4, 0), (11, 4, 2), (7, 2, 3), (3, 1, 1)])
def test_augment_s2d_equals_augment_then_fold(gpu, mean_mode, ksp, src_hw, monkeypatch):
    """The fused augment + space-to-depth kernel (row-tiled LDS path and the per-pixel
    path) is bitwise the two-pass result; odd source widths take the byte-load staging, and
    the 4 x 4 RGB fold's 32-bit-load path (any byte alignment, mirrored or not, padded or
    not) matches too — at CaffeNet's 256 -> 227 crop as well."""
    from sparknet_amd.ops import hip
    N, crop = 3, 35
    Hs, Ws = src_hw
    if Hs == 256:
        N, crop = 4, 227
    img = torch.randint(0, 256, (N, 3, Hs, Ws), dtype=torch.uint8, device="cuda")
    mean = (torch.rand(3, device="cuda") * 200) if mean_mode == 1 else (torch.rand(3, Hs, Ws, device="cuda") * 200)
    rng = torch.tensor([11, 5], dtype=torch.int64, device="cuda")
    k, st, pd = ksp
    s = ConvSpec(N, crop, crop, 3, 16, k, k, st, st, pd, pd)
    plan = hip.s2d_plan(s)
    assert plan is not None
    nhwc = torch.empty((N, crop, crop, 3), dtype=torch.bfloat16, device="cuda")
    hip.augment(img, nhwc, crop, mean, mean_mode, 0.25, rng, True, True)
    ref2 = hip._s2d_input(nhwc, s, plan)
    x2 = torch.empty_like(ref2)
    hip.augment_s2d(img, x2, crop, plan, s, mean, mean_mode, 0.25, rng, True, True)
    assert torch.equal(x2, ref2)
    x3 = torch.full_like(ref2, 7.0)
    labs = [4, 0, 9, 2][:N]
    lab = torch.tensor(labs, dtype=torch.int32, device="cuda")
    lab_out = torch.full((N, 1), -1.0, device="cuda")
    hip.augment_s2d(img, x3, crop, plan, s, mean, mean_mode, 0.25, rng, True, True, lab, lab_out)
    assert torch.equal(x3, ref2) and lab_out.flatten().tolist() == [float(v) for v in labs]


@pytest.mark.parametrize("k", [2, 3, 8, 11])
def test_sum_bf16(gpu, k):
    from sparknet_amd.ops import hip
    xs = [rnd(3, 5, 8) for _ in range(k)]
    close(hip.sum_bf16(xs), sum(x.float() for x in xs), 1e-2)


def test_concat_channels_fwd_bwd_gate(gpu):
    """NHWC channel concat (one launch) and its backward with per-part ReLU masks and a
    skipped part, against torch.cat / narrow."""
    from sparknet_amd.ops import hip
    chans = [64, 24, 128, 8]
    parts = [rnd(3, 7, 9, c) for c in chans]
    out = torch.empty(3, 7, 9, sum(chans), dtype=torch.bfloat16, device=gpu)
    hip.concat_channels(parts, out)
    assert torch.equal(out, torch.cat(parts, dim=-1))
    dy = rnd(3, 7, 9, sum(chans))
    parts[1][0, 0, 0, :4] = 0.0  # exact zeros: masked like relu_bwd (x > 0 fails)
    diffs = [torch.empty_like(p) for p in parts]
    diffs[2] = None
    gates = [parts[0], parts[1], None, parts[3]]
    hip.concat_channels_bwd(dy, diffs, gates, chans)
    off = 0
    for i, c in enumerate(chans):
        want = dy[..., off:off + c]
        if gates[i] is not None:
            want = want * (parts[i] > 0).to(want.dtype)
        if diffs[i] is not None:
            assert torch.equal(diffs[i], want), i
        off += c


def test_conv_image_chunking(gpu, monkeypatch):
    """Convolutions over more than 2^24 pixels per launch run as image chunks (forward /
    dgrad slices, accumulated weight gradients): forced small chunk limit vs one launch."""
    from sparknet_amd.ops import hip
    from sparknet_amd.ops.spec import ConvSpec
    s = ConvSpec(6, 20, 20, 16, 32, 3, 3, 1, 1, 1, 1)
    x = rnd(6, 20, 20, 16)
    w = rnd(32, 3, 3, 16, scale=0.1)
    b = torch.randn(32, device="cuda")
    dy = rnd(6, 20, 20, 32)
    y0 = hip.conv_forward(x, w, b, s, relu=True)
    dw0, db0 = torch.zeros(32, 3, 3, 16, device="cuda"), torch.zeros(32, device="cuda")
    dx0 = hip.conv_backward(dy, x, w, s, True, dw0, db0)
    monkeypatch.setattr(hip, "_MAX_PIX", 2 * 20 * 20 + 1)  # 2 images per launch
    assert hip._image_chunk(s) == 2
    y1 = hip.conv_forward(x, w, b, s, relu=True)
    dw1, db1 = torch.zeros_like(dw0), torch.zeros_like(db0)
    dx1 = hip.conv_backward(dy, x, w, s, True, dw1, db1)
    assert torch.equal(y0, y1) and torch.equal(dx0, dx1)
    close(dw1, dw0, 1e-3)
    close(db1, db0, 1e-3)
