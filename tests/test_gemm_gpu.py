"""Numerics of the MFMA GEMM against an fp32 PyTorch reference (all layouts)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(*shape, device):
    return (torch.randn(*shape, device=device) * 0.5).to(torch.bfloat16)


def _close(a, b, tol=8e-3):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err / scale < tol, f"rel err {err/scale:.3e}"


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 4096, 1024), (100, 70, 200), (77, 96, 363 + 5), (1000, 10, 64),
                                   (600, 48, 200)])
def test_linear_fwd(gpu, M, N, K):
    from sparknet_amd.ops import gemm
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    b = torch.randn(N, device=gpu)
    y = gemm.linear_fwd(x, w, b, relu=True)
    ref = torch.relu(x.float() @ w.float().t() + b)
    _close(y, ref)


@pytest.mark.parametrize("n", [128, 96, 192])
def test_identity_asymmetric(gpu, n):
    # A = I with an asymmetric B catches transposed C writes (96/192: the 128x96 tile).
    from sparknet_amd.ops import gemm
    eye = torch.eye(n, device=gpu).to(torch.bfloat16)
    w = (torch.arange(n * n, device=gpu).reshape(n, n) % 17).to(torch.bfloat16)
    y = gemm.linear_fwd(eye, w)
    assert torch.equal(y.float(), w.float().t())


@pytest.mark.parametrize("M,N,K", [(256, 4096, 9216), (64, 10, 500), (128, 200, 136), (300, 200, 40), (700, 64, 48)])
def test_linear_dgrad(gpu, M, N, K):
    from sparknet_amd.ops import gemm
    dy, w = _bf(M, N, device=gpu), _bf(N, K, device=gpu)
    dx = gemm.linear_dgrad(dy, w)
    _close(dx, dy.float() @ w.float())


@pytest.mark.parametrize("M,N,K", [(256, 4096, 9216), (64, 10, 500), (300, 24, 136), (100, 300, 48), (512, 320, 56)])
def test_linear_wgrad(gpu, M, N, K):
    from sparknet_amd.ops import gemm
    dy, x = _bf(M, N, device=gpu), _bf(M, K, device=gpu)
    dw = torch.ones(N, K, device=gpu)
    gemm.linear_wgrad(dy, x, dw, accumulate=True)
    _close(dw, 1 + dy.float().t() @ x.float())


@pytest.mark.parametrize("M,N", [(5000, 96), (256, 4096), (256, 1000), (77, 13), (3000, 700), (100000, 48)])
def test_colsum(gpu, M, N):
    from sparknet_amd.ops import gemm
    x = _bf(M, N, device=gpu)
    out = torch.ones(N, device=gpu)
    gemm.colsum(x, out)
    _close(out, 1 + x.float().sum(0), 1e-3)
    gemm.colsum(x, out, accumulate=False)
    _close(out, x.float().sum(0), 1e-3)


@pytest.mark.parametrize("splits", [1, 3, 16, 100])
def test_forced_splitk_epilogues(gpu, splits):
    """Split-K through both reduce kernels with every epilogue (bias, ReLU, gate, fp32
    store / accumulate) against the unsplit fp32 product."""
    from sparknet_amd.ops import gemm as G
    M, N, K = 96, 200, 64 * 110
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    b = torch.randn(N, device=gpu)
    gate = _bf(M, N, device=gpu)
    ref = x.float() @ w.float().t()
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    G.gemm(M, N, K, G.Dense(x, K, True), G.Dense(w, K, True), y, N, epi=G.EPI_BF16, bias=b, relu=True,
           splits=splits, gate=gate)
    _close(y, torch.relu(ref + b) * (gate.float() > 0))
    acc = torch.ones(M, N, device=gpu)
    G.gemm(M, N, K, G.Dense(x, K, True), G.Dense(w, K, True), acc, N, epi=G.EPI_F32_ACC, splits=splits)
    _close(acc, 1 + ref)


@pytest.mark.parametrize("splits", [1, 2, 20])
@pytest.mark.parametrize("acc", [True, False])
@pytest.mark.parametrize("M,N,K", [(96, 432, 64 * 40), (200, 64, 1000), (48, 1200, 333)])
def test_wgrad_bias_column(gpu, splits, acc, M, N, K):
    """Weight-gradient TN product with the virtual ones column: dw = A^T-sum and the bias
    gradient (row sums of A) from one GEMM, unsplit and through both reduce kernels."""
    from sparknet_amd.ops import gemm as G
    a, b = _bf(K, M, device=gpu), _bf(K, N, device=gpu)  # A: [K][M] (MC), B: [K][N] (MC)
    dw = torch.full((M, N), 3.0, device=gpu)
    db = torch.full((M,), -2.0, device=gpu)
    G.gemm(M, N, K, G.Dense(a, M, False), G.Dense(b, N, False), dw, N, epi=G.EPI_F32_ACC if acc else G.EPI_F32,
           splits=splits, bias_grad=db, bias_acc=acc)
    base = 3.0 if acc else 0.0
    _close(dw, base + a.float().t() @ b.float(), 1e-2)
    _close(db, (-2.0 if acc else 0.0) + a.float().sum(0), 1e-3)


def test_linear_dgrad_gate(gpu):
    from sparknet_amd.ops import gemm
    dy, w = _bf(256, 512, device=gpu), _bf(512, 384, device=gpu)
    gate = _bf(256, 384, device=gpu)
    dx = gemm.linear_dgrad(dy, w, gate=gate)
    _close(dx, (dy.float() @ w.float()) * (gate.float() > 0))


def _f8(t):
    """bf16/float tensor -> (e4m3 bytes as uint8, dequantised float) via torch's OCP e4m3."""
    q = t.float().clamp(-448, 448).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), q.float()


def test_quant_fp8_matches_torch(gpu):
    from sparknet_amd.ops import hip
    x = (torch.randn(64, 48, device=gpu) * 3).to(torch.bfloat16)
    sc = hip.Fp8Scales(1, gpu)
    sc.slots[0, 0] = 20.0
    sc.slots[0, 3] = 1.0  # an initialised slot: its scale is used as is
    q = hip.quant_fp8(x, sc.slot(0))
    ref, _ = _f8(x.float() * 20.0)
    mism = (q != ref).float().mean().item()
    assert mism < 1e-3, mism  # identical rounding (RNE) up to rare ties
    assert abs(sc.slots[0, 1].item() - x.float().abs().max().item()) < 1e-6
    sc.update()
    assert abs(sc.slots[0, 0].item() - 448.0 / x.float().abs().max().item()) < 1e-3
    assert sc.slots[0, 1].item() == 0.0
    assert sc.slots[0, 3].item() == 1.0


def test_quant_fp8_uninitialised_slot_uses_current_amax(gpu):
    """A slot that fp8_update_scales has not initialised yet quantises with the CURRENT
    tensor's scale (448 / amax), and its dequantisation factor says so — small gradients
    are not flushed to zero by the unit default scale on the first iteration."""
    from sparknet_amd.ops import hip
    x = (torch.randn(4096, 64, device=gpu) * 1e-5).to(torch.bfloat16)
    sc = hip.Fp8Scales(1, gpu)
    q = hip.quant_fp8(x, sc.slot(0))
    amax = x.float().abs().max().item()
    s = 448.0 / amax
    assert abs(sc.slots[0, 0].item() / s - 1) < 1e-5 and abs(sc.slots[0, 2].item() * s - 1) < 1e-5
    ref, _ = _f8(x.float() * s)
    assert (q != ref).float().mean().item() < 1e-3
    deq = q.view(torch.float8_e4m3fn).float() * sc.slots[0, 2].item()
    assert ((deq - x.float()).abs().max() / amax).item() < 0.07
    # a second quantisation before the update keeps the same scale (image chunks share a slot)
    sc.slots[0, 0] = 123.0
    hip.quant_fp8(x, sc.slot(0))
    assert abs(sc.slots[0, 0].item() / s - 1) < 1e-5
    sc.update()
    assert sc.slots[0, 3].item() == 1.0 and abs(sc.slots[0, 0].item() / s - 1) < 1e-3


FP8_TILES = [0, 11, 16]  # 128x128, and the large tiles of gemm_fp8big.hip


@pytest.mark.parametrize("tile", FP8_TILES)
@pytest.mark.parametrize("M,N,K", [(256, 256, 512), (300, 200, 384), (128, 1000, 4096 + 128)])
def test_fp8_dense_gemm(gpu, M, N, K, tile, monkeypatch):
    """e4m3 x e4m3 -> fp32 on the scaled MFMA: exact products of representable values."""
    from sparknet_amd.ops import gemm as G, hip
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    aq, af = _f8(torch.randn(M, K, device=gpu) * 8)
    bq, bf = _f8(torch.randn(N, K, device=gpu) * 8)
    da = torch.tensor([0.125], device=gpu)
    db = torch.tensor([0.25], device=gpu)
    bias = torch.randn(N, device=gpu)
    y = hip.linear_forward_fp8(aq, bq, bias, da, db, relu=True)
    ref = torch.relu(af @ bf.t() * (0.125 * 0.25) + bias)
    _close(y, ref, 1e-2)


@pytest.mark.parametrize("tile", FP8_TILES)
@pytest.mark.parametrize("case", [(2, 13, 13, 32, 48, 3, 3, 1, 1, 1), (2, 9, 9, 64, 32, 3, 3, 1, 1, 2),
                                  (2, 14, 14, 256, 128, 3, 3, 1, 1, 1), (3, 20, 20, 128, 320, 3, 3, 1, 1, 1)])
def test_fp8_conv_forward(gpu, case, tile, monkeypatch):
    from sparknet_amd.ops import gemm as G, hip
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    from sparknet_amd.ops.spec import ConvSpec
    import torch.nn.functional as F
    N, H, W, Cc, K, R, S, st, pd, g = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    xq, xf = _f8(torch.randn(N, H, W, Cc, device=gpu) * 4)
    wq, wf = _f8(torch.randn(K, R, S, Cc // g, device=gpu) * 4)
    dx, dw = torch.tensor([0.5], device=gpu), torch.tensor([0.0625], device=gpu)
    y = hip.conv_forward_fp8(xq, wq, None, s, dx, dw)
    ref = F.conv2d(xf.permute(0, 3, 1, 2), wf.permute(0, 3, 1, 2), stride=st, padding=pd, groups=g) * (0.5 * 0.0625)
    _close(y.permute(0, 3, 1, 2), ref, 1e-2)



@pytest.mark.parametrize("fmt,tile", [("e4m3", -1), ("e5m2", 0), ("e5m2", 11), ("e5m2", 16)])
@pytest.mark.parametrize("case", [(2, 14, 14, 64, 128, 1, False), (2, 9, 9, 96, 64, 2, True),
                                  (3, 20, 20, 128, 256, 1, True)])
def test_fp8_conv_dgrad(gpu, case, fmt, tile, monkeypatch):
    """fp8 data gradient of a stride-1 3x3 conv (ops.hip._conv_dgrad_fp8: e4m3 / e5m2 output
    gradient x e4m3 flip-transposed weights, dequantised + ReLU-gated epilogue) against
    the fp32 reference; the bf16 path on the same inputs sets the scale of the error."""
    from sparknet_amd.ops import gemm as G, hip
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    import torch.nn.functional as F
    N, H, W, Cc, K, g, gated = case
    s = ConvSpec(N, H, W, Cc, K, 3, 3, 1, 1, 1, 1, 1, 1, g)
    gen = torch.Generator(device=gpu).manual_seed(3)
    x = torch.randn(N, H, W, Cc, device=gpu, generator=gen).to(torch.bfloat16)
    w = (torch.randn(K, 3, 3, Cc // g, device=gpu, generator=gen) * 0.05).to(torch.bfloat16)
    dy = (torch.randn(N, H, W, K, device=gpu, generator=gen) * 1e-4).to(torch.bfloat16)
    gate = x if gated else None
    sc = hip.Fp8Scales(2, gpu)
    if fmt == "e5m2":
        sc.set_e5m2(0)
    assert hip.fp8_dgrad_ok(s)
    dx8 = hip.conv_backward(dy, x, w, s, True, ws={"fp8_dgrad": (sc, 0, 1)}, gate=gate)
    dxb = hip.conv_backward(dy, x, w, s, True, gate=gate)
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1,
                             groups=g).permute(0, 2, 3, 1)
    if gated:
        ref = ref * (x.float() > 0)
    err8 = ((dx8.float() - ref).norm() / ref.norm()).item()
    errb = ((dxb.float() - ref).norm() / ref.norm()).item()
    # e4m3: 3 mantissa bits on both operands; e5m2 gradients: 2 bits (rms rounding ~3.6 %)
    assert err8 < (0.05 if fmt == "e4m3" else 0.08), (err8, errb)
    assert errb < 0.01
    fmax = 448.0 if fmt == "e4m3" else 57344.0
    assert abs(sc.slots[0, 2].item() * fmax / dy.float().abs().max().item() - 1) < 1e-3  # current scaling on first use
    if gated:
        assert torch.all(dx8[x <= 0] == 0)


# --- gemm256_kernel (tiles 6 = 256x256, 7 = 256x128), the 8-wave 2-stage gemm_kernel
# tiles (11 = 256x256, 12 / 13 = 256x128, 14 = 256x192, K-contiguous B only), the 3-stage
# 4-wave tiles (19, 20: dense only): every operand
# layout, ragged edges, short and long K (the phased DMA pipeline issues zero-page DMAs past
# the last K-step), split-K, the bias-gradient column and the implicit-GEMM convolutions
BIG_TILES = [6, 7, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20]
MC_B = {6, 7, 11, 12, 13}  # tiles with MC (k-strided) A and B operand instances


@pytest.mark.parametrize("tile", BIG_TILES)
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 200, 136), (1000, 384, 2304), (513, 129, 1000), (64, 48, 40)])
def test_gemm256_layouts(gpu, tile, M, N, K, monkeypatch):
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    b = torch.randn(N, device=gpu)
    _close(G.linear_fwd(x, w, b, relu=True), torch.relu(x.float() @ w.float().t() + b))
    dy = _bf(M, N, device=gpu)
    w2 = _bf(N, K, device=gpu)
    if tile in MC_B or tile in (16, 18, 19, 20):  # NN: MC B operand (192-row tiles: MC A excluded)
        _close(G.linear_dgrad(dy, w2), dy.float() @ w2.float())
    if tile not in MC_B:
        return
    dw = torch.ones(N, K, device=gpu)
    G.linear_wgrad(dy, x, dw, accumulate=True)
    _close(dw, 1 + dy.float().t() @ x.float())


@pytest.mark.parametrize("tile", sorted(MC_B))
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm256_bias_column_and_splitk(gpu, tile, splits, monkeypatch):
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    M, N, K = 96, 432, 64 * 40 + 17
    a, bm = _bf(K, M, device=gpu), _bf(K, N, device=gpu)
    dw = torch.full((M, N), 3.0, device=gpu)
    db = torch.full((M,), -2.0, device=gpu)
    G.gemm(M, N, K, G.Dense(a, M, False), G.Dense(bm, N, False), dw, N, epi=G.EPI_F32_ACC, splits=splits,
           bias_grad=db, bias_acc=True)
    _close(dw, 3.0 + a.float().t() @ bm.float(), 1e-2)
    _close(db, -2.0 + a.float().sum(0), 1e-3)
    x, w = _bf(M * 3, K, device=gpu), _bf(N, K, device=gpu)
    y = torch.empty(M * 3, N, device=gpu, dtype=torch.bfloat16)
    gate = _bf(M * 3, N, device=gpu)
    G.gemm(M * 3, N, K, G.Dense(_pad(x), 64 * 41, True), G.Dense(_pad(w), 64 * 41, True), y, N, epi=G.EPI_BF16,
           splits=splits, gate=gate)
    _close(y, (x.float() @ w.float().t()) * (gate.float() > 0))


def _pad(t):
    out = torch.zeros(t.shape[0], 64 * 41, dtype=t.dtype, device=t.device)
    out[:, :t.shape[1]] = t
    return out


@pytest.mark.parametrize("tile", BIG_TILES)
@pytest.mark.parametrize("case", [(2, 13, 13, 64, 384, 3, 3, 1, 1, 1), (2, 27, 27, 96, 256, 5, 5, 1, 2, 2),
                                  (4, 14, 14, 32, 128, 1, 1, 1, 0, 1), (3, 9, 9, 64, 40, 3, 3, 1, 1, 2),
                                  (2, 7, 7, 192, 96, 3, 3, 1, 1, 2), (2, 9, 9, 24, 32, 2, 2, 1, 0, 1),
                                  (2, 11, 11, 40, 48, 3, 3, 1, 1, 1)])
def test_gemm256_conv(gpu, tile, case, monkeypatch):
    from sparknet_amd.ops import gemm as G, hip, ref
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    if tile in (19, 20):
        pytest.skip("3-stage 4-wave tiles: dense operands only")
    N, H, W, Cc, K, R, S, st, pd, g = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    x = _bf(N, H, W, Cc, device=gpu)
    w = (torch.randn(K, R, S, Cc // g, device=gpu) * 0.1).to(torch.bfloat16)
    bias = torch.randn(K, device=gpu)
    _close(hip.conv_forward(x, w, bias, s, relu=True), ref.conv_forward(x, w, bias, s, relu=True))
    if tile not in MC_B:  # forward only; the dgrad / wgrad products need MC B instances
        return
    dy = _bf(N, s.P, s.Q, K, device=gpu)
    dw, db = torch.zeros(K, R, S, Cc // g, device=gpu), torch.zeros(K, device=gpu)
    dw_r, db_r = torch.zeros_like(dw), torch.zeros_like(db)
    dx = hip.conv_backward(dy, x, w, s, True, dw, db)
    dx_r = ref.conv_backward(dy, x, w, s, True, dw_r, db_r)
    _close(dx, dx_r)
    _close(dw, dw_r)
    _close(db, db_r, 1e-3)


@pytest.mark.parametrize("nesterov", [False, True])
@pytest.mark.parametrize("B,O,I", [(256, 384, 512), (64, 200, 264), (128, 1000, 1024)])
def test_linear_wgrad_sgd_epilogue(gpu, nesterov, B, O, I):
    """EPI_SGD: the InnerProduct weight gradient consumed by the momentum update in the
    GEMM epilogue (interior 128x128 tiles go through the LDS-transposed path, ragged
    tiles and the bias column through the per-fragment path) == fp32 reference update."""
    from sparknet_amd.ops import gemm as G
    dy = (torch.randn(B, O, device=gpu) * 0.1).to(torch.bfloat16)
    x = _bf(B, I, device=gpu)
    w0 = torch.randn(O, I, device=gpu) * 0.05
    h0 = torch.randn(O, I, device=gpu) * 0.01
    w, h = w0.clone(), h0.clone()
    sh = torch.zeros(O, I, dtype=torch.bfloat16, device=gpu)
    lr, mom, wd = 0.01, 0.9, 5e-4
    hyper = torch.tensor([lr, mom, wd, 0.0, 1.0, 0, 0, 0], dtype=torch.float32, device=gpu)
    db = torch.zeros(O, device=gpu)
    sgd = dict(w=w, h=h, shadow=sh, hyper=hyper, lr_mult=1.0, decay_mult=1.0, flags=1 if nesterov else 0)
    assert G.linear_wgrad_sgd(dy, x, sgd, db, db_acc=False)
    g = dy.float().t() @ x.float() + wd * w0
    h_ref = mom * h0 + lr * g
    w_ref = w0 - ((1 + mom) * h_ref - mom * h0 if nesterov else h_ref)
    _close(h, h_ref, 1e-3)
    _close(w - w0, w_ref - w0, 1e-3)
    assert torch.equal(sh, w.to(torch.bfloat16))
    _close(db, dy.float().sum(0), 1e-3)


@pytest.mark.parametrize("M,N,K", [(304, 64, 640), (1000, 200, 136), (128, 64, 64)])
def test_tile64_layouts(gpu, M, N, K, monkeypatch):
    """The 128x64 tile (three blocks per CU): NT / TN dense products and a conv forward
    + weight gradient against the fp32 reference."""
    from sparknet_amd.ops import gemm as G, hip
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(G, "_FORCE_TILE", 10)
    a, b = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    bias = torch.randn(N, device=gpu)
    c = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    G.gemm(M, N, K, G.Dense(a, K, True), G.Dense(b, K, True), c, N, epi=G.EPI_BF16, bias=bias, relu=True)
    _close(c, torch.relu(a.float() @ b.float().t() + bias))
    at, bt = _bf(K, M, device=gpu), _bf(K, N, device=gpu)
    dw = torch.full((M, N), 1.0, device=gpu)
    G.gemm(M, N, K, G.Dense(at, M, False), G.Dense(bt, N, False), dw, N, epi=G.EPI_F32_ACC, splits=2)
    _close(dw, 1.0 + at.float().t() @ bt.float(), 1e-2)
    s = ConvSpec(4, 12, 12, 32, 64, 3, 3, 1, 1, 1, 1)
    x = _bf(4, 12, 12, 32, device=gpu)
    w = (torch.randn(64, 3, 3, 32, device=gpu) * 0.1).to(torch.bfloat16)
    y = hip.conv_forward(x, w, None, s)
    from sparknet_amd.ops import ref
    _close(y, ref.conv_forward(x.float().cpu(), w.float().cpu(), None, s).to(gpu))


# MC im2col stager (weight gradients): per-lane pixel state advanced BKE pixels per K-step
# with one q and one p carry (gemm_impl.h GStager).  Geometries that exercise every carry
# pattern: several images per K-step (P*Q < 64), a 1x1 output, stride 2 + padding, dilation,
# 5x5 taps over 48-channel groups, a pixel count that is not a multiple of 64, and split-K
# slices starting mid-image (the state is decoded per slice at its first row).
@pytest.mark.parametrize("tile", [0, 10, 1, 13, 6])
@pytest.mark.parametrize("splits", [1, 3, 7])
@pytest.mark.parametrize("case", [(5, 13, 13, 64, 96, 3, 3, 1, 1, 1, 1), (9, 3, 3, 32, 64, 3, 3, 1, 1, 1, 1),
                                  (70, 1, 1, 16, 32, 1, 1, 1, 0, 1, 1), (3, 17, 15, 24, 40, 3, 3, 2, 1, 1, 1),
                                  (2, 12, 12, 32, 48, 3, 3, 1, 2, 1, 2), (2, 27, 27, 96, 64, 5, 5, 1, 2, 2, 1),
                                  (4, 7, 9, 8, 16, 2, 3, 1, 0, 1, 1)])
def test_mc_im2col_wgrad_geometries(gpu, tile, splits, case, monkeypatch):
    from sparknet_amd.ops import gemm as G, hip, ref
    from sparknet_amd.ops.spec import ConvSpec
    N, H, W, Cc, K, R, S, st, pd, g, dil = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, dil, dil, g)
    x = _bf(N, H, W, Cc, device=gpu)
    dy = _bf(N, s.P, s.Q, K, device=gpu)
    M, kred = N * s.P * s.Q, R * S * (Cc // g)
    dw = torch.zeros(K, kred, device=gpu)
    db = torch.zeros(K, device=gpu)
    geom = hip._geom(s)
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    A = G.Dense(dy.view(M, K), K, kcontig=False, gstride=K // g)
    B = G.Im2col(x, geom, kcontig=False, gstride=Cc // g)
    try:
        G.gemm(K // g, kred, M, A, B, dw, kred, epi=G.EPI_F32, groups=g, c_gstride=(K // g) * kred,
               splits=splits, bias_grad=db if kred % 8 == 0 else None, bias_acc=False)
    except RuntimeError as e:
        pytest.skip(f"tile {tile}: no instance ({e})")
    w = torch.zeros(K, R, S, Cc // g)
    dw_r, db_r = torch.zeros(K, R, S, Cc // g), torch.zeros(K)
    ref.conv_backward(dy.float().cpu(), x.float().cpu(), w, s, False, dw_r, db_r)
    _close(dw, dw_r.view(K, kred).to(gpu), 1e-2)
    if kred % 8 == 0:
        _close(db, db_r.to(gpu), 1e-3)


def _db_tiles():
    """Every tile the packaged tuning database selects for a production product."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sparknet_amd", "ops",
                     "gemm_tuned.json")
    with open(p) as f:
        return sorted({int(v[0]) for v in json.load(f).values()})


# shapes with a ragged M / N edge and a K tail (K % 64 != 0) for every tile; wide / tall
# enough for two tiles along each axis
_EDGE = [(lambda bm, bn: (2 * bm + 17, 2 * bn + 8, 64 * 5 + 24)), (lambda bm, bn: (bm - 3, bn - 8, 64 * 33 + 8)),
         (lambda bm, bn: (3 * bm + 1, bn + 24, 136))]


@pytest.mark.parametrize("tile", _db_tiles())
@pytest.mark.parametrize("shape", range(len(_EDGE)))
def test_db_tiles_edges_and_k_tail(gpu, tile, shape, monkeypatch):
    """every tuned tile at 8e-3 on ragged M / N edges and K tails, through the
    NT (forward), NN (data gradient) and TN (weight gradient) layouts it has instances for."""
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    bm, bn = G.TILES[tile]
    M, N, K = _EDGE[shape](bm, bn)
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    b = torch.randn(N, device=gpu)
    _close(G.linear_fwd(x, w, b, relu=True), torch.relu(x.float() @ w.float().t() + b))
    dy = _bf(M, N, device=gpu)
    try:
        dx = G.linear_dgrad(dy, w)
    except RuntimeError:
        dx = None  # no MC-B instance for this tile
    if dx is not None:
        _close(dx, dy.float() @ w.float())
    dw = torch.ones(N, K, device=gpu)
    try:
        G.linear_wgrad(dy, x, dw, accumulate=True)
    except RuntimeError:
        return
    _close(dw, 1 + dy.float().t() @ x.float())


@pytest.mark.parametrize("tile", [21, 22])
@pytest.mark.parametrize("M,N,K", [(64, 576, 64 * 40), (48, 1200, 333 * 8), (24, 200, 1000), (64, 4096, 256)])
def test_thin_tiles(gpu, tile, M, N, K, monkeypatch):
    """64-row tiles (gemm_tiles_c.hip): NT / NN / TN dense products, split-K, the bias column."""
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    _close(G.linear_fwd(x, w), x.float() @ w.float().t())
    dy = _bf(M, N, device=gpu)
    _close(G.linear_dgrad(dy, w), dy.float() @ w.float())
    a, b = _bf(K, M, device=gpu), _bf(K, N, device=gpu)
    dw = torch.full((M, N), 3.0, device=gpu)
    db = torch.full((M,), -2.0, device=gpu)
    G.gemm(M, N, K, G.Dense(a, M, False), G.Dense(b, N, False), dw, N, epi=G.EPI_F32_ACC, splits=3,
           bias_grad=db, bias_acc=True)
    _close(dw, 3.0 + a.float().t() @ b.float())
    _close(db, -2.0 + a.float().sum(0), 1e-3)


@pytest.mark.parametrize("tile", [21, 22])
@pytest.mark.parametrize("case", [(2, 20, 20, 64, 64, 3, 3, 1, 1, 1), (3, 14, 14, 192, 16, 1, 1, 1, 0, 1),
                                  (2, 9, 9, 64, 48, 3, 3, 1, 1, 1)])
def test_thin_tiles_conv(gpu, tile, case, monkeypatch):
    from sparknet_amd.ops import gemm as G, hip, ref
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    N, H, W, Cc, K, R, S, st, pd, g = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    x = _bf(N, H, W, Cc, device=gpu)
    w = (torch.randn(K, R, S, Cc // g, device=gpu) * 0.1).to(torch.bfloat16)
    bias = torch.randn(K, device=gpu)
    _close(hip.conv_forward(x, w, bias, s, relu=True), ref.conv_forward(x, w, bias, s, relu=True))
    dy = _bf(N, s.P, s.Q, K, device=gpu)
    dw, db = torch.zeros(K, R, S, Cc // g, device=gpu), torch.zeros(K, device=gpu)
    dw_r, db_r = torch.zeros_like(dw), torch.zeros_like(db)
    hip.conv_backward(dy, x, w, s, False, dw, db)
    ref.conv_backward(dy, x, w, s, False, dw_r, db_r)
    _close(dw, dw_r)
    _close(db, db_r, 1e-3)


@pytest.mark.parametrize("tile", [0, 4, 5, 16])
@pytest.mark.parametrize("case", [(2, 9, 9, 24, 32, 2, 2, 1, 0, 1), (2, 11, 11, 40, 48, 3, 3, 1, 1, 1),
                                  (2, 13, 13, 96, 64, 5, 5, 1, 2, 2), (3, 10, 10, 56, 24, 3, 3, 2, 1, 1)])
def test_small_cg_im2col(gpu, tile, case, monkeypatch):
    """Implicit im2col with 16 < Cg < 64 channels per group: a 64-wide K-step straddles up
    to three filter taps (the branch-free carry of GStager.issue); fwd, dgrad, wgrad + bias
    against the fp32 reference."""
    from sparknet_amd.ops import gemm as G, hip, ref
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    N, H, W, Cc, K, R, S, st, pd, g = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    x = _bf(N, H, W, Cc, device=gpu)
    w = (torch.randn(K, R, S, Cc // g, device=gpu) * 0.1).to(torch.bfloat16)
    bias = torch.randn(K, device=gpu)
    _close(hip.conv_forward(x, w, bias, s, relu=True), ref.conv_forward(x, w, bias, s, relu=True))
    if tile != 0:  # 4 / 16: K-contiguous B only (forward products); 5: 48-wide outputs
        return
    dy = _bf(N, s.P, s.Q, K, device=gpu)
    dw, db = torch.zeros(K, R, S, Cc // g, device=gpu), torch.zeros(K, device=gpu)
    dw_r, db_r = torch.zeros_like(dw), torch.zeros_like(db)
    dx = hip.conv_backward(dy, x, w, s, True, dw, db)
    dx_r = ref.conv_backward(dy, x, w, s, True, dw_r, db_r)
    _close(dx, dx_r)
    _close(dw, dw_r)
    _close(db, db_r, 1e-3)


@pytest.mark.parametrize("tile,splits", [(22, 229), (22, 1), (21, 229), (0, 229)])
def test_thin_tiles_small_c(gpu, tile, splits, monkeypatch):
    """cifar10_quick's conv1 weight gradient (C 8 after channel padding, 5x5 pad 2, M = 32
    filters, N = 201 with the bias column, reduction over 100 x 32 x 32 pixels) at the
    split-K the first-call tuner picked (tile 22, 229 ways): against the fp32 reference."""
    from sparknet_amd.ops import gemm as G, hip, ref
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    s = ConvSpec(100, 32, 32, 8, 32, 5, 5, 1, 1, 2, 2, 1, 1, 1)
    kchunk = -(-(-(-102400 // splits)) // 64) * 64
    monkeypatch.setattr(G, "choose_splits", lambda *a, **k: (-(-102400 // kchunk), kchunk))
    x = _bf(100, 32, 32, 8, device=gpu)
    w = (torch.randn(32, 5, 5, 8, device=gpu) * 0.1).to(torch.bfloat16)
    dy = _bf(100, 32, 32, 32, device=gpu)
    dw, db = torch.zeros(32, 5, 5, 8, device=gpu), torch.zeros(32, device=gpu)
    dw_r, db_r = torch.zeros_like(dw), torch.zeros_like(db)
    hip.conv_backward(dy, x, w, s, False, dw, db)
    ref.conv_backward(dy, x, w, s, False, dw_r, db_r)
    _close(dw, dw_r)
    _close(db, db_r, 1e-3)


def test_thin_tiles_bitwise_equal_at_same_split(gpu, monkeypatch):
    """Round-5 root cause of the round-4 'thin tiles break cifar10_quick' report: at equal
    split-K the 64-row tiles 21 / 22 give bitwise the same weight and bias gradient as the
    default tiles 0 / 10 (same fp32 summation order per split, same split-K reduce), so a
    training difference between them can only come from the split count the tuner picked —
    and that order sensitivity is the training's own (tests/test_training_gpu.py)."""
    from sparknet_amd.ops import gemm as G, hip
    from sparknet_amd.ops.spec import ConvSpec
    s = ConvSpec(100, 32, 32, 8, 32, 5, 5, 1, 1, 2, 2, 1, 1, 1)
    g = torch.Generator(device="cpu").manual_seed(3)
    x = (torch.randn(100, 32, 32, 8, generator=g) * 40).to(torch.bfloat16)
    x[..., 3:] = 0
    dy = (torch.randn(100, 32, 32, 32, generator=g) * 1e-3).to(torch.bfloat16).to(gpu)
    x, w = x.to(gpu), (torch.randn(32, 5, 5, 8, device=gpu) * 0.1).to(torch.bfloat16)
    for splits in (229, 178):
        kchunk = -(-(-(-102400 // splits)) // 64) * 64
        monkeypatch.setattr(G, "choose_splits", lambda *a, **k: (-(-102400 // kchunk), kchunk))
        outs = []
        for tile in (0, 10, 21, 22):
            monkeypatch.setattr(G, "_FORCE_TILE", tile)
            dw, db = torch.zeros(32, 5, 5, 8, device=gpu), torch.zeros(32, device=gpu)
            hip.conv_backward(dy, x, w, s, False, dw, db)
            outs.append(torch.cat([dw.flatten(), db]))
        for o in outs[1:]:
            assert torch.equal(o, outs[0]), splits
