"""Numerics of the e4m3 direct 3x3 convolution (csrc/kernels/conv3x3_fp8.hip: 64 -> 64
channels, stride 1, pad 1) against fp32 PyTorch convolutions of the same dequantised
values: forward (bias, ReLU), data gradient (flip-transposed weights, ReLU-backward gate),
ragged spatial edges (partial 16 x 16 tiles), and more tiles than CUs (the persistent loop
with its cross-tile patch prefetch).  The GEMM path (SN_CONV_DIRECT_FP8=0 equivalent) on the
same bytes must agree too."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _f8(t):
    q = t.float().clamp(-448, 448).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), q.float()


def _close(a, b, tol):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err / scale < tol, f"rel err {err / scale:.3e}"


@pytest.mark.parametrize("N,H,W", [(1, 16, 16), (2, 13, 29), (3, 33, 17), (40, 56, 56), (2, 224, 224)])
@pytest.mark.parametrize("relu,bias", [(False, False), (True, True)])
def test_direct_fp8_forward(gpu, N, H, W, relu, bias, monkeypatch):
    from sparknet_amd.ops import hip
    monkeypatch.setattr(hip, "_DIRECT_FP8", True)
    from sparknet_amd.ops.spec import ConvSpec
    s = ConvSpec(N, H, W, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    assert hip.direct_fp8_ok(s)
    gen = torch.Generator(device=gpu).manual_seed(N * 1000 + H)
    xq, xf = _f8(torch.randn(N, H, W, 64, device=gpu, generator=gen) * 4)
    wq, wf = _f8(torch.randn(64, 3, 3, 64, device=gpu, generator=gen) * 4)
    b = torch.randn(64, device=gpu, generator=gen) * 20 if bias else None
    dx, dw = torch.tensor([0.5], device=gpu), torch.tensor([0.0625], device=gpu)
    y = hip.conv_forward_fp8(xq, wq, b, s, dx, dw, relu=relu)
    ref = F.conv2d(xf.permute(0, 3, 1, 2), wf.permute(0, 3, 1, 2), padding=1) * (0.5 * 0.0625)
    if bias:
        ref = ref + b.view(1, -1, 1, 1)
    if relu:
        ref = torch.relu(ref)
    _close(y.permute(0, 3, 1, 2), ref, 8e-3)


def test_direct_fp8_matches_gemm_path(gpu, monkeypatch):
    """The direct kernel and the implicit-GEMM fp8 path read the same bytes and scales."""
    from sparknet_amd.ops import hip
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(hip, "_DIRECT_FP8", True)
    s = ConvSpec(4, 40, 40, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    xq, _ = _f8(torch.randn(4, 40, 40, 64, device=gpu) * 4)
    wq, _ = _f8(torch.randn(64, 3, 3, 64, device=gpu) * 4)
    dx, dw = torch.tensor([0.25], device=gpu), torch.tensor([0.125], device=gpu)
    b = torch.randn(64, device=gpu)
    y1 = hip.conv_forward_fp8(xq, wq, b, s, dx, dw, relu=True)
    monkeypatch.setattr(hip, "_DIRECT_FP8", False)
    y2 = hip.conv_forward_fp8(xq, wq, b, s, dx, dw, relu=True)
    _close(y1, y2, 8e-3)


@pytest.mark.parametrize("N,H,W,gated", [(2, 20, 37, True), (24, 56, 56, False), (2, 224, 224, True)])
def test_direct_fp8_dgrad(gpu, N, H, W, gated, monkeypatch):
    """ops.hip._conv_dgrad_fp8 on a 64 -> 64 conv takes the direct kernel (e4m3 dy x e4m3
    flip-transposed weights), gate fused; error vs the fp32 transposed conv of the bf16
    inputs within e4m3 rounding, like the GEMM path's test (test_gemm_gpu.test_fp8_conv_dgrad)."""
    from sparknet_amd.ops import hip
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(hip, "_DIRECT_FP8", True)
    s = ConvSpec(N, H, W, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    gen = torch.Generator(device=gpu).manual_seed(7)
    x = torch.randn(N, H, W, 64, device=gpu, generator=gen).to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, device=gpu, generator=gen) * 0.05).to(torch.bfloat16)
    dy = (torch.randn(N, H, W, 64, device=gpu, generator=gen) * 1e-4).to(torch.bfloat16)
    gate = x if gated else None
    sc = hip.Fp8Scales(2, gpu)
    dx8 = hip.conv_backward(dy, x, w, s, True, ws={"fp8_dgrad": (sc, 0, 1)}, gate=gate)
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2),
                             padding=1).permute(0, 2, 3, 1)
    if gated:
        ref = ref * (x.float() > 0)
        assert torch.all(dx8[x <= 0] == 0)
    err8 = ((dx8.float() - ref).norm() / ref.norm()).item()
    assert err8 < 0.05, err8
