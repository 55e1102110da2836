"""Numerics of the MFMA GEMM against an fp32 PyTorch reference (all layouts)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(*shape, device):
    return (torch.randn(*shape, device=device) * 0.5).to(torch.bfloat16)


def _close(a, b, tol=2e-2):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err / scale < tol, f"rel err {err/scale:.3e}"


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 4096, 1024), (100, 70, 200), (77, 96, 363 + 5), (1000, 10, 64)])
def test_linear_fwd(gpu, M, N, K):
    from sparknet_amd.ops import gemm
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    b = torch.randn(N, device=gpu)
    y = gemm.linear_fwd(x, w, b, relu=True)
    ref = torch.relu(x.float() @ w.float().t() + b)
    _close(y, ref)


def test_identity_asymmetric(gpu):
    # A = I with an asymmetric B catches transposed C writes.
    from sparknet_amd.ops import gemm
    n = 128
    eye = torch.eye(n, device=gpu).to(torch.bfloat16)
    w = (torch.arange(n * n, device=gpu).reshape(n, n) % 17).to(torch.bfloat16)
    y = gemm.linear_fwd(eye, w)
    assert torch.equal(y.float(), w.float().t())


@pytest.mark.parametrize("M,N,K", [(256, 4096, 9216), (64, 10, 500), (128, 200, 136), (300, 200, 40)])
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


def test_colsum(gpu):
    from sparknet_amd.ops import gemm
    x = _bf(5000, 96, device=gpu)
    out = torch.ones(96, device=gpu)
    gemm.colsum(x, out)
    _close(out, 1 + x.float().sum(0), 1e-3)
