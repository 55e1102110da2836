"""Numerics of the persistent ring-pipelined GEMM tiles (csrc/kernels/gemm_pk.h, tiles 30-36)
against fp32 PyTorch references: every operand layout, ragged M / N / K edges, short K (fewer
K-steps than ring slots), more output tiles than CUs (the persistent tile loop and the
cross-tile prefetch), split-K, the bias-gradient column, and the implicit-GEMM convolutions
(forward, data and weight gradients)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

PK = [30, 31, 32, 33, 34, 36, 37, 38]
MC_B = {30, 31, 32, 33, 36, 38}  # tiles whose B image accepts k-strided (MC) operands
TOL = 8e-3


def _bf(*shape, device):
    return (torch.randn(*shape, device=device) * 0.5).to(torch.bfloat16)


def _close(a, b, tol=TOL):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err / scale < tol, f"rel err {err / scale:.3e}"


@pytest.mark.parametrize("tile", PK)
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 200, 136), (1000, 384, 2304), (513, 129, 1000), (64, 48, 40),
                                   (40000, 384, 200), (9000, 96, 1216)])
def test_pk_dense_layouts(gpu, tile, M, N, K, monkeypatch):
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    b = torch.randn(N, device=gpu)
    _close(G.linear_fwd(x, w, b, relu=True), torch.relu(x.float() @ w.float().t() + b))
    if tile not in MC_B:
        return
    dy = _bf(M, N, device=gpu)
    w2 = _bf(N, K, device=gpu)
    _close(G.linear_dgrad(dy, w2), dy.float() @ w2.float())
    dw = torch.ones(N, K, device=gpu)
    G.linear_wgrad(dy, x, dw, accumulate=True)
    _close(dw, 1 + dy.float().t() @ x.float())


@pytest.mark.parametrize("tile", sorted(MC_B))
@pytest.mark.parametrize("splits", [1, 3, 11])
def test_pk_bias_column_splitk_gate(gpu, tile, splits, monkeypatch):
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    M, N, K = 96, 432, 64 * 40 + 17
    a, bm = _bf(K, M, device=gpu), _bf(K, N, device=gpu)
    dw = torch.full((M, N), 3.0, device=gpu)
    db = torch.full((M,), -2.0, device=gpu)
    G.gemm(M, N, K, G.Dense(a, M, False), G.Dense(bm, N, False), dw, N, epi=G.EPI_F32_ACC, splits=splits,
           bias_grad=db, bias_acc=True)
    _close(dw, 3.0 + a.float().t() @ bm.float())
    _close(db, -2.0 + a.float().sum(0), 1e-3)
    Kp = 64 * 41
    x, w = _bf(M * 7, K, device=gpu), _bf(N, K, device=gpu)
    xp = torch.zeros(M * 7, Kp, dtype=x.dtype, device=gpu)
    xp[:, :K] = x
    wp = torch.zeros(N, Kp, dtype=w.dtype, device=gpu)
    wp[:, :K] = w
    y = torch.empty(M * 7, N, device=gpu, dtype=torch.bfloat16)
    gate = _bf(M * 7, N, device=gpu)
    bias = torch.randn(N, device=gpu)
    G.gemm(M * 7, N, K, G.Dense(xp, Kp, True), G.Dense(wp, Kp, True), y, N, epi=G.EPI_BF16, splits=splits,
           gate=gate, bias=bias, relu=True)
    _close(y, torch.relu(x.float() @ w.float().t() + bias) * (gate.float() > 0))


@pytest.mark.parametrize("tile", PK)
@pytest.mark.parametrize("case", [(2, 13, 13, 64, 384, 3, 3, 1, 1, 1), (2, 27, 27, 96, 256, 5, 5, 1, 2, 2),
                                  (4, 14, 14, 32, 128, 1, 1, 1, 0, 1), (3, 9, 9, 64, 40, 3, 3, 1, 1, 2),
                                  (2, 7, 7, 192, 96, 3, 3, 1, 1, 2), (16, 27, 27, 48, 128, 5, 5, 1, 2, 1),
                                  (64, 13, 13, 256, 384, 3, 3, 1, 1, 1)])
def test_pk_conv(gpu, tile, case, monkeypatch):
    from sparknet_amd.ops import gemm as G, hip, ref
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    N, H, W, Cc, K, R, S, st, pd, g = case
    s = ConvSpec(N, H, W, Cc, K, R, S, st, st, pd, pd, 1, 1, g)
    x = _bf(N, H, W, Cc, device=gpu)
    w = (torch.randn(K, R, S, Cc // g, device=gpu) * 0.1).to(torch.bfloat16)
    bias = torch.randn(K, device=gpu)
    _close(hip.conv_forward(x, w, bias, s, relu=True), ref.conv_forward(x, w, bias, s, relu=True))
    if tile not in MC_B:
        return
    dy = _bf(N, s.P, s.Q, K, device=gpu)
    dw, db = torch.zeros(K, R, S, Cc // g, device=gpu), torch.zeros(K, device=gpu)
    dw_r, db_r = torch.zeros_like(dw), torch.zeros_like(db)
    dx = hip.conv_backward(dy, x, w, s, True, dw, db)
    dx_r = ref.conv_backward(dy, x, w, s, True, dw_r, db_r)
    _close(dx, dx_r)
    _close(dw, dw_r)
    _close(db, db_r, 1e-3)


@pytest.mark.parametrize("tile", [30, 31])
def test_pk_repeatable(gpu, tile, monkeypatch):
    """Same inputs, same tile and split -> bitwise identical outputs (no atomics, fixed
    per-tile reduction order regardless of which block runs the tile)."""
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    x, w = _bf(30000, 1152, device=gpu), _bf(256, 1152, device=gpu)
    y0 = G.linear_fwd(x, w)
    for _ in range(3):
        assert torch.equal(G.linear_fwd(x, w), y0)
