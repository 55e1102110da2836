"""In-launch deterministic split-K combine (gemm_kernel fix_cnt, ops.gemm SN_GEMM_FIXUP):
the last-arriving K-slice block of each output tile sums every slice's fp32 slab in split
order and runs the product's real epilogue, instead of a separate splitk_reduce launch.

* against the reduce-launch path on the same tile / split: fp32 outputs (plain, accumulate,
  the bias-gradient ones column) bitwise equal below 16 slices (both sum slices 0..S-1 in
  order from zero), bf16 epilogues (bias, ReLU, gate, dropout) within bf16 rounding;
* bitwise repeatable run to run (whichever block arrives last);
* replayed from a captured hipGraph: the counters return to zero after every launch.

Reference: the reduction Caffe does in one cuBLAS call (caffe/src/caffe/util/math_functions.cu:
caffe_gpu_gemm); split-K is this engine's own decomposition."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# gemm_kernel tile family: 4-wave (0, 1, 4, 5, 10, 16, 17, 20), 8-wave (2, 12), 64-row (21),
# 32x32x16 MFMA (23)
TILES = [0, 1, 2, 4, 5, 10, 12, 16, 17, 20, 21, 23]


def _bf(*shape, device):
    return torch.randn(*shape, device=device).to(torch.bfloat16)


def _close(a, b, tol=8e-3):
    err = float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6))
    assert err < tol, err


def _run_both(G, monkeypatch, fn):
    out = {}
    for mode in (0, 2, 2):
        monkeypatch.setattr(G, "_FIXUP", mode)
        r = fn()
        torch.cuda.synchronize()
        out.setdefault(mode, []).append(r)
    return out[0][0], out[2][0], out[2][1]


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("splits", [2, 7, 19])
def test_fixup_fp32_products_match_reduce(gpu, tile, splits, monkeypatch):
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    bm, bn = G.TILES[tile]
    M, N, K = 2 * bm + 5, bn + 24, 64 * 3 * splits + 40
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)

    def fwd_acc():
        acc = torch.ones(M, N, device=gpu)
        G.gemm(M, N, K, G.Dense(x, K, True), G.Dense(w, K, True), acc, N, epi=G.EPI_F32_ACC, splits=splits)
        return acc
    try:
        red, fix, fix2 = _run_both(G, monkeypatch, fwd_acc)
    except RuntimeError:
        pytest.skip(f"tile {tile}: no dense NT instance")
    assert torch.equal(fix, fix2)
    if splits < 16:
        assert torch.equal(fix, red)
    _close(fix, 1 + x.float() @ w.float().t(), 1e-2)
    # weight-gradient TN form with the virtual ones column routed to the bias gradient
    M = M - M % 8  # MC operands: 16-B rows
    a, b = _bf(K, M, device=gpu), _bf(K, N - N % 8, device=gpu)
    Nb = b.shape[1]

    def wgrad():
        dw = torch.full((M, Nb), 3.0, device=gpu)
        db = torch.full((M,), -2.0, device=gpu)
        G.gemm(M, Nb, K, G.Dense(a, M, False), G.Dense(b, Nb, False), dw, Nb, epi=G.EPI_F32_ACC, splits=splits,
               bias_grad=db, bias_acc=True)
        return torch.cat([dw.flatten(), db])
    try:
        red, fix, fix2 = _run_both(G, monkeypatch, wgrad)
    except RuntimeError:
        return  # no MC x MC instance for this tile
    assert torch.equal(fix, fix2)
    if splits < 16:
        assert torch.equal(fix, red)
    _close(fix[:M * Nb].view(M, Nb), 3.0 + a.float().t() @ b.float(), 1e-2)
    _close(fix[M * Nb:], -2.0 + a.float().sum(0), 1e-3)


@pytest.mark.parametrize("tile", [0, 10, 16, 21])
@pytest.mark.parametrize("splits", [3, 11])
def test_fixup_bf16_epilogues(gpu, tile, splits, monkeypatch):
    """bias + ReLU + gate, and the fused dropout epilogue, after the in-launch combine."""
    from sparknet_amd.ops import gemm as G
    monkeypatch.setattr(G, "_FORCE_TILE", tile)
    M, N, K = 300, 200, 64 * 4 * splits
    x, w = _bf(M, K, device=gpu), _bf(N, K, device=gpu)
    b = torch.randn(N, device=gpu)
    gate = _bf(M, N, device=gpu)
    ref = x.float() @ w.float().t()
    rng = torch.tensor([1234, 0], dtype=torch.int64, device=gpu)

    def bf16():
        y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        G.gemm(M, N, K, G.Dense(x, K, True), G.Dense(w, K, True), y, N, epi=G.EPI_BF16, bias=b, relu=True,
               splits=splits, gate=gate)
        yd = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        G.gemm(M, N, K, G.Dense(x, K, True), G.Dense(w, K, True), yd, N, epi=G.EPI_BF16, bias=b, relu=True,
               splits=splits, dropout=(rng, 3, 0.5))
        return y, yd
    (y0, d0), (y1, d1), (y2, d2) = _run_both(G, monkeypatch, bf16)
    assert torch.equal(y1, y2) and torch.equal(d1, d2)
    _close(y1, torch.relu(ref + b) * (gate.float() > 0))
    _close(y1, y0)
    # the same Philox keep mask on both paths; kept values within bf16 rounding
    assert torch.equal(d1 == 0, d0 == 0)
    _close(d1, d0)


def test_fixup_grouped_conv_wgrad_and_graph_replay(gpu, monkeypatch):
    """A grouped implicit-im2col weight gradient (MC B operand, ones column, split-K) through
    the combine, eager and replayed three times from one captured graph."""
    from sparknet_amd.ops import gemm as G, hip
    from sparknet_amd.ops.spec import ConvSpec
    monkeypatch.setattr(G, "_FORCE_TILE", 10)
    s = ConvSpec(4, 27, 27, 96, 256, 5, 5, 1, 1, 2, 2, 1, 1, 2)
    x = _bf(4, 27, 27, 96, device=gpu)
    w = (torch.randn(256, 5, 5, 48, device=gpu) * 0.05).to(torch.bfloat16)
    dy = _bf(4, s.P, s.Q, 256, device=gpu)

    def wg():
        dw = torch.zeros(256, 5, 5, 48, device=gpu)
        db = torch.zeros(256, device=gpu)
        hip.conv_backward(dy, x, w, s, False, dw, db)
        return torch.cat([dw.flatten(), db])
    red, fix, fix2 = _run_both(G, monkeypatch, wg)
    assert torch.equal(fix, fix2)
    _close(fix, red, 1e-5)
    monkeypatch.setattr(G, "_FIXUP", 2)
    dw = torch.zeros(256, 5, 5, 48, device=gpu)
    db = torch.zeros(256, device=gpu)
    hip.conv_backward(dy, x, w, s, False, dw, db)  # warm (pool, workspace) before capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
        dw.zero_()
        db.zero_()
        hip.conv_backward(dy, x, w, s, False, dw, db)
    torch.cuda.current_stream().wait_stream(st)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(torch.cat([dw.flatten(), db]), fix)
