"""Fused max-pool + cross-channel LRN (csrc/kernels/pool_lrn.hip, engine.fuse_pool_lrn).

* kernel level: the fused forward (pooled tensor, argmax mask, LRN output) and the fused
  backward (pooling-input gradient from the LRN-output gradient) are BITWISE equal to the
  unfused launches (maxpool_fwd_k + lrn_across_fwd, lrn_across_bwd + pool_bwd_k3s2) on
  CaffeNet's pool1/norm1 and pool2/norm2 shapes, GoogLeNet's pool1/norm1 and a padded
  odd-sized case, with and without the folded ReLU gate; and they track the fp32 CPU
  reference (ops.ref);
* net level: CaffeNet fuses both pairs, and a fused GPU step equals an unfused one;
* the other order (LRN -> max pool, AlexNet / GoogLeNet; engine.fuse_lrn_pool_backward):
  the one-launch backward (pool_lrn_bwd_rev) is BITWISE equal to pool_bwd_k3s2 followed by
  lrn_across_bwd, and AlexNet / GoogLeNet steps with it equal steps without it.
Reference: caffe/src/caffe/layers/pooling_layer.cu:11-47,217-260, lrn_layer.cu:9-177."""
import pytest
import torch

from sparknet_amd.ops.spec import PoolSpec

pytestmark = pytest.mark.gpu

CASES = [  # N, H, W, C, pad, LRN size
    (4, 55, 55, 96, 0, 5),    # CaffeNet pool1 -> norm1
    (4, 27, 27, 256, 0, 5),   # CaffeNet pool2 -> norm2
    (2, 112, 112, 64, 0, 5),  # GoogLeNet pool1/3x3_s2 -> pool1/norm1
    (3, 14, 15, 40, 1, 3),    # padded, odd sizes, C not a multiple of 16
]


def _inputs(N, H, W, C, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(N, H, W, C, generator=g) * 2.0).to(torch.bfloat16)
    return x


@pytest.mark.parametrize("gate", [False, True])
@pytest.mark.parametrize("case", CASES)
def test_fused_pool_lrn_bitwise(gpu, case, gate):
    from sparknet_amd.ops import hip
    N, H, W, C, pad, size = case
    s = PoolSpec(N, H, W, C, 3, 3, 2, 2, pad, pad)
    assert hip.pool_lrn_eligible(s, size, False)
    alpha, beta, k = 1e-4 * 50, 0.75, 1.0  # a large alpha so the normalisation matters
    x = _inputs(N, H, W, C, 1).to(gpu)
    if gate:
        x = x.clamp_min(0)  # the in-place ReLU output the gate stands for
    pooled, mask, y = hip.pool_lrn_forward(x, s, gate, size, alpha, beta, k)
    p_ref, m_ref = hip.pool_forward_mask(x, s, gate)
    y_ref = hip.lrn_forward(p_ref, size, alpha, beta, k)
    assert torch.equal(pooled, p_ref) and torch.equal(mask, m_ref) and torch.equal(y, y_ref)
    dy = _inputs(N, s.P, s.Q, C, 2).to(gpu)
    dx = hip.lrn_pool_backward(dy, pooled, mask, s, size, alpha, beta, k)
    dp = hip.lrn_backward(dy, p_ref, size, alpha, beta, k)
    dx_ref = hip.pool_backward(dp, x, s, m_ref, gate=gate)
    assert torch.equal(dx, dx_ref)
    # and against the fp32 CPU reference of the two layers
    from sparknet_amd.ops import ref
    pr = ref.pool_forward(x.float().cpu(), s)  # NHWC, like the device tensors
    yr = ref.lrn_forward(pr, size, alpha, beta, k)
    err = (y.float().cpu() - yr).abs().max() / yr.abs().max()
    assert err < 2e-2, err


def test_caffenet_step_fused_equals_unfused(gpu):
    from sparknet_amd import engine, models
    from sparknet_amd.core.solver import Solver
    results = []
    for fuse in (True, False):
        sp = models.zoo.caffenet_solver(models.caffenet(train_batch=8, test_batch=8, crop=227, classes=10))
        solver = Solver(sp, device=torch.device(gpu), seed=5, build_test_nets=False)
        net = solver.net
        if fuse:
            engine.fuse_relu(net)
            assert sum(l.fused_lrn is not None for l in net.layers if l.type_name == "Pooling") == 2
        else:
            orig = engine.fuse_pool_lrn
            engine.fuse_pool_lrn = lambda n: 0
            try:
                engine.fuse_relu(net)
            finally:
                engine.fuse_pool_lrn = orig
        g = torch.Generator().manual_seed(9)
        x = torch.randn(8, 3, 227, 227, generator=g) * 50
        lab = torch.randint(0, 10, (8, 1), generator=g).float()
        losses = []
        for _ in range(3):
            net.blob_by_name("data").set_nchw(x)
            net.blob_by_name("label").set_nchw(lab)
            losses.append(float(solver.iteration()))
            solver.iter += 1
        torch.cuda.synchronize()
        results.append((losses, net.flat_data.detach().clone()))
    assert results[0][0] == results[1][0]
    assert torch.equal(results[0][1], results[1][1])


@pytest.mark.parametrize("case", [(1, 200, 200, 56, 0, 5), (1, 260, 260, 56, 0, 3), (2, 27, 27, 56, 0, 5)])
def test_pool_lrn_eligibility_matches_kernels(gpu, case):
    """the Python eligibility check mirrors the kernels' own host tests (prime
    channel-chunk counts such as C = 56, cv = 7, at wide pooled rows), so every shape it
    accepts launches, and every shape it refuses takes the unfused path without error."""
    from sparknet_amd.ops import hip
    N, H, W, C, pad, size = case
    s = PoolSpec(N, H, W, C, 3, 3, 2, 2, pad, pad)
    alpha, beta, k = 1e-4, 0.75, 1.0
    x = _inputs(N, H, W, C, 3).to(gpu)
    p_ref, m_ref = hip.pool_forward_mask(x, s, False)
    dy = _inputs(N, s.P, s.Q, C, 4).to(gpu)
    dp = hip.lrn_backward(dy, p_ref, size, alpha, beta, k)
    dx_ref = hip.pool_backward(dp, x, s, m_ref)
    if hip.pool_lrn_eligible(s, size, False):
        pooled, mask, y = hip.pool_lrn_forward(x, s, False, size, alpha, beta, k)
        assert torch.equal(hip.lrn_pool_backward(dy, pooled, mask, s, size, alpha, beta, k), dx_ref)
    else:
        with pytest.raises(RuntimeError):
            hip.lrn_pool_backward(dy, p_ref, m_ref, s, size, alpha, beta, k)



REV_CASES = [  # N, H, W, C, pad, LRN size: LRN input shape = pooling input shape
    (4, 55, 55, 96, 0, 5),    # AlexNet norm1 -> pool1
    (4, 27, 27, 256, 0, 5),   # AlexNet norm2 -> pool2
    (2, 56, 56, 192, 0, 5),   # GoogLeNet conv2/norm2 -> pool2/3x3_s2
    (3, 14, 15, 40, 1, 3),    # padded, odd sizes
    (2, 13, 13, 8, 0, 9),     # one channel chunk: every neighbour chunk is outside [0, C)
    (2, 9, 12, 24, 2, 7),
]


@pytest.mark.parametrize("gate", [False, True])
@pytest.mark.parametrize("case", REV_CASES)
def test_lrn_pool_backward_rev_bitwise(gpu, case, gate):
    from sparknet_amd.ops import hip
    N, H, W, C, pad, size = case
    s = PoolSpec(N, H, W, C, 3, 3, 2, 2, pad, pad)
    assert hip.pool_lrn_rev_eligible(s, size, False)
    alpha, beta, k = 1e-4 * 50, 0.75, 1.0
    x = _inputs(N, H, W, C, 5).to(gpu)
    if gate:
        x = x.clamp_min(0)
    y = hip.lrn_forward(x, size, alpha, beta, k)
    _, mask = hip.pool_forward_mask(y, s, False)
    dy = _inputs(N, s.P, s.Q, C, 6).to(gpu)
    dl = hip.pool_backward(dy, y, s, mask)
    dx_ref = hip.lrn_backward(dl, x, size, alpha, beta, k, gate=gate)
    dx = hip.pool_lrn_backward_rev(dy, mask, x, s, size, alpha, beta, k, gate)
    assert torch.equal(dx, dx_ref)


@pytest.mark.parametrize("model", ["alexnet", "googlenet"])
def test_step_lrn_pool_bwd_fused_equals_unfused(gpu, model, monkeypatch):
    from sparknet_amd import engine, models
    from sparknet_amd.core.solver import Solver
    B, crop = (8, 227) if model == "alexnet" else (4, 224)
    want = 2 if model == "alexnet" else 1
    results = []
    for fuse in (True, False):
        monkeypatch.setenv("SN_FEATURES", "" if fuse else "fuse_lrn_pool_bwd=0")
        sp = models.zoo.solver_for(model, train_batch=B, test_batch=B, crop=crop, classes=10)
        solver = Solver(sp, device=torch.device(gpu), seed=5, build_test_nets=False)
        net = solver.net
        engine.fuse_relu(net)
        n = sum(l.bwd_lrn is not None for l in net.layers if l.type_name == "Pooling")
        assert n == (want if fuse else 0)
        g = torch.Generator().manual_seed(9)
        x = torch.randn(B, 3, crop, crop, generator=g) * 50
        lab = torch.randint(0, 10, (B, 1), generator=g).float()
        losses = []
        for _ in range(3):
            net.blob_by_name("data").set_nchw(x)
            net.blob_by_name("label").set_nchw(lab)
            losses.append(float(solver.iteration()))
            solver.iter += 1
        torch.cuda.synchronize()
        results.append((losses, net.flat_data.detach().clone()))
    assert results[0][0] == results[1][0]
    assert torch.equal(results[0][1], results[1][1])
