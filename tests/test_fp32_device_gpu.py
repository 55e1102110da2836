"""The fp32 device mode: a net built with dtype=torch.float32 on the GPU runs
the reference's numerics — Caffe's fp32 im2col + GEMM (/root/reference/libccaffe/ccaffe.h:3,
caffe/src/caffe/layers/base_conv_layer.cpp:312-376) on exact-f32 matrix cores
(csrc/kernels/fp32.hip, ops/f32dev.py).

* the fp32 MFMA GEMM against a float64 product (ragged M / N / K, unaligned rows, bias / ReLU /
  accumulate epilogues);
* convolution forward / data / weight / bias gradients against the fp32 CPU engine (groups,
  strides, padding, dilation);
* CaffeNet b256: one SGD iteration from identical weights and batches — every weight update
  within 1e-3 of the fp32 CPU engine's in relative L2 norm (2e-3 in the largest element),
  every bias update within 3e-3 (L2) / 2e-2 (largest element), where the bf16 engine's floor
  is ~11 % (L2) / ~15 % (max) on conv1 (tests/test_bench_fidelity_gpu.py).  The bias bounds
  are fp32 summation-order noise: a bias gradient sums 43,264-774,400 pixel terms that nearly
  cancel at this initialisation (conv2's: 186,624 terms, max-element deviation ~1e-2 between
  two fp32 reduction orders; measured on one MI355X, profiles/r6_fp32_device.txt).
Reference check pattern: caffe/src/caffe/test/test_gradient_based_solver.cpp:225-320."""
import pytest
import torch

from sparknet_amd import models

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (300, 200, 77), (5, 1000, 4096), (1000, 7, 363), (257, 129, 1),
                                   (64, 200, 100003), (96, 363, 20000)])  # the last two: split-K slabs
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "acc"])
def test_gemm_f32_matches_fp64(gpu, M, N, K, epi):
    from sparknet_amd.ops import f32dev
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    a = torch.randn(M, K + 3, generator=g)[:, :K]  # unaligned row stride
    b = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    c0 = torch.randn(M, N, generator=g)
    ref = a.double() @ b.double().t()
    out = c0.clone().to(gpu) if epi == "acc" else torch.empty(M, N, device=gpu)
    f32dev.gemm_nt(a.to(gpu), b.to(gpu), out, bias=bias.to(gpu) if epi == "bias_relu" else None,
                   relu=epi == "bias_relu", accumulate=epi == "acc")
    if epi == "acc":
        ref = ref + c0.double()
    elif epi == "bias_relu":
        ref = torch.relu(ref + bias.double())
    err = (out.double().cpu() - ref).abs().max().item()
    scale = (a.double().abs() @ b.double().abs().t()).max().item()
    assert err <= 4e-7 * scale + 1e-6, (err, scale)


@pytest.mark.parametrize("M,N,K", [(128, 128, 32), (300, 200, 77), (6, 1003, 5001), (96, 363, 20000), (130, 9, 3)])
@pytest.mark.parametrize("a_t,b_t", [(True, False), (False, True), (True, True)])
def test_gemm_f32_kmajor_operands(gpu, M, N, K, a_t, b_t):
    """Operands stored k-major ([K][M] / [K][N]) are read in place, with row strides wider than
    the rows (a channel slice of a wider tensor), through the plain and the split-K paths."""
    from sparknet_amd.ops import f32dev
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N + K)
    a_full = torch.randn(K, M + 5, generator=g) if a_t else torch.randn(M, K + 5, generator=g)
    b_full = torch.randn(K, N + 4, generator=g) if b_t else torch.randn(N, K + 4, generator=g)
    ag, bg = a_full.to(gpu), b_full.to(gpu)
    a = ag[:, 1:M + 1] if a_t else ag[:, 1:K + 1]
    b = bg[:, 4:N + 4] if b_t else bg[:, 4:K + 4]
    am = (a.t() if a_t else a).double().cpu()
    bm = (b.t() if b_t else b).double().cpu()
    out = torch.empty(M, N, device=gpu)
    f32dev.gemm(a, b, out, M, N, K, a_t=a_t, b_t=b_t)
    ref = am @ bm.t()
    err = (out.double().cpu() - ref).abs().max().item()
    scale = (am.abs() @ bm.abs().t()).max().item()
    assert err <= 4e-7 * scale + 1e-6, (err, scale)


@pytest.mark.parametrize("case", [(2, 13, 13, 16, 24, 3, 3, 1, 1, 1, 1), (2, 27, 27, 8, 16, 5, 5, 1, 2, 2, 1),
                                  (3, 23, 23, 3, 8, 11, 11, 4, 0, 1, 1), (2, 9, 9, 8, 8, 3, 3, 2, 2, 1, 2)])
def test_conv_f32_matches_cpu_engine(gpu, case):
    from sparknet_amd.ops import f32dev, ref
    from sparknet_amd.ops.spec import ConvSpec
    N, H, W, C, K, R, S, st, pd, g, dil = case
    s = ConvSpec(N, H, W, C, K, R, S, st, st, pd, pd, dil, dil, g)
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(N, H, W, C, generator=gen)
    w = torch.randn(K, R, S, C // g, generator=gen) * 0.2
    b = torch.randn(K, generator=gen)
    dy = torch.randn(N, s.P, s.Q, K, generator=gen)
    y = f32dev.conv_forward(x.to(gpu), w.to(gpu), b.to(gpu), s)
    yr = ref.conv_forward(x, w, b, s)
    assert torch.allclose(y.cpu(), yr, rtol=1e-5, atol=1e-4)
    dw, db = torch.zeros(K, R, S, C // g, device=gpu), torch.zeros(K, device=gpu)
    dwr, dbr = torch.zeros_like(w), torch.zeros(K)
    dx = f32dev.conv_backward(dy.to(gpu), x.to(gpu), w.to(gpu), s, True, dw, db)
    dxr = ref.conv_backward(dy, x, w, s, True, dwr, dbr)
    for a_, b_ in ((dx, dxr), (dw, dwr), (db, dbr)):
        assert torch.allclose(a_.cpu(), b_, rtol=1e-5, atol=2e-4 * max(1.0, b_.abs().max().item())), \
            (a_.cpu() - b_).abs().max()


def _fp32_gpu_updates(fid, dev, w0, x, y):
    """bench.py --dtype fp32's step: fp32 net on the GPU, the device feeder (fp32 augment),
    eager, no fusions."""
    from sparknet_amd.core.solver import Solver
    from sparknet_amd.data.prefetch import DeviceFeeder, TensorSource
    from sparknet_amd.engine import LocalSGDTrainer, fuse_input_fold, fuse_relu
    solver = Solver(fid._solver_param(), device=dev, seed=1701, build_test_nets=False, dtype=torch.float32)
    net = solver.net
    net.flat_data.copy_(w0.to(dev))
    net.sync_compute()
    assert fuse_relu(net) == 0
    feeder = DeviceFeeder(TensorSource(x, y, fid.B, pin=True), net.blob_by_name("data"), net.blob_by_name("label"),
                          crop=227, mean=fid.MEAN, mirror=True, train=True, rng_state=net.ctx.rng_state, device=dev)
    assert not fuse_input_fold(net, feeder)
    tr = LocalSGDTrainer(solver, None, tau=1000, feeder=feeder, use_graph=False)
    tr.local_step()
    torch.cuda.synchronize()
    return fid._updates(solver, w0)


def test_caffenet_fp32_one_step_matches_cpu_engine(gpu):
    import test_bench_fidelity_gpu as fid
    x, y = fid._data(n=2 * fid.B)
    w0 = fid._initial_weights()
    uc = fid._one_step_updates(torch.device("cpu"), w0, x, y)
    ug = _fp32_gpu_updates(fid, gpu, w0, x, y)
    errs = fid._errs(ug, uc)
    bad = {}
    for k, (emax, el2) in errs.items():
        bias = k.endswith("/1")
        if el2 > (3e-3 if bias else 1e-3) or emax > (2e-2 if bias else 2e-3):
            bad[k] = (emax, el2)
    print("fp32 device vs fp32 CPU engine (max, L2):", {k: (round(a, 6), round(b, 6)) for k, (a, b) in errs.items()})
    assert not bad, bad


@pytest.mark.parametrize("case", [(2, 55, 55, 16, 3, 3, 2, 2, 0, 0), (2, 13, 15, 8, 3, 3, 2, 2, 1, 1),
                                  (3, 14, 14, 12, 3, 3, 1, 1, 1, 1), (2, 7, 7, 8, 7, 7, 1, 1, 0, 0),
                                  (2, 9, 9, 4, 2, 2, 2, 2, 0, 0)])
@pytest.mark.parametrize("method", ["max", "ave"])
def test_pool_f32_matches_reference(gpu, case, method):
    """fp32 pooling kernels (pooling_layer.cu semantics: clipped windows, ceil-mode outputs,
    AVE divisor over the padded window) against the fp32 reference formulas, both passes."""
    from sparknet_amd.ops import f32dev, ref
    from sparknet_amd.ops.spec import POOL_AVE, POOL_MAX, PoolSpec
    N, H, W, C, kh, kw, sh, sw, ph, pw = case
    s = PoolSpec(N, H, W, C, kh, kw, sh, sw, ph, pw, POOL_MAX if method == "max" else POOL_AVE)
    g = torch.Generator().manual_seed(H * 31 + C)
    x = torch.randn(N, H, W, C, generator=g)
    y, mask = f32dev.pool_forward_aux(x.to(gpu), s)
    yr = ref.pool_forward(x, s)
    assert torch.allclose(y.cpu(), yr, rtol=1e-6, atol=1e-6)
    dy = torch.randn(N, s.P, s.Q, C, generator=g)
    dx = f32dev.pool_backward(dy.to(gpu), x.to(gpu), s, mask)
    dxr = ref.pool_backward(dy, x, s)
    assert torch.allclose(dx.cpu(), dxr, rtol=1e-5, atol=1e-5)



@pytest.mark.parametrize("slope", [0.0, 0.1])
def test_relu_f32_bitwise_reference(gpu, slope):
    from sparknet_amd.ops import f32dev, ref
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 7, 9, 16, generator=g)
    x[0, 0, 0, :4] = 0.0
    dy = torch.randn(3, 7, 9, 16, generator=g)
    assert torch.equal(f32dev.relu_forward(x.to(gpu), slope).cpu(), ref.relu_forward(x, slope))
    assert torch.equal(f32dev.relu_backward(dy.to(gpu), x.to(gpu), slope).cpu(), ref.relu_backward(dy, x, slope))
