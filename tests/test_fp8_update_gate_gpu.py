"""fp8 one-step update gate on VGG-16: every parameter's update in the
production fp8 mode against the fp32 CPU engine, bounded by the e4m3-storage floor.

Configuration: VGG-16 at batch 64, crop 64, 10 classes (the fidelity trajectory's shape,
tests/test_fp8_fidelity_gpu.py), trained first for 300 bf16 GraphStep iterations on the
template task (loss 2.33 -> 0.01), then one fp8 step; fused ReLU epilogues, ``enable_fp8``
with bench.py's defaults (layers with >= 1000 forward MACs per input element plus the e4m3
direct 64 -> 64 conv, e4m3 data gradients of the stride-1 convs, e4m3 weight gradients of
the layers that run both), the same initial weights and Philox dropout draws on both engines.

* reference: the fp32 CPU engine (Caffe's numerics, libccaffe/ccaffe.h:3);
* floor: the CPU engine with bf16 storage and e4m3 quantisation at exactly the GPU's fp8
  product operands (utils/fp8emu.py; the first fp8 iteration's scales are the tensors' own
  amax on both sides) — what e4m3 storage alone does to each update;
* gate: per parameter, the GPU update's largest deviation relative to the largest fp32
  update AND its relative L2 deviation within max(BOUND, RATIO x the floor's), and the mean
  GPU / floor ratio over all parameters <= MEAN_RATIO (no systematic error beyond e4m3);
* teeth: with the conv5_x e4m3 weight gradients made to drop 7/8 of their reduction the
  gate fails on them.

What the floor says (profiles/r6_fp8_gates.txt): e4m3 storage moves VGG-16's one-step updates
by 20-45 % (relative L2; bf16 storage alone 3-17 %), and CDNA4-style per-32-element E8M0 block
scales (fp8emu block=32) do NOT lower it (0.2-0.6): the deviation is the 3-bit mantissa's, not
the dynamic range's, so block scales were not built into the GEMM.  The GPU lands on the floor
(ratio 0.8-1.3 on the convolutions; fc8, bf16 itself but fed by fp8 layers, 1.7).

Pattern: caffe/src/caffe/test/test_gradient_based_solver.cpp:225-320 (one update against
an independently computed one)."""
import pytest
import torch

from sparknet_amd import models

pytestmark = pytest.mark.gpu

import os

B, CROP, CLASSES, NOISE, LR = 64, 64, 10, 0.8, 0.002
BOUND, RATIO, MEAN_RATIO = 0.03, 2.0, 1.3
# bf16 GPU iterations that train the initial weights first (at VGG-16's initialisation the
# first updates of the deep layers are dominated by rounding-sensitive ReLU flips: even bf16
# storage moves them by 30-40 %, which would leave a floor-relative gate without teeth)
PRETRAIN = int(os.environ.get("SN_FP8_GATE_PRETRAIN", "300"))


def _solver(dev, w0=None, dtype=None):
    from sparknet_amd.core.solver import Solver
    net_p = models.vgg16(train_batch=B, test_batch=B, crop=CROP, classes=CLASSES)
    sp = models.zoo.vgg16_solver(net_p)
    sp.base_lr = LR
    solver = Solver(sp, device=dev, seed=5, build_test_nets=False, dtype=dtype)
    if w0 is not None:
        solver.net.flat_data.copy_(w0.to(solver.net.flat_data.device))
        solver.net.sync_compute()
    return solver


def _batches(seed):
    g0 = torch.Generator().manual_seed(11)
    templates = torch.randn(CLASSES, 3, CROP, CROP, generator=g0)
    g = torch.Generator().manual_seed(seed)
    while True:
        y = torch.randint(0, CLASSES, (B,), generator=g)
        x = templates[y] + NOISE * torch.randn(B, 3, CROP, CROP, generator=g)
        yield x, y.float().view(-1, 1)


def _batch():
    return next(_batches(99))


def _pretrained(gpu):
    """fp32 masters after PRETRAIN bf16 GraphStep iterations from the seed-5 initialisation."""
    from sparknet_amd.engine import GraphStep, fuse_relu
    solver = _solver(torch.device(gpu))
    if PRETRAIN <= 0:
        return solver.net.flat_data.detach().float().cpu().clone(), []
    fuse_relu(solver.net)
    it = _batches(12)

    def pre():
        x, y = next(it)
        solver.net.blob_by_name("data").set_nchw(x)
        solver.net.blob_by_name("label").set_nchw(y)
    st = GraphStep(solver, warmup=2, pre=pre, overlap=False)
    losses = [float(st.step()) for _ in range(PRETRAIN)]
    torch.cuda.synchronize()
    return solver.net.flat_data.detach().float().cpu().clone(), losses


def _one_step(solver, x, y, w0):
    solver.net.blob_by_name("data").set_nchw(x)
    solver.net.blob_by_name("label").set_nchw(y)
    solver.step(1)
    if solver.net.device.type == "cuda":
        torch.cuda.synchronize()
    w1 = solver.net.flat_data.detach().float().cpu()
    out = {}
    for layer in solver.net.layers:
        for pi, p in enumerate(layer.params):
            if p.owner is None and p.count:
                out[f"{layer.name}/{pi}"] = w1[p.offset:p.offset + p.count] - w0[p.offset:p.offset + p.count]
    return out


def _errs(u, uc):
    return {k: (float((u[k] - c).abs().max() / (c.abs().max() + 1e-12)),
                float((u[k] - c).norm() / (c.norm() + 1e-12))) for k, c in uc.items()}


def _violations(ug, uc, floor):
    bad = []
    for k, (emax, el2) in _errs(ug, uc).items():
        fmax, fl2 = floor[k]
        if emax > max(BOUND, RATIO * fmax) or el2 > max(BOUND, RATIO * fl2):
            bad.append((k, round(emax, 4), round(el2, 4), round(fmax, 4), round(fl2, 4)))
    return bad


def _gpu_fp8_solver(gpu, w0):
    from sparknet_amd.engine import enable_fp8, fuse_relu
    solver = _solver(torch.device(gpu), w0)
    fuse_relu(solver.net)
    n = enable_fp8(solver.net, 1000.0, dgrad=True, wgrad=True)  # bench.py --dtype fp8 defaults
    assert n >= 20, n
    return solver


@pytest.fixture(scope="module")
def gate_data(gpu):
    from sparknet_amd.utils import fp8emu
    x, y = _batch()
    w0, losses = _pretrained(gpu)
    if losses:
        print(f"\npretrain: {PRETRAIN} bf16 steps, loss {sum(losses[:20]) / 20:.3f} -> {sum(losses[-20:]) / 20:.3f}")
    modes = fp8emu.fp8_modes(_gpu_fp8_solver(gpu, w0).net)
    uc = _one_step(_solver(torch.device("cpu"), w0), x, y, w0)
    emu = _solver(torch.device("cpu"), w0, dtype=torch.bfloat16)
    with fp8emu.emulate(emu.net, modes):
        ue = _one_step(emu, x, y, w0)
    ub = _one_step(_solver(torch.device("cpu"), w0, dtype=torch.bfloat16), x, y, w0)
    # what CDNA4 E8M0 block scales (32 elements along each reduction) would make of the floor
    emb = _solver(torch.device("cpu"), w0, dtype=torch.bfloat16)
    with fp8emu.emulate(emb.net, modes, block=32):
        ubk = _one_step(emb, x, y, w0)
    return x, y, w0, modes, uc, _errs(ue, uc), _errs(ub, uc), _errs(ubk, uc)


@pytest.mark.timeout(900)
def test_vgg16_fp8_one_step_updates_within_e4m3_floor(gpu, gate_data):
    x, y, w0, modes, uc, floor, bf16_floor, block_floor = gate_data
    assert sum(m[2] for m in modes.values()) >= 8  # fp8 weight gradients really run
    ug = _one_step(_gpu_fp8_solver(gpu, w0), x, y, w0)
    assert ug.keys() == uc.keys() and len(uc) == 32  # 16 learnable layers x (weight, bias)
    e = _errs(ug, uc)
    print("\nparam: fp8 GPU (max, L2) | e4m3 floor | bf16 floor | e4m3 block-32 floor")
    for k in uc:
        print(f"  {k:12s} {e[k][0]:.4f} {e[k][1]:.4f} | {floor[k][0]:.4f} {floor[k][1]:.4f} | "
              f"{bf16_floor[k][0]:.4f} {bf16_floor[k][1]:.4f} | {block_floor[k][0]:.4f} {block_floor[k][1]:.4f}"
              f"  {modes.get(k.split('/')[0], '')}")
    assert not _violations(ug, uc, floor)
    ratios = [e[k][1] / max(floor[k][1], BOUND) for k in uc]
    print(f"mean GPU / floor L2 ratio {sum(ratios) / len(ratios):.3f}")
    assert sum(ratios) / len(ratios) <= MEAN_RATIO


@pytest.mark.timeout(900)
def test_fp8_gate_catches_a_broken_fp8_wgrad(gpu, gate_data, monkeypatch):
    """The conv5_x e4m3 weight-gradient products (512 x 4608 over B x 4 x 4 pixels) drop 7/8
    of their reduction: the gate fails on conv5_3's weight."""
    from sparknet_amd.ops import gemm as G
    x, y, w0, modes, uc, floor, _, _ = gate_data
    assert modes["conv5_3"][2]
    orig = G._launch
    pixels = B * (CROP // 16) ** 2

    def broken(M, N, K, *a, **k):
        if M == 512 and N in (512 * 9, 512 * 9 + 1) and K == pixels:  # (+1: the bias ones column)
            K = K // 8
        return orig(M, N, K, *a, **k)
    monkeypatch.setattr(G, "_launch", broken)
    ug = _one_step(_gpu_fp8_solver(gpu, w0), x, y, w0)
    bad = _violations(ug, uc, floor)
    assert any(b[0] == "conv5_3/0" for b in bad), bad
