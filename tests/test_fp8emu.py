"""utils.fp8emu: the CPU engine's e4m3 storage emulation (the floor of the fp8 update gate,
tests/test_fp8_update_gate_gpu.py)."""
import torch

from sparknet_amd import models
from sparknet_amd.ops import ref
from sparknet_amd.utils import fp8emu


def test_quant_is_e4m3_with_current_scaling():
    g = torch.Generator().manual_seed(0)
    t = torch.randn(4096, generator=g) * 3.0
    q = fp8emu.quant(t)
    s = 448.0 / float(t.abs().max())
    # the scaled values are e4m3 numbers: a second cast changes nothing, the amax maps to 448
    assert torch.equal((q * s).to(torch.float8_e4m3fn).float(), (q * s).float().to(torch.float8_e4m3fn).float())
    assert abs(float((q * s).abs().max()) - 448.0) < 1e-3
    # 3 mantissa bits: relative error <= 2^-4 on normal values
    big = (t * s).abs() >= 2.0 ** -6
    assert float(((q - t).abs()[big] / t.abs()[big]).max()) <= 2.0 ** -4 + 1e-6
    assert torch.equal(fp8emu.quant(torch.zeros(5)), torch.zeros(5))


def _solver(dtype=None):
    from sparknet_amd.core.solver import Solver
    sp = models.solver_for("cifar10_quick", train_batch=8, test_batch=8)
    return Solver(sp, device=torch.device("cpu"), seed=3, build_test_nets=False, dtype=dtype)


def test_emulate_quantises_only_the_named_layers_and_restores():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (8, 1), generator=g).float()
    saved = (ref.conv_forward, ref.conv_backward, ref.linear_forward)

    def losses(modes):
        s = _solver(torch.bfloat16)
        s.net.blob_by_name("data").set_nchw(x)
        s.net.blob_by_name("label").set_nchw(y)
        if modes is None:
            loss = float(s.net.forward())
            s.net.backward()
        else:
            with fp8emu.emulate(s.net, modes):
                loss = float(s.net.forward())
                s.net.backward()
        grads = {ly.name: ly.params[0].diff.detach().float().clone() for ly in s.net.layers if ly.params}
        return loss, grads

    base, gb = losses(None)
    fwd, gf = losses({"conv2": (True, False, False)})
    full, gfull = losses({"conv2": (True, True, True), "ip1": (True, False, False)})
    assert (ref.conv_forward, ref.conv_backward, ref.linear_forward) == saved
    assert fwd != base and full != base
    # conv1 is upstream of every quantised product in the forward but only its backward input
    # changes; conv2's weight gradient changes under wgrad quantisation, and stays within e4m3 noise
    rel = float((gfull["conv2"] - gb["conv2"]).norm() / gb["conv2"].norm())
    assert 0.0 < rel < 0.2, rel
    # after the block every layer is back to its own methods
    s = _solver(torch.bfloat16)
    with fp8emu.emulate(s.net, {"conv1": (True, True, True)}):
        assert [ly.name for ly in s.net.layers if "forward" in vars(ly)] == ["conv1"]
    assert not any("forward" in vars(ly) or "backward" in vars(ly) for ly in s.net.layers)


def test_block_scaled_quant_tracks_local_magnitude():
    """Power-of-two scales per 32-element run along the reduction dimension: runs of tiny
    values keep their mantissas where one per-tensor scale flushes them."""
    g = torch.Generator().manual_seed(2)
    t = torch.randn(64, 96, generator=g) * torch.logspace(-6, 0, 96)  # columns span 6 decades
    qb = fp8emu.quant(t, 32, dim=0)  # blocks run down the columns: each column's own scale
    qt = fp8emu.quant(t)
    rel_b = float(((qb - t).norm(dim=0) / t.norm(dim=0)).max())
    rel_t = float(((qt - t).norm(dim=0) / t.norm(dim=0)).max())
    assert rel_b <= 2.0 ** -4 and rel_t > 0.5, (rel_b, rel_t)
    # every 32-run's scale is a power of two: q / scale is an e4m3 value
    blk = qb[:32, 5]
    sc = torch.exp2(torch.ceil(torch.log2(t[:32, 5].abs().max() / 448.0)))
    assert torch.equal((blk / sc).to(torch.float8_e4m3fn).float(), blk / sc)
    assert qb.shape == t.shape and torch.equal(fp8emu.quant(torch.zeros(3, 40), 32), torch.zeros(3, 40))
