"""Host-side eligibility rules of the round-6 kernel paths (no GPU needed):
* hip.packed3x3k64_ok — VGG-16 conv1_1 after its fold on the tap-packed <3, 64> kernel;
* hip.conv_dy_fp8_only_ok — when a max pooling may store the conv's output gradient as fp8 alone
  (engine.fuse_fp8_quant fp8_dx_only).
Reference for the layers: caffe/src/caffe/layers/conv_layer.cu:8-53, pooling_layer.cu:217-260."""
from types import SimpleNamespace

from sparknet_amd.ops import hip
from sparknet_amd.ops.spec import ConvSpec


def test_packed3x3k64_eligibility():
    vgg = ConvSpec(2, 224, 224, 3, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1)
    folded = hip.s2d_plan(vgg)[4]
    assert hip.packed3x3k64_ok(folded)
    assert not hip.packed3x3k64_ok(ConvSpec(2, 226, 226, 16, 64, 3, 3, 1, 1, 0, 0, 1, 1, 1))  # C != 8
    assert not hip.packed3x3k64_ok(ConvSpec(2, 226, 226, 8, 64, 3, 3, 1, 1, 1, 1, 1, 1, 1))  # pad 1
    assert not hip.packed3x3k64_ok(ConvSpec(2, 226, 226, 8, 96, 3, 3, 1, 1, 0, 0, 1, 1, 1))  # K != 64
    assert not hip.packed3x3k64_ok(ConvSpec(1, 8, 2000, 8, 64, 3, 3, 1, 1, 0, 0, 1, 1, 1))   # patch > LDS tile


def _layer(dgrad=True, wgrad=True, bias=True, need_w=True, need_b=True):
    lay = SimpleNamespace(fp8_dgrad_slots=(0, 1) if dgrad else None, fp8_wgrad=wgrad,
                          bias=object() if bias else None)
    lay.param_grads_needed = lambda i: need_w if i == 0 else need_b
    return lay


def test_conv_dy_fp8_only_eligibility():
    s = ConvSpec(4, 56, 56, 128, 128, 3, 3, 1, 1, 1, 1, 1, 1, 1)  # a VGG block conv (kred 1152)
    assert hip.conv_dy_fp8_only_ok(_layer(), s)
    assert not hip.conv_dy_fp8_only_ok(_layer(dgrad=False), s)          # bf16 data gradient
    assert not hip.conv_dy_fp8_only_ok(_layer(wgrad=False), s)          # bf16 weight gradient reads dy
    assert hip.conv_dy_fp8_only_ok(_layer(wgrad=False, need_w=False, bias=False), s)  # no weight gradient
    assert not hip.conv_dy_fp8_only_ok(_layer(need_w=False), s)         # bias alone: an exact column sum
    s2 = ConvSpec(4, 56, 56, 128, 128, 3, 3, 2, 2, 1, 1, 1, 1, 1)       # stride 2: no flip-path dgrad
    assert not hip.conv_dy_fp8_only_ok(_layer(), s2)
