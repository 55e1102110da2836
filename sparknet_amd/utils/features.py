"""Switches of the engine's optional fusions and kernel paths.

Every switch defaults to the configuration measured fastest on MI355X (docs/PERF_NOTES.md);
they exist for numerics tests (fused vs unfused must agree) and A/B probes.  One environment
variable covers all of them, read on every query so a test can flip it in-process:

    SN_FEATURES="fuse_dropout=0,conv_packed=0"

Reference parity: Caffe has no such switches (each layer is one fixed implementation);
these only select between equivalent implementations of the same layer semantics.
"""
from __future__ import annotations

import os

DEFAULTS = {
    # engine fusion passes (engine.py)
    "fuse_pool_lrn": True,      # max pool + cross-channel LRN in one kernel each way
    "fuse_lrn_pool_bwd": True,  # LRN -> max pool: the two backwards in one kernel
    "zero_copy_concat": True,   # producers write straight into the Concat top
    "fuse_dropout": True,       # Dropout forward in the InnerProduct epilogue
    "fuse_fp8_quant": True,     # fp8 quantisation in the producing GEMM's epilogue
    "branch_depfree": True,     # dependency-free backward nodes on the least recently used stream
    "fuse_splitk": False,       # solver update sums split-K slabs (measured slower, opt-in)
    # convolution kernel selection (ops/hip.py)
    "conv_direct_c64": True,    # LDS-resident direct 3x3 conv, 64 -> 64 channels
    "conv_direct_k96": True,    # the same kernel at 96 outputs (AlexNet conv1 after the fold)
    "conv_direct96": True,      # GoogLeNet conv2/3x3 as two 96-output direct launches
    "conv_packed": True,        # tap-packed direct conv (CaffeNet conv1)
    "conv_packed44": True,      # tap-packed <4, 4> instance
    "conv_packed11": False,     # tap-packed 1x1 64 -> 64 (neutral end to end, opt-in)
    "conv_packed_k64": True,    # tap-packed <3, 64> instance (VGG-16 conv1_1 after its fold)
    "conv_direct_fp8": True,    # e4m3 direct conv for fp8 layers
    # fp8 details
    "fp8_wgrad_bias": True,     # fp8 weight-gradient bias through the e4m3 ones column
    "fp8_side_frag": True,      # per-fragment epilogues also store the fp8 side output
    "fp8_dx_only": True,        # a max pooling stores its input gradient as fp8 alone when the conv reads only that
}

_cache: tuple[str, dict] = ("", {})


def _parsed() -> dict:
    global _cache
    raw = os.environ.get("SN_FEATURES", "")
    if raw != _cache[0]:
        out = {}
        for item in filter(None, (p.strip() for p in raw.split(","))):
            name, _, val = item.partition("=")
            if name not in DEFAULTS:
                raise ValueError(f"SN_FEATURES: unknown switch {name!r} (known: {', '.join(sorted(DEFAULTS))})")
            out[name] = val.strip().lower() not in ("0", "false", "off", "no")
        _cache = (raw, out)
    return _cache[1]


def enabled(name: str) -> bool:
    if name not in DEFAULTS:
        raise KeyError(name)
    return _parsed().get(name, DEFAULTS[name])
