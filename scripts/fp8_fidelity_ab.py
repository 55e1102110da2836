"""A/B of the fp8 training-fidelity components: the 200-step VGG-16-small
trajectory of tests/test_fp8_fidelity_gpu.py under one fp8 variant at a time, against bf16
and the bf16alt chaos floor.

python scripts/fp8_fidelity_ab.py [lr]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

import test_fp8_fidelity_gpu as T  # noqa: E402
from sparknet_amd import engine  # noqa: E402
from sparknet_amd.ops import hip  # noqa: E402


class MP:
    """minimal monkeypatch stand-in"""
    def __init__(self):
        self.undo = []

    def setattr(self, obj, name, val):
        self.undo.append((obj, name, getattr(obj, name)))
        setattr(obj, name, val)

    def close(self):
        for obj, name, val in reversed(self.undo):
            setattr(obj, name, val)
        self.undo = []


if len(sys.argv) > 1:
    T.LR = float(sys.argv[1])
dev = torch.device("cuda:0")
orig_enable = engine.enable_fp8
res = {}


def run(mode, label, **kw):
    mp = MP()
    if "wgrad" in kw:
        mp.setattr(engine, "enable_fp8", lambda net, m, **a: orig_enable(net, m, **{**a, "wgrad": kw["wgrad"]}))
    if "bias" in kw:
        mp.setattr(hip, "FP8_WGRAD_BIAS", kw["bias"])
    if "history" in kw:
        mp.setattr(hip, "FP8_HISTORY", kw["history"])
    try:
        losses, n8 = T._trajectory(mode, dev, mp)
    finally:
        mp.close()
    res[label] = T._smooth(losses)
    print(label, n8, [round(v, 3) for v in res[label]], flush=True)


run("bf16", "bf16")
run("bf16alt", "bf16alt")
run("fp8", "fp8 default (fwd+dgrad+wgrad, exact bias, history 16)")
run("fp8", "fp8 no wgrad", wgrad=False)
run("fp8", "fp8 fused e4m3 bias column", bias=True)
run("fp8", "fp8 history 1 (current scaling)", history=1)
sb = res["bf16"]
for k, v in res.items():
    print(f"{k:55s} max dev vs bf16 {max(abs(a - b) for a, b in zip(sb, v)):.3f}  last {v[-1]:.3f}", flush=True)
