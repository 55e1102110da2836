"""Register-pressure guard for the HIP kernels (no GPU needed): the build records each
kernel's compiler resource report (``-Rpass-analysis=kernel-resource-usage``,
``sparknet_amd/build_native.py``) next to its object file; no GEMM / convolution kernel the
engine can select may use scratch memory.

Why: round 5 added an in-launch split-K combine to the GEMM epilogue whose second register
tile made every 256x256 / 256x192 tile spill 170-450 VGPRs into scratch inside the K-loop —
VGG-16's weight gradients ran 2x slower (8.6k -> 4.2k img/s) while every numerics test still
passed.  (Round 6 removed the measured-and-rejected A/B families that were exempt: the
persistent ring tiles and the 8-phase 256x256 schedule.)"""
import json
from pathlib import Path

import pytest

OBJ = Path(__file__).resolve().parent.parent / "build" / "obj"
ALLOWED_SCRATCH_TUS: set = set()


def _reports():
    return sorted(OBJ.glob("kernels_*.hip.resources.json")) if OBJ.exists() else []


def test_resource_reports_parse():
    from sparknet_amd.build_native import _resources
    err = ("a.hip:3:1: remark: Function Name: _Z1kv [-Rpass-analysis=kernel-resource-usage]\n"
           "a.hip:3:1: remark:     VGPRs: 134 [-Rpass-analysis=kernel-resource-usage]\n"
           "a.hip:3:1: remark:     ScratchSize [bytes/lane]: 16 [-Rpass-analysis=kernel-resource-usage]\n"
           "a.hip:3:1: remark:     VGPRs Spill: 4 [-Rpass-analysis=kernel-resource-usage]\n")
    assert _resources(err) == {"_Z1kv": {"vgpr": 134, "scratch": 16, "vgpr_spill": 4}}


def test_every_hip_object_has_a_current_report():
    """A stale or missing report would let the spill guard below pass on old data."""
    objs = sorted(OBJ.glob("kernels_*.hip.o")) if OBJ.exists() else []
    if not objs:
        pytest.skip("no built HIP objects (run sparknet_amd.build_native.build() first)")
    bad = []
    for o in objs:
        rep = o.with_suffix(".resources.json")
        if not rep.exists():
            bad.append((o.name, "missing"))
        elif rep.stat().st_mtime < o.stat().st_mtime:
            bad.append((o.name, "older than the object"))
    assert not bad, bad


def test_no_selectable_kernel_uses_scratch():
    reports = _reports()
    if not reports:
        pytest.skip("no build resource reports (run sparknet_amd.build_native.build() first)")
    bad = []
    for rep in reports:
        tu = rep.name.split(".")[0]
        if tu in ALLOWED_SCRATCH_TUS:
            continue
        for name, r in json.loads(rep.read_text()).items():
            if r.get("scratch", 0) > 0 or r.get("vgpr_spill", 0) > 0:
                bad.append((tu, name[-90:], r))
    assert not bad, bad[:10]
