#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv): mean
counter value per kernel instantiation (short name), plus derived metrics:
MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs) — the one
normalisation used for every PMC figure in this repo (GRBM_GUI_ACTIVE sums the 8 XCDs'
active cycles; MFMA busy cycles sum over all 1024 SIMDs), L2 hit %, LDS conflict
ratio, fetched bytes (FETCH_SIZE is reported x2 per MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"


def short(name, grid=""):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    head = name.split("(")[0] if not name.startswith("void (") else name[5:].split(")(")[0]
    head = re.sub(r"^void ", "", head)
    head = head if len(head) < 90 else head[:90]
    return f"{head} grid={grid}"


agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
order = []
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"], r["Grid_Size"])
        if k not in order:
            order.append(k)
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["_vgpr"] = [float(r["VGPR_Count"])]
        agg[k]["_agpr"] = [float(r.get("Accum_VGPR_Count", 0) or 0)]
        agg[k]["_lds"] = [float(r["LDS_Block_Size"])]
CUS = 256
for k in order:
    d = {c: sum(v) / len(v) for c, v in agg[k].items()}
    if "SQ_WAVES" not in d and "FETCH_SIZE" not in d:
        continue
    out = [k]
    if "GRBM_GUI_ACTIVE" in d and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
        out.append(f"mfma_util={100 * d['SQ_VALU_MFMA_BUSY_CYCLES'] / (d['GRBM_GUI_ACTIVE'] / 8 * 4 * CUS):.1f}%")
        out.append(f"gui_cycles={d['GRBM_GUI_ACTIVE']:.0f}")
    if "TCC_HIT_sum" in d:
        out.append(f"L2_hit={100 * d['TCC_HIT_sum'] / max(1, d['TCC_HIT_sum'] + d['TCC_MISS_sum']):.1f}%")
    if "SQ_LDS_BANK_CONFLICT" in d:
        out.append(f"lds_conflict_cyc={d['SQ_LDS_BANK_CONFLICT']:.3g} lds_insts={d.get('SQ_INSTS_LDS', 0):.3g}")
    if "FETCH_SIZE" in d:
        out.append(f"fetch_MB(x2)={2 * d['FETCH_SIZE'] / 1024:.1f}")
    if "WRITE_SIZE" in d:
        out.append(f"write_MB={d['WRITE_SIZE'] / 1024:.1f}")
    for c in ("TA_BUSY_avr", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_INSTS_VALU",
              "SQ_INSTS_MFMA"):
        if c in d:
            out.append(f"{c}={d[c]:.3g}")
    out.append(f"vgpr={d['_vgpr']:.0f}/{d['_agpr']:.0f} lds={d['_lds']:.0f}")
    print("  ".join(out))
