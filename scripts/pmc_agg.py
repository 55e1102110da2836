#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter CSVs (p*/run_counter_collection.csv) per kernel:
mean counter value per dispatch of the GEMM kernels."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm" not in k and "splitk" not in k and "Cijk" not in k:
            continue
        k = k.replace("(anonymous namespace)::", "").split("(SnGemmArgs")[0].split("(")[0][-70:]
        if "--by-grid" in sys.argv:
            k += (f"  grid={r.get('Grid_Size', '?')} wg={r.get('Workgroup_Size', '?')} lds={r.get('LDS_Block_Size', '?')}"
                  f" vgpr={r.get('VGPR_Count', '?')} agpr={r.get('Accum_VGPR_Count', '?')}")
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(m):
        print(f"   {c:30s} {m[c]:14.4g}")
    g = m.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CU_CYCLES" in m:
        # GRBM_GUI_ACTIVE sums the 8 XCDs; busy cycles sum the 1024 SIMDs (scripts/pmc_summary.py)
        print(f"   MFMA util = MFMA_BUSY / (GUI_ACTIVE / 8 x 1024 SIMD) = {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.3f}")
