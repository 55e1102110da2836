#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc passes (gpurun_out/pmct/p*/run_counter_collection.csv) per GEMM
kernel template (gemm*_kernel<...>) and print MFMA utilisation and instruction mix per MFMA."""
import csv
import glob
import re
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmct"
acc = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(gemm\w*kernel<[^>]*>|splitk_reduce\w*)", r["Kernel_Name"])
        if not m:
            continue
        acc[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    mf = c.get("SQ_INSTS_MFMA", 0.0)
    gui = c.get("GRBM_GUI_ACTIVE", 0.0)
    util = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 1024) if gui else 0.0
    print(k)
    for n in sorted(c):
        print(f"   {n:32s} {c[n]:12.4g}")
    if mf:
        print(f"   MFMA util {util:.3f} | non-MFMA VALU/MFMA {(c.get('SQ_INSTS_VALU', 0) - mf) / mf:.2f}  "
              f"SALU/MFMA {c.get('SQ_INSTS_SALU', 0) / mf:.2f}  LDS/MFMA {c.get('SQ_INSTS_LDS', 0) / mf:.2f}  "
              f"VMEM/MFMA {c.get('SQ_INSTS_VMEM', 0) / mf:.3f}")
