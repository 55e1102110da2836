"""Aggregate rocprofv3 --pmc passes of scripts/newk_probe.py per kernel: MFMA utilisation
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024), as every PMC figure here), LDS bank
conflicts per LDS cycle, HBM bytes and rate."""
import csv
import glob
import re
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
dur = defaultdict(float)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(conv_packed_kernel|lrn_pool_bwd<[^>]*>|pool_lrn_fwd<[^>]*>)", r["Kernel_Name"])
        if m:
            acc[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    print(k)
    for n in sorted(c):
        print(f"   {n:28s} {c[n]:12.4g}")
    gui = c.get("GRBM_GUI_ACTIVE", 0.0)
    if gui and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        print(f"   MFMA util {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui / 8 * 1024):.3f}")
    if c.get("SQ_LDS_IDX_ACTIVE"):
        print(f"   LDS bank-conflict cycles / LDS cycles {c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.3f}")
