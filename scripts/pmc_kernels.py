#!/usr/bin/env python3
"""Per-dispatch averages of rocprofv3 --pmc counters by kernel (template arguments kept,
parameter list dropped), over every pass directory given.

    python scripts/pmc_kernels.py gpurun_out/pmc_pool/pA gpurun_out/pmc_pool/pB [--match pool]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    args = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in args.dirs:
        for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                if args.match and args.match not in name:
                    continue
                acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[(name, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "?")))
    for name, c in sorted(acc.items()):
        print(name)
        for k in sorted(c):
            n = max(1, len(disp[(name, k)]))
            print(f"   {k:30s} {c[k] / n:14.5g}  (per dispatch, {n} dispatches)")


if __name__ == "__main__":
    main()
