"""Summarise a rocprofv3 kernel trace: per-kernel time of one training iteration
(between the last two fused solver-update launches)."""
import csv
import sys

import os

path = sys.argv[1]
if os.path.isdir(path):
    path = os.path.join(path, "run_kernel_trace.csv")
rows = list(csv.DictReader(open(path)))


def kname(n, width=60):
    """Kernel name without 'void', the argument list or the anonymous-namespace prefix
    (splitting at the first '(' blanked every '(anonymous namespace)::' kernel)."""
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(SnGemmArgs")[0] if "gemm" in n else n.split("(")[0]
    return n[-width:]

idx = [i for i, r in enumerate(rows) if 'solver_update' in r['Kernel_Name']]
a, b = idx[-2], idx[-1]
tot = 0
agg = {}
for r in rows[a + 1:b + 1]:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += d
    n = r['Kernel_Name']
    k = kname(n)
    agg[k] = agg.get(k, 0) + d
print("per-iteration kernel time by kernel (us):")
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:25]:
    print(f"{v:9.1f}us {k}")
print(f"sum of kernel time in one iteration: {tot:.1f} us; wall {(int(rows[b]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e3:.1f} us")
if len(sys.argv) > 2:
    for r in rows[a + 1:b + 1]:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        n = r['Kernel_Name']
        if sys.argv[2] == "all" or sys.argv[2] in n:
            print(f"{d:8.1f}us grid=({int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])},{r['Grid_Size_Y']},"
                  f"{r['Grid_Size_Z']}) {kname(n, 70)}")
