#!/usr/bin/env python3
"""Critical-path view of one training iteration from a rocprofv3 kernel trace: per queue
(HIP stream) the busy time, the idle gaps while other queues run, and the wall-clock share
during which 0 / 1 / 2 / 3+ kernels are in flight.  The iteration is delimited like
prof_summary.py (between the last two solver-update launches).

    python scripts/stream_timeline.py <run_kernel_trace.csv | dir> [--top 25]
"""
import argparse
import csv
import os
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--iters", action="store_true", help="also list every iteration's wall, idle total and largest gap")
    args = ap.parse_args()
    path = args.path
    if os.path.isdir(path):
        path = os.path.join(path, "run_kernel_trace.csv")
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("empty trace")
        return 1
    qkey = next((k for k in ("Queue_Id", "Stream_Id", "Queue_ID") if k in rows[0]), None)
    idx = [i for i, r in enumerate(rows) if "solver_update" in r["Kernel_Name"]]
    if len(idx) < 2:
        print("fewer than two solver-update launches in the trace")
        return 1
    if args.iters:
        for j in range(len(idx) - 1):
            its = rows[idx[j] + 1:idx[j + 1] + 1]
            sp = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in its)
            reach, rk, tot, big = sp[0][1], sp[0], 0, (0, None, None)
            for x in sp[1:]:
                if x[0] > reach:
                    tot += x[0] - reach
                    if x[0] - reach > big[0]:
                        big = (x[0] - reach, rk, x)
                if x[1] > reach:
                    reach, rk = x[1], x
            nm = (lambda k: k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-40:])
            where = f"{nm(big[1][2])} -> {nm(big[2][2])}" if big[1] else ""
            print(f"iter {j}: wall {(sp[-1][1] - sp[0][0]) / 1e3:8.1f} us, {len(its)} launches, idle {tot / 1e3:7.1f} us, "
                  f"largest gap {big[0] / 1e3:7.1f} us {where}")
    a, b = idx[-2], idx[-1]
    it = rows[a + 1:b + 1]
    t0 = min(int(r["Start_Timestamp"]) for r in it)
    t1 = max(int(r["End_Timestamp"]) for r in it)
    wall = (t1 - t0) / 1e3
    per_q = {}
    ev = []
    for r in it:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get(qkey, "?") if qkey else "?"
        per_q.setdefault(q, []).append((s, e, r["Kernel_Name"]))
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    occ = {}
    cur, last = 0, t0
    for t, d in ev:
        if t > last:
            occ[min(cur, 3)] = occ.get(min(cur, 3), 0) + (t - last)
        cur += d
        last = t
    # idle intervals (no kernel of the iteration in flight) and the launches on either side
    spans = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get(qkey, "?") if qkey else "?",
                    r["Kernel_Name"]) for r in it)
    gaps = []
    reach, reach_k = spans[0][1], spans[0]
    for sp in spans[1:]:
        if sp[0] > reach:
            gaps.append((sp[0] - reach, reach_k, sp))
        if sp[1] > reach:
            reach, reach_k = sp[1], sp

    def short(n):
        n = n.replace("(anonymous namespace)::", "").replace("void ", "")
        return (n.split("(SnGemmArgs")[0] if "gemm" in n else n.split("(")[0])[-48:]
    gaps.sort(reverse=True)
    print(f"idle gaps: {len(gaps)}, total {sum(g[0] for g in gaps) / 1e3:.1f} us; largest:")
    for g, a_, b_ in gaps[:12]:
        print(f"  {g / 1e3:7.1f} us  after q{a_[2]} {short(a_[3])}  ->  q{b_[2]} {short(b_[3])}")
    hist = {}
    for g, _, _ in gaps:
        k = 0 if g < 2000 else (1 if g < 5000 else (2 if g < 20000 else 3))
        hist[k] = hist.get(k, 0) + 1
    print("  gap sizes: " + ", ".join(f"{lbl}: {hist.get(i, 0)}" for i, lbl in
                                       enumerate(("<2us", "2-5us", "5-20us", ">=20us"))))
    print(f"iteration wall {wall:.1f} us, {len(it)} launches, queue column {qkey!r}")
    print("in flight: " + "  ".join(f"{k}{'+' if k == 3 else ''}: {100.0 * v / 1e3 / wall:.1f} %"
                                    for k, v in sorted(occ.items())))
    for q, ks in sorted(per_q.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1])):
        busy = sum(e - s for s, e, _ in ks) / 1e3
        print(f"queue {q}: {len(ks)} launches, busy {busy:.1f} us ({100.0 * busy / wall:.1f} % of wall)")
    # the longest launches and what else ran beside them
    print(f"top {args.top} launches (us, overlap with other queues %):")
    flat = [(e - s, s, e, q, n) for q, ks in per_q.items() for s, e, n in ks]
    flat.sort(reverse=True)
    for d, s, e, q, n in flat[:args.top]:
        ov = 0
        for q2, ks in per_q.items():
            if q2 == q:
                continue
            for s2, e2, _ in ks:
                ov += max(0, min(e, e2) - max(s, s2))
        name = n.replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(SnGemmArgs")[0] if "gemm" in name else name.split("(")[0]
        print(f"  {d / 1e3:8.1f}  q{q}  ovl {100.0 * min(ov, d) / max(d, 1):5.1f}%  {name[-70:]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
