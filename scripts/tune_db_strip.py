#!/usr/bin/env python3
"""Drop the GEMM tuning-database entries of one product family so the next tuning pass
(bench.py --autotune --save-tuned DB) re-times them, e.g. after a mainloop or stager
change.  Families: wgrad (MC dense A x MC implicit-im2col B: the conv weight gradients).

    python scripts/tune_db_strip.py DB.json wgrad
"""
import ast
import json
import sys

FAMILIES = {"wgrad": lambda k: k[4] == 1 and k[5] == 0 and k[6] == 1 and k[7] == 1}


def main():
    path, fam = sys.argv[1], sys.argv[2]
    pred = FAMILIES[fam]
    with open(path) as f:
        db = json.load(f)
    keep = {k: v for k, v in db.items() if not pred(ast.literal_eval(k))}
    with open(path, "w") as f:
        json.dump(dict(sorted(keep.items())), f, indent=0)
    print(f"{path}: dropped {len(db) - len(keep)} {fam} entries, {len(keep)} left")


if __name__ == "__main__":
    main()
