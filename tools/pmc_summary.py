"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel (and grid size), the mean
of every counter over its dispatches.  Usage: python tools/pmc_summary.py DIR [kernel-substr]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "**", "*.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if "Counter_Name" not in r:  # agent-info and other non-counter CSVs
                break
            k = r.get("Kernel_Name", "")
            if sub not in k:
                continue
            key = (k[:90], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (k, grid), cs in sorted(vals.items(), key=lambda kv: kv[0][1]):
        print(f"{k}  grid={grid}")
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} n={len(v):4d} mean={sum(v) / len(v):.4g}")


if __name__ == "__main__":
    main()
