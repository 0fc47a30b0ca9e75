"""Sums rocprofv3 --pmc counter records of the dx3 kernel launches (dev analysis).
usage: python tools/analysis/sq_sum.py counter_collection.csv [kernel substring]"""
import csv
import sys


def main():
    sub = sys.argv[2] if len(sys.argv) > 2 else "conv3_dx3_kernel"
    acc, n = {}, {}
    for r in csv.DictReader(open(sys.argv[1])):
        if sub not in r["Kernel_Name"]:
            continue
        k = r["Counter_Name"]
        acc[k] = acc.get(k, 0.0) + float(r["Counter_Value"])
        n[k] = n.get(k, 0) + 1
    for k in sorted(acc):
        print(f"{k:28s} {acc[k]:16.0f}  (records {n[k]})")


if __name__ == "__main__":
    main()
