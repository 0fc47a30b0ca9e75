"""Do the decode's rANS kernels slow the other lane's / the next encode's convs (dev analysis)?
A rans_decode block holds 75 KiB of LDS, so a CU running one cannot also hold an L0 dx3 block
(149.5 KiB): per layer of the L0 dx3 kernel, compares launches that ran beside a rANS decode
kernel for most of their time with launches that did not, split by whether another conv launch
overlapped them.

usage: python tools/analysis/overlap.py run_kernel_trace.csv"""
import csv
import re
import sys
from collections import defaultdict


def overlap(a0, a1, b0, b1):
    return max(0, min(a1, b1) - max(a0, b0))


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    skey = "Stream_Id" if rows and "Stream_Id" in rows[0] else "Queue_Id"
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[skey])
                for r in rows)
    dec = [(s, e) for s, e, n, _ in ev if "rans_decode_kernel" in n]
    convs = [(s, e, n, q) for s, e, n, q in ev if "conv3_dx3_kernel" in n]
    layer = defaultdict(lambda: -1)
    out = defaultdict(list)
    for s, e, n, q in ev:
        if "split_cols" in n or "dxb_cols" in n:
            layer[q] = 0
            continue
        if "conv3_dx3_kernel<3, 4, 18, 11" not in n:
            if "conv3_dx3_kernel" in n and layer[q] >= 0:
                layer[q] += 1
            continue
        d = e - s
        od = sum(overlap(s, e, a, b) for a, b in dec)
        oc = sum(overlap(s, e, a, b) for a, b, _, qq in convs if (a, b) != (s, e) or qq != q)
        key = ("rans" if od > d / 2 else "no-rans", "conv" if oc > d / 4 else "alone")
        out[(layer[q], key)].append(d / 1e3)
        if layer[q] >= 0:
            layer[q] += 1
    for (li, key), v in sorted(out.items()):
        print(f"L0 layer {li:3d} {key[0]:8s} {key[1]:6s} n {len(v):4d} mean {sum(v) / len(v):8.1f} us")


if __name__ == "__main__":
    main()
