"""Per-layer durations of the DenseBlocks' dx3 / dxb launches from a rocprofv3 kernel trace (dev
analysis): on each stream a block's layers follow its input split (dx3_split_cols / dxb_cols),
so the n-th conv launch after a split is layer n.  Prints, per kernel instantiation and layer,
the launch count and the mean / min duration, and the share of the dx3 time each layer takes.

usage: python tools/analysis/layer_times.py run_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    skey = "Stream_Id" if rows and "Stream_Id" in rows[0] else "Queue_Id"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    layer = defaultdict(lambda: -1)
    acc = defaultdict(list)
    for r in rows:
        name, st = r["Kernel_Name"], r[skey]
        if "split_cols" in name or "dxb_cols" in name:
            layer[st] = 0
            continue
        if "conv3_dx3_kernel" not in name:
            continue
        m = re.search(r"conv3_dx3_kernel<([^>]*)>", name)
        key = (m.group(1) if m else name, layer[st])
        acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if layer[st] >= 0:
            layer[st] += 1
    tot = sum(sum(v) for v in acc.values())
    for (k, i), v in sorted(acc.items()):
        print(f"{k:24s} layer {i:3d}  n {len(v):5d}  mean {sum(v) / len(v):8.1f} us  "
              f"min {min(v):8.1f} us  share {100 * sum(v) / tot:5.1f}%")


if __name__ == "__main__":
    main()
