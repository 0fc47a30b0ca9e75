"""CU occupancy of a bench run from a rocprofv3 kernel trace (dev analysis), for pipelined runs
too: every kernel is taken to hold min(256, its workgroups) CUs while it runs (the convs run one
512-thread block per CU), and the timeline of the sum over concurrent kernels, capped at 256,
gives the CU-time in use over the window from the first to the last dequant launch (the timed
steps' encodes).  Also prints each kernel family's CU-time share and the busy-CU histogram.

usage: python tools/analysis/cu_util.py run_kernel_trace.csv [first dequant index, default 3]
"""
import csv
import re
import sys
from collections import Counter, defaultdict


def family(name):
    m = re.search(r"conv3_dx3_kernel<([^>]*)>", name)
    if m:
        return "dx3<" + m.group(1) + ">"
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) if m else name[:40]


def main():
    path = sys.argv[1]
    k0 = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ev = []
    for r in csv.DictReader(open(path)):
        blocks = max(1, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                   min(256, blocks)))
    ev.sort()
    marks = [e[0] for e in ev if "dequant" in e[2]]
    a, b = marks[k0], marks[-1]
    seg = [e for e in ev if a <= e[0] < b]
    pts = sorted([(s, c) for s, _, _, c in seg] + [(min(e, b), -c) for _, e, _, c in seg])
    cur, last, acc, busy = 0, a, 0, 0
    hist = Counter()
    for t, d in pts:
        if t > last:
            acc += (t - last) * min(256, cur)
            busy += (t - last) if cur > 0 else 0
            hist[min(256, cur) // 64 * 64] += t - last
            last = t
        cur += d
    span = b - a
    print(f"window {span / 1e6:.2f} ms ({len(marks) - 1 - k0} encodes): CU-time in use "
          f"{100 * acc / (span * 256):.1f}%, some kernel running {100 * busy / span:.1f}%")
    for c in sorted(hist):
        print(f"  {c:3d}-{min(c + 63, 256):3d} CUs busy: {100 * hist[c] / span:5.1f}% of the window")
    fam = defaultdict(float)
    for s, e, n, c in seg:
        fam[family(n)] += (min(e, b) - s) * c
    tot = sum(fam.values())
    for n, v in sorted(fam.items(), key=lambda x: -x[1])[:12]:
        print(f"  {100 * v / tot:5.1f}% of kernel CU-time  {n}")


if __name__ == "__main__":
    main()
