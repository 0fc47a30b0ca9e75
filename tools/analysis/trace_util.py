"""Chip utilisation of one bench step from a rocprofv3 kernel trace (dev analysis).

A step runs from one dequant launch (the start of an encode) to the next.  Every kernel is
taken to hold min(256, its workgroups) CUs while it runs (the convs run one 512-thread block
per CU; the serial rANS passes a handful of waves per CU at most), and the timeline of the sum
over concurrent kernels, capped at 256, gives the CU-time actually in use -- the share of the
step each half (encode: up to the first rans_decode_kernel launch; decode: the rest) leaves idle.
Run it on a --pipeline 0 trace: pipelined steps overlap an encode with a decode.

usage: python tools/analysis/trace_util.py run_kernel_trace.csv [step index, default 2]
"""
import csv
import sys
from collections import Counter


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ev = []
    for r in csv.DictReader(open(path)):
        blocks = max(1, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                   min(256, blocks)))
    ev.sort()
    marks = [e[0] for e in ev if "dequant" in e[2]]
    a, b = marks[k], marks[k + 1]
    seg = [e for e in ev if a <= e[0] < b]
    pts = sorted([(s, c) for s, _, _, c in seg] + [(e, -c) for _, e, _, c in seg])
    dp = min(e[0] for e in seg if "rans_decode_kernel" in e[2])

    def util(x, y):
        cur, last, acc = 0, x, 0
        for t, d in pts:
            if t <= x:
                cur += d
                continue
            if t > y:
                break
            acc += (t - last) * min(256, cur)
            cur += d
            last = t
        acc += (y - last) * min(256, cur)
        return acc / ((y - x) * 256)

    print(f"step {k}: {(b - a) / 1e6:.2f} ms, CU-time in use {100 * util(a, b):.1f}%")
    print(f"  encode {(dp - a) / 1e6:.2f} ms {100 * util(a, dp):.1f}%   "
          f"decode {(b - dp) / 1e6:.2f} ms {100 * util(dp, b):.1f}%")
    hist, cur, last = Counter(), 0, a
    for t, d in pts:
        if t > b:
            break
        if t > a:
            hist[min(256, cur) // 64 * 64] += t - last
            last = t
        cur += d
    for c in sorted(hist):
        print(f"  {c:3d}-{min(c + 63, 256):3d} CUs busy: {hist[c] / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
