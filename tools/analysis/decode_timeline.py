"""Where a bench step's decode spends its time, from a rocprofv3 kernel trace (dev analysis).

The decode of step k runs from its first rans_decode_kernel launch to the next step's first
dequant (the encode's first kernel).  The interval is cut into: time the GPU runs only serial
rANS decode kernels ("rANS only": the chains nothing overlaps), time with no kernel at all
(idle), and time with other work; and per decode level (by the rANS launch's grid size) the
rANS launches' start, end and what ran beside them.

usage: python tools/analysis/decode_timeline.py run_kernel_trace.csv [step index, default 1]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ev = []
    for r in csv.DictReader(open(path)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                   r.get("Stream_Id", r.get("Queue_Id", ""))))
    ev.sort()
    deq = [e[0] for e in ev if "dequant" in e[2]]
    a = deq[k]
    d0 = min(e[0] for e in ev if "rans_decode_kernel" in e[2] and e[0] > a)
    ends = [t for t in deq if t > d0]
    d1 = ends[0] if ends else max(e[1] for e in ev)
    seg = [e for e in ev if d0 <= e[0] < d1]
    pts = sorted([(s, 1, "rans" in n) for s, _, n, _ in seg] + [(e, -1, "rans" in n) for _, e, n, _ in seg])
    cur_r = cur_o = 0
    last = d0
    t_rans_only = t_idle = t_other = 0
    for t, d, isr in pts:
        t = min(max(t, d0), d1)
        dt = t - last
        if cur_o > 0:
            t_other += dt
        elif cur_r > 0:
            t_rans_only += dt
        else:
            t_idle += dt
        last = t
        if isr:
            cur_r += d
        else:
            cur_o += d
    tot = d1 - d0
    print(f"decode step {k}: {tot / 1e6:.3f} ms  rANS only {t_rans_only / 1e6:.3f} ms  "
          f"idle {t_idle / 1e6:.3f} ms  other work {t_other / 1e6:.3f} ms")
    print("rANS decode launches (start, end ms from the decode start; stream):")
    for s, e, n, q in seg:
        if "rans_decode_kernel" in n:
            print(f"  {(s - d0) / 1e6:7.3f} {(e - d0) / 1e6:7.3f}  ({(e - s) / 1e6:.3f} ms) q={q}")
    # the encode before it: dequant .. the decode's first rANS launch (serial runs only)
    eseg = [e for e in ev if a <= e[0] < d0]
    e_end = max(e[1] for e in eseg)
    busy = sorted((s, e) for s, e, _, _ in eseg)
    covered, cs, ce = 0, busy[0][0], busy[0][1]
    for s, e in busy[1:]:
        if s > ce:
            covered += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    covered += ce - cs
    rans_e = [(s, e) for s, e, n, _ in eseg if "rans_encode_kernel" in n]
    print(f"encode before it: {(e_end - a) / 1e6:.3f} ms to its last kernel end, GPU busy "
          f"{covered / 1e6:.3f} ms; rANS encode launches: " +
          ", ".join(f"{(s - a) / 1e6:.2f}-{(e - a) / 1e6:.2f}" for s, e in rans_e))
    # per decode level: the last kernel of the decode before each rANS launch, the gap
    conv = [e for e in seg if "conv3" in e[2]]
    if conv:
        print(f"decode: first conv {(conv[0][0] - d0) / 1e6:.3f} ms, last conv end "
              f"{(max(e[1] for e in conv) - d0) / 1e6:.3f} ms, last kernel end "
              f"{(max(e[1] for e in seg) - d0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
