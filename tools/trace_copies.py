"""Where do the __amd_rocclr_copyBuffer blits of a bench run come from? (dev tool)
usage: python tools/trace_copies.py <dir with run_kernel_trace.csv [run_memory_copy_trace.csv]>
Prints the copy count and time, per-stream counts, and the kernels that precede copies."""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(kt)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cp = [r for r in rows if "copyBuffer" in r["Kernel_Name"]]
    print("kernels", len(rows), "copyBuffer", len(cp),
          "copy ms", sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in cp) / 1e6)
    print("copy streams", collections.Counter(r.get("Stream_Id", "?") for r in cp))
    print("copy grid sizes", collections.Counter((r.get("Grid_Size", r.get("Grid_Size_X", "?")),
                                                  r.get("Workgroup_Size", r.get("Workgroup_Size_X", "?")))
                                                 for r in cp).most_common(8))
    prev = collections.Counter()
    last = None
    for r in rows:
        if "copyBuffer" in r["Kernel_Name"]:
            prev[(last or "")[:90]] += 1
        else:
            last = r["Kernel_Name"]
    print("kernel before each copy:")
    for k, v in prev.most_common(15):
        print(f"  {v:6d}  {k}")
    mt = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)
    if mt:
        m = list(csv.DictReader(open(mt[0])))
        print("memory copies", len(m), collections.Counter(r.get("Direction", "?") for r in m))
        print("sizes", collections.Counter(r.get("Bytes", "?") for r in m).most_common(10))
    # the copies inside one step: the longest gap-free window around the last encode kernel
    t0 = int(rows[0]["Start_Timestamp"])
    for r in cp[-12:]:
        print("copy at", (int(r["Start_Timestamp"]) - t0) / 1e6, "ms dur",
              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us", r.get("Stream_Id"))


if __name__ == "__main__":
    main()
