"""Which HIP API calls launch the __amd_rocclr_copyBuffer kernels (dev analysis): joins a
rocprofv3 --kernel-trace --hip-trace run's kernel records to the API records by correlation id
and counts the copy kernels per API function (and per size bucket).

usage: python tools/copy_trace.py <rocprofv3 output dir>"""
import csv
import glob
import sys
from collections import Counter


def main():
    d = sys.argv[1]
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    ht = glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0]
    api = {}
    for r in csv.DictReader(open(ht)):
        api[r["Correlation_Id"]] = r["Function"]
    cnt, dur = Counter(), Counter()
    n = 0
    for r in csv.DictReader(open(kt)):
        if "copyBuffer" not in r["Kernel_Name"] and "fillBuffer" not in r["Kernel_Name"]:
            continue
        n += 1
        f = api.get(r["Correlation_Id"], "?")
        key = (r["Kernel_Name"][:32], f, int(r["Grid_Size_X"]))
        cnt[key] += 1
        dur[key] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"{n} copy / fill kernels")
    for k, v in cnt.most_common(20):
        print(f"{v:6d}  {dur[k] / v / 1e3:8.1f} us avg  {k}")


if __name__ == "__main__":
    main()
