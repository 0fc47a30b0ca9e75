"""Which processes x threads split gives the CPU baseline's best throughput on a GPU box?
Every split codes 256 images in total (bench.CpuPool, one pass after the warm-up)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

if __name__ == "__main__":
    aff, quota, usable = bench.usable_cpus()
    print(json.dumps({"affinity": len(aff), "quota": quota, "usable": usable}), flush=True)
    for split in sys.argv[1:] or ["16x1", "8x2", "4x4", "1x16", "64x4"]:
        p, t = (int(v) for v in split.split("x"))
        n = max(1, 256 // p)
        t0 = time.perf_counter()
        pool = bench.CpuPool(n, chunk=16, split=split)
        try:
            pool.wait_ready()
            start = time.perf_counter() - t0
            r = bench.cpu_baseline_pool(pool, runs=1)
        finally:
            pool.close()
        print(json.dumps({"split": split, "images": p * n, "startup_s": round(start, 1),
                          "mpx_s": r["value"], "effective_cpus": r["effective_cpus"],
                          "sample": r["sample"]}), flush=True)
