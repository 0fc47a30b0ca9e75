"""Block timeline of one dx3 launch (a tools/dx3_build_knobs.sh build with -DIDF_DX3_TL=1, loaded
through IDF_LIB_PATH): runs kbench's dx3 at one level / layer (KB_* env), then prints, over the
blocks of the LAST launch, the percentiles of each phase in microseconds (s_memrealtime, 100 MHz):
start skew, bias table, first-slab wait, k-loop, split-K hand-off (store + counter), the last
block's reduction, epilogue, and the whole block."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
os.environ.setdefault("KB_ONLY", "dx3")
os.environ.setdefault("KB_LEVELS", "2")
os.environ.setdefault("KB_LAYERS", "6")
os.environ.setdefault("KB_REPS", "1")
sys.path.insert(0, os.path.join(REPO, "tools"))
import kbench  # noqa: E402
from idfcodec._lib import lib  # noqa: E402

kbench.main()
buf = (ctypes.c_ulonglong * (4096 * 8))()
assert lib().idf_dx3_timeline(buf) == 0
rows = [[buf[b * 8 + j] for j in range(8)] for b in range(4096)]
rows = [r for r in rows if r[0]]
t0 = min(r[0] for r in rows)
end = max(max(r[5], r[6], r[3]) for r in rows)
print(f"blocks {len(rows)}  launch span {(end - t0) / 100:.2f} us")


def pct(name, vals):
    vals = sorted(v / 100.0 for v in vals)
    if not vals:
        return
    q = lambda f: vals[min(len(vals) - 1, int(f * len(vals)))]  # noqa: E731
    print(f"{name:22s} n {len(vals):5d}  p10 {q(.1):7.2f}  p50 {q(.5):7.2f}  p90 {q(.9):7.2f}  max {vals[-1]:7.2f}")


pct("start skew", [r[0] - t0 for r in rows])
pct("bias table", [r[1] - r[0] for r in rows])
pct("slab-0 wait", [r[2] - r[1] for r in rows if r[2]])
pct("k-loop", [r[3] - r[2] for r in rows if r[2]])
pct("hand-off", [r[6] - r[3] for r in rows if r[6]])
pct("last: reduction", [r[4] - r[6] for r in rows if r[4] and r[6]])
pct("epilogue", [r[5] - (r[4] or r[3]) for r in rows if r[5]])
pct("block total", [max(r[5], r[6], r[3]) - r[0] for r in rows])
pct("block end", [max(r[5], r[6], r[3]) - t0 for r in rows])
