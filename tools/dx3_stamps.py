"""Per-slab s_memtime stamps of one dx3 block (a tools/dx3_build_knobs.sh build with
-DIDF_DX3_STAMPS=1, loaded through IDF_LIB_PATH): runs the L0 c=496 layer, then prints per wave
the mean cycles of: barrier wait (stamp 1 - 0), steps 0-8 (2 - 1), steps 9-end (3 - 2), and the
slab-to-slab period."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
os.environ.setdefault("KB_ONLY", "dx3")
os.environ.setdefault("KB_LEVELS", "0")
os.environ.setdefault("KB_LAYERS", "11")
os.environ.setdefault("KB_REPS", "3")
sys.path.insert(0, os.path.join(REPO, "tools"))
import kbench  # noqa: E402
from idfcodec._lib import lib  # noqa: E402

kbench.main()
buf = (ctypes.c_ulonglong * (8 * 40 * 4 + 8 * 6))()
assert lib().idf_dx3_stamps(buf) == 0
for w in range(8):
    rows = [[buf[(w * 40 + s) * 4 + j] for j in range(4)] for s in range(31)]
    wait = [r[1] - r[0] for r in rows[1:30]]
    a = [r[2] - r[1] for r in rows[1:30]]
    b = [r[3] - r[2] for r in rows[1:30]]
    per = [rows[s + 1][0] - rows[s][0] for s in range(1, 29)]
    m = lambda v: sum(v) / len(v)  # noqa: E731
    print(f"wave {w}: wait {m(wait):7.0f}  steps0-8 {m(a):7.0f}  steps9-end {m(b):7.0f}  period {m(per):7.0f}"
          f"  (slab0 wait {rows[0][1] - rows[0][0]})")
ph = [[buf[8 * 40 * 4 + w * 6 + j] for j in range(6)] for w in range(8)]
for w in range(8):
    p = ph[w]
    clk = (p[3] - p[0]) / max(1, p[5] - p[4]) * 100.0  # MHz: memtime ticks per 10 ns
    print(f"wave {w}: bias table {p[1] - p[0]:7d}  to loop end {p[2] - p[1]:8d}  epilogue {p[3] - p[2]:7d}"
          f"  total {p[3] - p[0]:8d} ticks  clock {clk:6.0f} MHz")
