"""ISA check of the reproducer's four head-init forms (head_init_variants.s): for each kernel,
the instructions between its table fill (ds_write / buffer_load ... lds) and the first s_barrier,
and whether a wait covering the fill (lgkmcnt(0) for ds_write, vmcnt(0) for LDS-DMA) is among them.
usage: python tools/repro_lds/check_isa.py [tools/repro_lds/head_init_variants.s]"""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "tools/repro_lds/head_init_variants.s"
src = open(path).read().splitlines()
kern = None
out = {}
for ln in src:
    m = re.match(r"^(_Z\w*head_init_lds\w*):", ln)
    if m:
        kern = m.group(1)
        out[kern] = {"fill": [], "between": [], "barrier": False}
        continue
    if kern is None or out[kern]["barrier"]:
        continue
    s = ln.strip()
    if s.startswith(";") or not s or s.startswith("."):
        continue
    k = out[kern]
    if s.startswith("ds_write") or (s.startswith("buffer_load") and s.endswith(" lds")):
        k["fill"].append(s)
        k["between"] = []
    elif s.startswith("s_barrier"):
        k["barrier"] = True
    elif k["fill"]:
        k["between"].append(s)
ok_all = True
for name, k in out.items():
    v = int(re.search(r"ILi(\d)E", name).group(1))
    dma = any(f.startswith("buffer_load") for f in k["fill"])
    need = "vmcnt(0)" if dma else "lgkmcnt(0)"
    waited = any(s.startswith("s_waitcnt") and need in s for s in k["between"])
    expect = v in (2, 4)
    ok_all &= waited == expect
    print(f"variant {v}: fill {'LDS-DMA' if dma else 'ds_write'} x{len(k['fill'])}, "
          f"{need} before s_barrier: {'yes' if waited else 'NO'} "
          f"(between: {[s.split()[0] + (' ' + s.split()[1] if s.startswith('s_waitcnt') else '') for s in k['between']]})")
print("isa check", "ok" if ok_all else "FAILED")
sys.exit(0 if ok_all else 1)
