"""LDS ordering audit of libidfcodec's device code: for every s_barrier of every kernel, the waits
that directly precede it (scanning back within its basic block to the previous memory
instruction), against the LDS writers the kernel holds -- ds_write* (counted by lgkmcnt) and
LDS-DMA (buffer_load ... lds, counted by vmcnt).  A gfx950 s_barrier waits for neither counter,
so a barrier that orders LDS writes before other waves' reads needs the writer's counter drained
first (or the writes drained by earlier waits on the same wave, which this scan does not prove:
such barriers are listed for review).
usage: python tools/repro_lds/barrier_audit.py [out.txt]   (compiles csrc/*.hip to assembly)"""
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(REPO, "finalproject-losslessimagecompression_amd", "csrc")
MEM = re.compile(r"^(ds_|buffer_|global_|flat_|scratch_|s_load|s_buffer_load|s_store|s_atomic)")


def kernels(asm):
    kern, body = None, []
    for ln in asm.splitlines():
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", ln)
        if m and ".Lfunc_end" not in ln:
            if kern:
                yield kern, body
            kern, body = m.group(1), []
            continue
        if kern and ln.startswith(".Lfunc_end"):
            yield kern, body
            kern, body = None, []
            continue
        if kern:
            body.append(ln.strip())
    if kern:
        yield kern, body


def audit(asm):
    """Per s_barrier: the window of instructions since the previous s_barrier or branch label.
    A writer in the window must be followed by a drain of its counter before the barrier
    ("writer not drained": a hazard).  A window that starts at a label can inherit writers
    from a predecessor block: if the barrier is not preceded by drains of every writer kind the
    kernel holds, it is listed as "entry: check the predecessors"."""
    rows = []
    for kern, body in kernels(asm):
        ins = [s for s in body if s and not s.startswith((";", "//")) and not
               (s.startswith(".") and not s.endswith(":"))]
        has_dsw = any(s.startswith(("ds_write", "ds_store")) for s in ins)
        has_dma = any(s.startswith("buffer_load") and s.endswith(" lds") for s in ins)
        for i, s in enumerate(ins):
            if not s.startswith("s_barrier"):
                continue
            j = i - 1
            while j >= 0 and not ins[j].startswith("s_barrier") and not ins[j].endswith(":"):
                j -= 1
            at_label = j >= 0 and ins[j].endswith(":")
            pend_dsw = pend_dma = False
            for t in ins[j + 1:i]:
                if t.startswith(("ds_write", "ds_store")):
                    pend_dsw = True
                elif t.startswith("buffer_load") and t.endswith(" lds"):
                    pend_dma = True
                elif t.startswith("s_waitcnt"):
                    if "lgkmcnt(0)" in t:
                        pend_dsw = False
                    if "vmcnt(0)" in t:
                        pend_dma = False
            # drains directly before the barrier (no memory instruction after them)
            vm = lg = False
            k = i - 1
            while k > j and not MEM.match(ins[k]):
                if ins[k].startswith("s_waitcnt"):
                    vm |= "vmcnt(0)" in ins[k]
                    lg |= "lgkmcnt(0)" in ins[k]
                k -= 1
            if pend_dsw or pend_dma:
                verdict = "HAZARD: writer not drained " + " ".join(
                    (["ds_write (lgkmcnt)"] if pend_dsw else []) + (["LDS-DMA (vmcnt)"] if pend_dma else []))
            elif at_label and ((has_dsw and not lg) or (has_dma and not vm)):
                verdict = "entry: check the predecessors"
            else:
                verdict = "ok"
            rows.append((kern, i, has_dsw, has_dma, vm, lg, verdict))
    return rows


def main():
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout
    tmp = tempfile.mkdtemp()
    review = 0
    for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        s_path = os.path.join(tmp, os.path.basename(src) + ".s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-ffp-contract=off", "-I" + CSRC, "--cuda-device-only", "-S", src, "-o",
                        s_path], check=True, stderr=subprocess.DEVNULL)
        rows = audit(open(s_path).read())
        for kern, i, dsw, dma, vm, lg, verdict in rows:
            review += verdict != "ok"
            name = re.sub(r"^_Z\d+", "", kern)[:60]
            print(f"{os.path.basename(src):18s} {name:60s} barrier@{i:<6d} writers "
                  f"{'ds_write ' if dsw else '':9s}{'LDS-DMA' if dma else '':8s} drained "
                  f"{'vmcnt(0) ' if vm else '':9s}{'lgkmcnt(0)' if lg else '':10s} {verdict}", file=out)
    print(f"barriers not ok: {review}", file=out)


if __name__ == "__main__":
    main()
