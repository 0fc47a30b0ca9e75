"""Decode lanes probe: when does lane 1 start relative to lane 0 (timing events recorded on
each lane stream right after its wait), and the decode's total time.  Variants: staggered by
an event or not; torch pool streams or HIP streams created here with hipStreamNonBlocking."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "finalproject-losslessimagecompression_amd"))
from idfcodec import configs, synthetic  # noqa: E402

model = synthetic.build_model(configs.get("imagenet64")).cuda()
codec = model.codec()
img = synthetic.images(256).cuda()
bs = codec.encode(img)
hip = ctypes.CDLL("libamdhip64.so.7")
ext = []
for _ in range(4):
    h = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) == 0
    ext.append(torch.cuda.ExternalStream(h.value))
torch_streams = [torch.cuda.Stream(), torch.cuda.Stream()]
V = [(1, "event", "torch", "4")]
V += [(2, st, "ext", "4") for st in ("event", "none", "event", "none")]
for lanes, stg, kind, wpb in V:
    os.environ["IDF_DECODE_WPB"] = wpb
    codec.lanes = lanes
    os.environ["IDF_LANE_STAGGER"] = stg
    codec._streams = list(ext if kind == "ext" else torch_streams)
    for rep in range(2):
        codec.lane_marks = []
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        out, info = codec.decode(bs, verify=False)
        t1 = time.perf_counter()
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        marks = [round(e0.elapsed_time(m), 2) for m in codec.lane_marks]
        ok = torch.equal(out, img)
        print(f"lanes {lanes} stagger={stg} streams={kind} wpb={wpb}: issue {1e3*(t1-t0):.2f} ms, "
              f"gpu {e0.elapsed_time(e1):.2f} ms, lane starts {marks} ms, exact {ok}", flush=True)
