"""Host issue time vs GPU time of encode / decode (lanes 1, 2): is the decode host-bound?"""
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
for lanes, stg, dst, wpb in ((1, "host", "0", "4"), (2, "host", "1", "4"), (2, "event", "1", "4"),
                             (2, "host", "0", "4"), (2, "host", "1", "1"), (4, "host", "1", "4"),
                             (2, "host", "1", "4")):
    codec.lanes = lanes
    os.environ["IDF_LANE_STAGGER"] = stg
    os.environ["IDF_LANE_DEC_STREAM"] = dst
    os.environ["IDF_DECODE_WPB"] = wpb
    stg = f"{stg} decstream={dst} wpb={wpb}"
    codec.decode(bs, verify=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, info = codec.decode(bs, verify=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    t3 = time.perf_counter()
    b2 = codec.encode(img, compact=False)
    t4 = time.perf_counter()
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    print(f"lanes {lanes} {stg}: decode issue {1e3*(t1-t0):.2f} ms, done {1e3*(t2-t0):.2f} ms; "
          f"encode(compact=False) issue {1e3*(t4-t3):.2f} ms, done {1e3*(t5-t3):.2f} ms", flush=True)
