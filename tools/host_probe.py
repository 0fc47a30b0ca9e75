"""Host enqueue cost vs GPU time (dev probe).  1) encode / decode: time for the host to issue
the whole call vs the GPU time.  2) one decode lane's flow steps (B = 128, one coupling per
step, levels top-down): host time to issue each step vs its GPU time (events on the stream) --
where the host is slower the lane's queue runs dry and the GPU idles."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "finalproject-losslessimagecompression_amd"))
from idfcodec import configs, synthetic  # noqa: E402

model = synthetic.build_model(configs.get("imagenet64")).cuda()
codec = model.codec()
eng = model.engine()
img = synthetic.images(256).cuda()
for _ in range(2):
    bs = codec.encode(img)
    codec.decode(bs, verify=False)
torch.cuda.synchronize()
for name, fn in (("encode", lambda: codec.encode(img)), ("decode", lambda: codec.decode(bs, verify=False))):
    for _ in range(2):
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name}: host issue {1e3 * (t1 - t0):.2f} ms, gpu {e0.elapsed_time(e1):.2f} ms",
              flush=True)

B = 128
for rep in range(3):
    gen = eng.inverse_pm_steps(B, lambda l, ws: None, slot=0)
    torch.cuda.synchronize()
    rows = []
    if rep == 1:  # hold the GPU while the host enqueues: event gaps are then GPU time alone
        torch.cuda._sleep(int(3e8))
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    while True:
        t0 = time.perf_counter()
        try:
            lvl = next(gen)
        except StopIteration:
            break
        t1 = time.perf_counter()
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        rows.append((lvl, 1e3 * (t1 - t0), ev, e))
        ev = e
    torch.cuda.synchronize()
    if rep == 0:
        continue
    print("GPU held during the enqueue (gpu = GPU time alone):" if rep == 1 else
          "GPU free (gpu = max(host, GPU) per step):")
    agg = {}
    for lvl, h, a, b in rows:
        g = a.elapsed_time(b)
        s = agg.setdefault(lvl, [0, 0.0, 0.0])
        s[0] += 1
        s[1] += h
        s[2] += g
    for lvl in sorted(agg, reverse=True):
        n, h, g = agg[lvl]
        print(f"lane B={B} level {lvl}: {n} steps, host {h:.2f} ms ({h / n:.3f}/step), "
              f"gpu {g:.2f} ms ({g / n:.3f}/step)", flush=True)
