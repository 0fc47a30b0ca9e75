"""Where do the bench's device copies (rocprof: __amd_rocclr_copyBuffer) come from?  One codec
encode + decode of the headline batch under torch.profiler with Python stacks; prints the
memcpy / copy / fill events grouped by their top Python frames, with counts.

    python tools/find_copies.py  (GPU box)"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))

from idfcodec import configs, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = int(os.environ.get("FC_B", "256"))
    model = synthetic.build_model(configs.get("imagenet64")).to(dev)
    codec = model.codec()
    img = synthetic.images(B, seed=2).to(dev)
    for _ in range(2):
        bs = codec.encode(img)
        out, _ = codec.decode(bs, verify=False)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        bs = codec.encode(img)
        out, _ = codec.decode(bs, verify=False)
        torch.cuda.synchronize()
    assert torch.equal(out, img)
    keys = ("copy", "memcpy", "fill", "zero", "to", "cat", "clone", "contiguous", "index")
    avg = prof.key_averages(group_by_stack_n=6)
    rows = [e for e in avg if any(k in e.key.lower() for k in keys)]
    rows.sort(key=lambda e: -e.count)
    for e in rows[:40]:
        print(f"{e.count:6d}  {e.key}")
        for fr in (e.stack or [])[:6]:
            print(f"          {fr}")
    print("---- device events")
    dev_rows = [e for e in prof.key_averages() if e.device_time_total > 0]
    dev_rows.sort(key=lambda e: -e.count)
    for e in dev_rows[:25]:
        print(f"{e.count:6d} {e.device_time_total / 1e3:9.3f} ms  {e.key[:100]}")


if __name__ == "__main__":
    main()
