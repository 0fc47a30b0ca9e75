"""Is the decode host-bound?  Times the host's enqueue of codec.decode (until the call returns,
no sync) against the wall time to the GPU's completion, at the bench workload (dev tool)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
import torch  # noqa: E402

from idfcodec import configs, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda")
    model = synthetic.build_model(configs.get("imagenet64")).to(dev)
    codec = model.codec()
    img = synthetic.images(256, seed=2).to(dev)
    for _ in range(2):
        bs = codec.encode(img)
        codec.decode(bs, verify=False)
    torch.cuda.synchronize()
    for it in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bs = codec.encode(img)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out, _ = codec.decode(bs, verify=False)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"encode call {1e3*(t1-t0):.2f} ms (ends in a sync) | decode issue {1e3*(t3-t2):.2f} ms, "
              f"decode wall {1e3*(t4-t2):.2f} ms, exact {torch.equal(out, img)}", flush=True)


if __name__ == "__main__":
    main()
