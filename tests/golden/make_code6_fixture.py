"""Makes tests/golden/imagenet64_code6_r4.npz: a version-2 bitstream with conv code 6 ("dx3",
round 4's split-f16 direct conv at the 16-wide levels; read today as "dx3w16") encoded by the
round-4 build itself, and the images it holds.  Run on a GPU box with the round-4 tree
(git archive 23b932c finalproject-losslessimagecompression_amd include oracle) unpacked and
built under tools/legacy_r4/:
    python tests/golden/make_code6_fixture.py tools/legacy_r4 [out.npz]
The fixture is data only: the synthetic imagenet64 model is re-seeded (synthetic.build_model) on
the decoding side, so the test decodes these bytes with today's library and compares pixels."""
import os
import sys

import numpy as np
import torch

legacy = os.path.abspath(sys.argv[1])
sys.path.insert(0, os.path.join(legacy, "finalproject-losslessimagecompression_amd"))
from idfcodec import configs, synthetic  # noqa: E402  (the round-4 package)
from idfcodec.codec import Bitstream  # noqa: E402

assert torch.cuda.is_available()
B = 4
model = synthetic.build_model(configs.get("imagenet64")).cuda()
codec = model.codec()
img = synthetic.images(B, seed=11).cuda()
eng = model.engine()
assert eng.conv_mode == "dx3", eng.conv_mode
bs = codec.encode(img)
raw = bs.to_bytes()
back = Bitstream.from_bytes(raw)
out, info = codec.decode(back)
assert info["ok"] and torch.equal(out.cpu(), img.cpu()), "round-4 build does not round-trip"
assert back.meta.get("conv") == "dx3", back.meta
path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                           "imagenet64_code6_r4.npz")
np.savez_compressed(path, images=img.cpu().numpy(), bitstream=np.frombuffer(raw, dtype=np.uint8),
                    commit=np.array("23b932c"), bpd=np.array(bs.bpd()))
print(f"wrote {path}: {len(raw)} bytes, {bs.bpd():.4f} bits/subpixel, conv {back.meta.get('conv')}")
