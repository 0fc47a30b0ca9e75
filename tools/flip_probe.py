"""Round flips of the imagenet64 forward per level against the reference's recorded latents
(tests/golden/imagenet64_b2.npz, B=2) and against the torch-fp32 oracle (B=16), in each conv
mode: how much of the flip count is the kernels' arithmetic and how much is fp32 itself."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import flow_oracle as FO  # noqa: E402
from idfcodec import configs, synthetic  # noqa: E402

cfg = configs.get("imagenet64")
model = synthetic.build_model(cfg).cuda()
eng = model.engine()
d = np.load(os.path.join(REPO, "tests", "golden", "imagenet64_b2.npz"))
x2 = FO.dequant(torch.from_numpy(d["image_u8"]))
o = FO.FlowOracle(cfg, {k: v.detach().cpu() for k, v in model.state_dict().items()})
x16 = FO.dequant(synthetic.images(16, seed=2))
r16, _, _ = o.forward(x16)
r2o, _, _ = o.forward(x2)
print("oracle vs reference (B=2):", [int((a != torch.from_numpy(d[f"latent{i}"])).sum())
                                      for i, a in enumerate(r2o)])
with torch.no_grad():
    for mode in ("dx3", "dx3w16", "x3", "f32"):
        eng.set_conv_mode(mode)
        lat, _, _, _ = model(x2.cuda(), None)
        fr = [int((lat[i].cpu() != torch.from_numpy(d[f"latent{i}"])).sum()) for i in range(3)]
        lat16, _, _, _ = model(x16.cuda(), None)
        fo = [int((a.cpu() != b).sum()) for a, b in zip(lat16, r16)]
        print(f"{mode:7s} vs reference (B=2) {fr}  vs oracle (B=16) {fo}", flush=True)
eng.set_conv_mode("dx3")
