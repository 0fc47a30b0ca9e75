import os, sys, torch
sys.path.insert(0, "finalproject-losslessimagecompression_amd")
from idfcodec import synthetic
from idfcodec.codec import RANS_L
name = sys.argv[1] if len(sys.argv) > 1 else "resflows_smallpatch_split"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
mode = sys.argv[3] if len(sys.argv) > 3 else None
codec, fl, vq, size = synthetic.build_residual(name)
if mode:
    fl.engine().set_conv_mode(mode)
src = (256, 256) if name == "resflows_smallpatch_split" else (215, 178)
x = synthetic.images(B, H=src[0], W=src[1], seed=23).cuda()
rbs = codec.encode(x)
out, info = codec.decode(rbs)
fs = info.get("final_states")
print("B", B, "mode", mode, "lanes", os.environ.get("IDF_LANES"), "stagger", os.environ.get("IDF_LANE_STAGGER"),
      "ok", info.get("ok"), "equal", torch.equal(out, x),
      "bad_final", None if fs is None else int((fs != RANS_L).sum()),
      "off_grid", int(info["off_grid"].item()), "nimg", rbs.flow.n_images, flush=True)
if fs is not None:
    bad = (fs != RANS_L).nonzero().flatten()
    if bad.numel():
        print("  bad streams", bad.min().item(), "..", bad.max().item(), "of", fs.numel())
