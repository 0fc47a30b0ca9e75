"""Digest of the VQ-VAE conv outputs (encoder and decoder, conv modes x3t and f32) of the two
reference-fixture models, for checking that two builds of libidfcodec (IDF_LIB_PATH) compute
bit-identical VQ convs (e.g. conv_taps_kernel's IDF_TAPS_PREFETCH variants).  Prints one sha256
per (fixture, mode, pass).  Timing / A-B tool, not a test."""
import hashlib
import os
import random
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
CASES = {"vq_t1_3down": [8, 16, 24], "vq_t2_2down": [12, 20]}


def main():
    import vqvae as mirror
    from idfcodec.packing import round_up
    for name, hidden in CASES.items():
        z = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))
        sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd/")}
        K, D, nh, nb, B, H, W = [int(v) for v in z["meta"]]
        random.seed(0)
        torch.manual_seed(0)
        m = mirror.EnDecoder.get("VQVAE")(
            channel=3, embed_num=K, embed_dim=D,
            encoder={"name": "VQEncoder", "block_num": nb, "block": {"name": "ResBlock"}},
            decoder={"name": "VQDecoder", "block_num": nb, "block": {"name": "ResBlock"}},
            distribution={"name": "BinomialDistribution"}, hidden_dims=hidden)
        m.load_state_dict(sd)
        m = m.cuda().eval()
        eng = m.engine()
        data = torch.from_numpy(z["data"]).cuda()
        Bd, C, Hd, Wd = data.shape
        for mode in ("x3t", "f32"):
            eng.conv_mode = mode
            zz, (h, w) = eng.encoder_raw_pm(m._to_pm((data - 0.5) / 0.5), Bd, Hd, Wd)
            g = torch.Generator().manual_seed(1)
            v = torch.zeros(Bd * h * w, round_up(D, 4))
            v[:, :D] = torch.randn(Bd * h * w, D, generator=g)
            y, _ = eng.decoder_raw_pm(v.cuda().reshape(-1).contiguous(), Bd, h, w)
            torch.cuda.synchronize()
            for what, t in (("encoder", zz), ("decoder", y)):
                dg = hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]
                print(f"{name} {mode} {what} {dg}", flush=True)


if __name__ == "__main__":
    main()
