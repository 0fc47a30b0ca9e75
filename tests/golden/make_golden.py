"""tests/golden/make_golden.py -- generates the committed golden fixtures.

Runs ONLY in the build container, where the reference tree exists:
  * the reference's Python flows are imported from /root/reference (with a
    `colorama` stub); bytecode writing is disabled so nothing is
    written into the reference tree;
  * the reference's own rANS coder is the Cython module compiled from
    /root/reference/rans/rans.cpp into oracle/_ref by oracle/Makefile.
The fixtures hold data only (inputs, weights, expected outputs); no reference
source travels.  Re-run:  python tests/golden/make_golden.py

Synthetic-weight recipe (shared with idfcodec.synthetic): the model is
constructed right after `random.seed(0); torch.manual_seed(0)`; then every
DenseBlock's zero-initialised 1x1 head (nnblock.py:48-51) gets weight and bias
drawn N(0, 0.05^2) from a torch.Generator seeded 1, in named_modules() order.
"""
from __future__ import annotations

import copy
import math
import os
import random
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.modules.setdefault("colorama", types.SimpleNamespace(reinit=None))
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import rans_oracle  # noqa: E402  (for building/loading oracle/_ref)
import flows as ref_flows  # noqa: E402
import yaml  # noqa: E402

torch.set_num_threads(8)
ref_coder = rans_oracle.load_reference_coder()
assert ref_coder is not None, "build oracle/_ref first: make -C oracle"


# ----------------------------------------------------------------------------- configs
def dense(growth, depth, act="ReLU"):
    return {"name": "DenseBlock", "growth_channel": growth, "depth": depth,
            "layer": {"name": "DenseLayer", "act": act}}


def flows_cfg(name, nflows, nsplit, H, W, C=3, cg=24, cd=3, pg=16, pd=2, act="ReLU", scale=2,
              **extra):
    cfg = {"name": name, "nflows": nflows, "nbits": 8, "nsplit": nsplit, "H": H, "W": W, "C": C,
           "couple": {"name": "AdditiveCouple", "split": 0.75, "nn": dense(cg, cd, act),
                      "round": {"name": "Round", "nbits": 8}},
           "extenddim": {"name": "ExtendDim", "scale": scale},
           "prior": {"name": "Prior", "round": {"name": "Round", "nbits": 8},
                     "nn": dense(pg, pd, act)},
           "distribution": {"name": "DLogistic"},
           "round": {"name": "Round", "nbits": 8}}
    cfg.update(extra)
    return cfg


TINY = {
    "t1_idflows_2lvl": flows_cfg("IDFlows", 2, 2, 8, 8),
    "t2_idflows_3lvl_leaky": flows_cfg("IDFlows", 2, 3, 16, 16, cg=32, cd=2, pg=24, pd=2,
                                       act="LeakyReLU"),
    "t3_cond_convcond": flows_cfg("ConditionalFlows", 2, 2, 8, 8, conv_for_cond=True),
    "t4_cond_s1_odd": flows_cfg("ConditionalFlows", 2, 1, 9, 7, cg=16, cd=2, pg=16, pd=2,
                                act="LeakyReLU", scale=1, conv_for_cond=False),
}


def build_model(cfg):
    cfg = copy.deepcopy(cfg)
    random.seed(0)
    torch.manual_seed(0)
    model = ref_flows.NNFlows.get(cfg.pop("name"))(**cfg)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for _, m in model.named_modules():
            if type(m).__name__ == "DenseBlock":
                head = m.layers[-1]
                head.weight.copy_(torch.randn(head.weight.shape, generator=g) * 0.05)
                head.bias.copy_(torch.randn(head.bias.shape, generator=g) * 0.05)
    return model.eval()


def dequant(u8: torch.Tensor) -> torch.Tensor:
    """trainer.py:101,131-136: ToTensor (k/255) then Round(nbits=8)."""
    x = u8.to(torch.float32) / 255.0
    return torch.round(x * 256) / 256


def images(B, C, H, W, seed=2):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (B, C, H, W), generator=g, dtype=torch.uint8)


def sd_arrays(model, prefix="sd/"):
    return {prefix + k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}


# ----------------------------------------------------------------------------- rANS
def rans_case(out, name, x, mean, scale, state=1 << 32):
    x = [float(v) for v in np.float32(x)]
    mean = [float(v) for v in np.float32(mean)]
    scale = [float(v) for v in np.float32(scale)]
    n = len(x)
    st, words = ref_coder.encode(state, n, x, mean, scale)
    dst, msg = ref_coder.decode(st, words[::-1], n, mean[::-1], scale[::-1])
    out[f"{name}/x"] = np.float32(x)
    out[f"{name}/mean"] = np.float32(mean)
    out[f"{name}/scale"] = np.float32(scale)
    out[f"{name}/init_state"] = np.uint64(state)
    out[f"{name}/state"] = np.uint64(st)
    out[f"{name}/words"] = np.asarray(words, np.uint32)
    out[f"{name}/dec_state"] = np.uint64(dst)
    out[f"{name}/dec_x"] = np.float32(msg[::-1])


def rans_fixtures():
    out = {}
    # KAT1
    N = 4096
    f32 = lambda v: float(np.float32(v))  # noqa: E731
    mean = [f32(((37 * i) % 513 - 256) / 256) for i in range(N)]
    scale = [f32((1 + (13 * i) % 200) / 1024) for i in range(N)]
    x = [round((mean[i] + scale[i] * ((7 * i) % 11 - 5)) * 256) / 256 for i in range(N)]
    rans_case(out, "kat1", x, mean, scale)
    # chained (coder.py:18-27 state chaining)
    st, w0 = ref_coder.encode(1 << 32, 10, x[:10], mean[:10], scale[:10])
    st2, w1 = ref_coder.encode(st, 10, x[10:20], mean[10:20], scale[10:20])
    out["chain/state0"] = np.uint64(st)
    out["chain/words0"] = np.asarray(w0, np.uint32)
    out["chain/state1"] = np.uint64(st2)
    out["chain/words1"] = np.asarray(w1, np.uint32)
    # rans/test.py-style random streams (rans/test.py:8-10), seeded
    for n in (1, 96, 1863, 3072, 6144):
        rng = random.Random(1000 + n)
        mean = [rng.randint(-256, 256) / 256 for _ in range(n)]
        scale = [math.exp(10 * rng.random() - 5) / 256 for _ in range(n)]
        msg = [round((mean[i] + scale[i] * (10 * rng.random() - 5)) * 256) / 256 for i in range(n)]
        rans_case(out, f"rand{n}", msg, mean, scale)
    # coder.py __main__ style: narrow scales (coder.py:45-48)
    rng = random.Random(7)
    n = 5000
    mean = [rng.randint(-32, 32) / 256 for _ in range(n)]
    scale = [math.exp(rng.random() * 0.01 - 0.005) for _ in range(n)]
    msg = [round((mean[i] + scale[i] * (1.0 * rng.random() - 0.5)) * 256) / 256 for i in range(n)]
    rans_case(out, "narrow", msg, mean, scale)
    # edges: tiny / huge scales, window ends, out-of-window symbols
    rng = np.random.default_rng(11)
    n = 512
    mean = (rng.integers(-512, 512, n) / 256 + rng.normal(0, 0.3, n)).astype(np.float32)
    lower = np.round(mean.astype(np.float64) * 256 - 1024)
    pick = rng.integers(0, 4, n)
    xs = np.where(pick == 0, lower, np.where(pick == 1, lower + 2047,
                  np.round(mean.astype(np.float64) * 256) + rng.integers(-3, 4, n))) / 256
    scale = np.where(rng.random(n) < 0.5, 1e-8, 1e6).astype(np.float32)
    scale[::7] = np.exp(rng.normal(-3, 2, scale[::7].size)).astype(np.float32)
    rans_case(out, "edge_window", xs, mean, scale)
    # out-of-window (silent corruption in the reference; bit pattern pinned)
    n = 64
    mean = np.zeros(n, np.float32)
    xs = np.where(np.arange(n) % 8 == 3, 5.0, np.round(rng.normal(0, 0.5, n) * 256) / 256)
    scale = np.full(n, 0.25, np.float32)
    rans_case(out, "out_of_window", xs, mean, scale)
    # empty stream
    st, w = ref_coder.encode(1 << 32, 0, [], [], [])
    out["empty/state"] = np.uint64(st)
    out["empty/nwords"] = np.int64(len(w))
    # CDF spot values (x, mean, scale, lower) -> CDF, via start/freq of single encodes
    return out


# ----------------------------------------------------------------------------- flows
def flow_fixture(name, cfg, B=2):
    model = build_model(cfg)
    H, W, C = cfg["H"], cfg["W"], cfg["C"]
    u8 = images(B, C, H, W, seed=2)
    x = dequant(u8)
    out = {"cfg_yaml": np.frombuffer(yaml.safe_dump(cfg).encode(), np.uint8), "image_u8": u8.numpy()}
    out.update(sd_arrays(model))
    blocks_io = []

    def make_hook(name):
        def hook(mod, inp, outp):
            if len(blocks_io) < 4:
                blocks_io.append((name, inp[0].detach().clone(), outp.detach().clone()))
        return hook

    hooks = [m.register_forward_hook(make_hook(n)) for n, m in model.named_modules()
             if type(m).__name__ == "DenseBlock"]
    with torch.no_grad():
        if cfg["name"] == "ConditionalFlows":
            g = torch.Generator().manual_seed(3)
            rec = torch.round(torch.rand((B, C, H, W), generator=g) * 256) / 256
            res = x - rec
            lat, means, logs, _ = model.forward(res, None, rec)
            out["cond"] = rec.numpy()
            out["input"] = res.numpy()
        else:
            lat, means, logs, _ = model.forward(x, None)
            out["input"] = x.numpy()
        for h in hooks:
            h.remove()
        logp, logps = model.log_likelihood(lat, means, logs)
        gen = model.generated_from_latents(lat)
    for i, (nm, a, b) in enumerate(blocks_io):
        out[f"dense{i}/name"] = np.frombuffer(nm.encode(), np.uint8)
        out[f"dense{i}/in"] = a.numpy()
        out[f"dense{i}/out"] = b.numpy()
    for i in range(len(lat)):
        out[f"latent{i}"] = lat[i].numpy()
        out[f"mean{i}"] = means[i].numpy()
        out[f"logscale{i}"] = logs[i].numpy()
    out["log_prob"] = logp.numpy()
    out["generated"] = gen.numpy()
    np.savez_compressed(os.path.join(HERE, f"flow_{name}.npz"), **out)
    return model


def imagenet64_fixture():
    """configs/imagenet64.yaml at the synthetic recipe, B=2 (SURVEY 8(d) config 1 inputs).
    Weights are NOT stored (60 M params): they are regenerated from the seeded recipe by the
    build's own modules, which create parameters in the reference's order."""
    with open(os.path.join(REF, "configs", "imagenet64.yaml")) as f:
        cfg = yaml.safe_load(f)["train"]["model"]
    model = build_model(cfg)
    B = 2
    u8 = images(B, 3, 64, 64, seed=2)
    x = dequant(u8)
    with torch.no_grad():
        lat, means, logs, _ = model.forward(x, None)
        logp, _ = model.log_likelihood(lat, means, logs)
        gen = model.generated_from_latents(lat)
    out = {"cfg_yaml": np.frombuffer(yaml.safe_dump(cfg).encode(), np.uint8),
           "image_u8": u8.numpy(), "log_prob": logp.numpy(),
           "gen_maxabs": np.float32((gen - x).abs().max().item())}
    # parameter checksums: pin that the build regenerates the same synthetic model
    sd = model.state_dict()
    out["param_names"] = np.frombuffer("\n".join(sd.keys()).encode(), np.uint8)
    out["param_sums"] = np.array([float(v.double().sum()) for v in sd.values()], np.float64)
    out["param_abs_sums"] = np.array([float(v.double().abs().sum()) for v in sd.values()],
                                     np.float64)
    for i in range(len(lat)):
        out[f"latent{i}"] = lat[i].numpy()
        out[f"mean{i}"] = means[i].numpy()
        out[f"logscale{i}"] = logs[i].numpy()
        scale = torch.exp(logs[i])
        # per-(image, level) streams: one reference encode() per image and level
        for b in range(B):
            xs = lat[i][b].reshape(-1).tolist()
            ms = means[i][b].reshape(-1).tolist()
            ss = scale[b].reshape(-1).tolist()
            st, w = ref_coder.encode(1 << 32, len(xs), xs, ms, ss)
            out[f"enc{i}_{b}/state"] = np.uint64(st)
            out[f"enc{i}_{b}/words"] = np.asarray(w, np.uint32)
        # trainer.py:310-315 contract: one stream per level over the whole batch
        xs = lat[i].reshape(-1).tolist()
        ms = means[i].reshape(-1).tolist()
        ss = scale.reshape(-1).tolist()
        st, w = ref_coder.encode(1 << 32, len(xs), xs, ms, ss)
        out[f"enclevel{i}/state"] = np.uint64(st)
        out[f"enclevel{i}/nwords"] = np.int64(len(w))
        out[f"enclevel{i}/wordsum"] = np.uint64(sum(w) % (1 << 64))
        out[f"scale{i}"] = scale.numpy()
    np.savez_compressed(os.path.join(HERE, "imagenet64_b2.npz"), **out)


def main():
    np.savez_compressed(os.path.join(HERE, "rans_kat.npz"), **rans_fixtures())
    for name, cfg in TINY.items():
        flow_fixture(name, cfg)
    imagenet64_fixture()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
