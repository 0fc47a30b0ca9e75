"""Synthetic models and images for tests and benchmarks (no checkpoints exist:
every config points at an absent /home/yanming/... path).

Recipe (identical to tests/golden/make_golden.py, so the reference's outputs
recorded there pin this build's regenerated model):
  * construct the model right after `random.seed(0); torch.manual_seed(0)` --
    the mirror modules create parameters in the reference's order, so the
    weights equal the reference's seeded initialisation;
  * every DenseBlock's zero-initialised head (nnblock.py:48-51) gets weight and
    bias ~ N(0, 0.05^2) from torch.Generator().manual_seed(1), in
    named_modules() order (a fresh model is otherwise a pure permutation);
  * images: torch.randint(0, 256, (B, C, H, W), generator seed 2, uint8).
"""
from __future__ import annotations

import copy
import random

import torch


def build_model(cfg: dict, head_std: float = 0.05, seed: int = 0, head_seed: int = 1):
    import flows  # noqa: F401  (registers the mirror classes)
    from moduleregister import Register
    cfg = copy.deepcopy(cfg)
    random.seed(seed)
    torch.manual_seed(seed)
    model = Register.get(cfg.pop("name"))(**cfg)
    g = torch.Generator().manual_seed(head_seed)
    with torch.no_grad():
        for _, m in model.named_modules():
            if type(m).__name__ == "DenseBlock":
                head = m.layers[-1]
                head.weight.copy_(torch.randn(head.weight.shape, generator=g) * head_std)
                head.bias.copy_(torch.randn(head.bias.shape, generator=g) * head_std)
    return model.eval()


def images(B: int, C: int = 3, H: int = 64, W: int = 64, seed: int = 2) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (B, C, H, W), generator=g, dtype=torch.uint8)


def build_vqvae(cfg: dict, seed: int = 0):
    """The residual configs' VQ-VAE at its seeded initialisation (vqvae.py mirror)."""
    import vqvae  # noqa: F401  (registers VQVAE / VQEncoder / VQDecoder)
    cfg = copy.deepcopy(cfg)
    random.seed(seed)
    torch.manual_seed(seed)
    from vqvae import EnDecoder
    return EnDecoder.get(cfg.pop("name"))(**cfg).eval()


def build_residual(name: str, device="cuda", precision: str | None = None):
    """(ResidualCodec, flows model, vqvae, input_size) of a residual north-star config.
    precision: the flow's DenseLayer arithmetic ("f32" | "bf16"); default: the config's
    (bf16 for resflow-cond-imagenet64, BASELINE configs[2]; f32 otherwise)."""
    from idfcodec import configs
    from idfcodec.residual import ResidualCodec
    vcfg, size = configs.get_vqvae(name)
    flows_model = build_model(configs.get(name)).to(device)
    flows_model.idf_precision = precision or configs.PRECISION.get(name, "f32")
    vq = build_vqvae(vcfg).to(device)
    return (ResidualCodec(flows_model, vq, size, configs.PAD.get(name, (0, 0))), flows_model,
            vq, size)
