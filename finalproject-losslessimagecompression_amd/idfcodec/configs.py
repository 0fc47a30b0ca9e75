"""Model sections of the four north-star configs (BASELINE.json `configs`),
restated as data from the reference YAML files they cite.  The full YAML files
(trainers, data loaders, optimisers) are outside this path; a user's own YAML
loads the same way through load_yaml()."""
from __future__ import annotations

import copy

import yaml


def _dense(growth, depth, act="ReLU"):
    return {"name": "DenseBlock", "growth_channel": growth, "depth": depth,
            "layer": {"name": "DenseLayer", "act": act}}


def _flows(name, nflows, nsplit, H, W, C, c_nn, p_nn, scale, **extra):
    d = {"name": name, "nflows": nflows, "nbits": 8, "nsplit": nsplit, "H": H, "W": W, "C": C,
         "couple": {"name": "AdditiveCouple", "split": 0.75, "nn": c_nn,
                    "round": {"name": "Round", "nbits": 8}},
         "extenddim": {"name": "ExtendDim", "scale": scale},
         "prior": {"name": "Prior", "round": {"name": "Round", "nbits": 8}, "nn": p_nn},
         "distribution": {"name": "DLogistic"},
         "round": {"name": "Round", "nbits": 8}}
    d.update(extra)
    return d


CONFIGS = {
    # configs/imagenet64.yaml:2-40
    "imagenet64": _flows("IDFlows", 8, 3, 64, 64, 3, _dense(512, 12), _dense(512, 12), 2),
    # configs/resflow-cond-imagenet64.yaml:3-44 (flows section)
    "resflow-cond-imagenet64": _flows("ConditionalFlows", 8, 3, 64, 64, 3, _dense(512, 12),
                                      _dense(512, 12), 2, conv_for_cond=True),
    # configs/resflows_smallpatch_split.yaml:3-41 (flows section, 8x8 patches)
    "resflows_smallpatch_split": _flows("IDFlows", 8, 2, 8, 8, 3, _dense(512, 8), _dense(512, 4), 2),
    # configs/resflow-patches-vqvae.yaml:3-42 (flows section, 27x23 patches)
    "resflow-patches-vqvae": _flows("ConditionalFlows", 8, 1, 27, 23, 3,
                                    _dense(384, 12, "LeakyReLU"), _dense(512, 12, "LeakyReLU"), 1,
                                    conv_for_cond=False),
}


def _vqvae(embed_num, embed_dim, hidden, block_num=8):
    blk = {"name": "ResBlock", "batch_norm": False}
    return {"name": "VQVAE", "channel": 3, "embed_num": embed_num, "embed_dim": embed_dim,
            "encoder": {"name": "VQEncoder", "block_num": block_num, "block": dict(blk)},
            "decoder": {"name": "VQDecoder", "block_num": block_num, "block": dict(blk)},
            "distribution": {"name": "BinomialDistribution"},
            "vectorquantizer": {"reinit_interval": 1000, "threshold": 0.1},
            "hidden_dims": list(hidden), "batch_norm": False}


# VQ-VAE sections and input sizes of the residual configs (ResidualTrainer; the
# checkpoints they name are absent, so the weights are the seeded initialisation)
VQVAE = {
    # configs/resflow-cond-imagenet64.yaml:46-73, input_size :75-77
    "resflow-cond-imagenet64": (_vqvae(16384, 512, [128, 256, 384]), (64, 64)),
    # configs/resflows_smallpatch_split.yaml:44-75 (BASELINE configs[3]: synthetic 256x256)
    "resflows_smallpatch_split": (_vqvae(8192, 512, [128, 256, 512]), (256, 256)),
    # configs/resflow-patches-vqvae.yaml:46-78 (215x178 CelebA padded to 216x184)
    "resflow-patches-vqvae": (_vqvae(8192, 512, [128, 256, 512]), (216, 184)),
}


# BASELINE configs[2] names "MFMA bf16 coupling convs with fp32 CDF" for this config
PRECISION = {"resflow-cond-imagenet64": "bf16"}
# dataloader ReplicationPad2d (bottom, right) before coding (trainer.py:62; the 215x178
# CelebA crops of configs/resflow-patches-vqvae.yaml:84-93 become 216x184)
PAD = {"resflow-patches-vqvae": (1, 6)}


def get(name: str) -> dict:
    return copy.deepcopy(CONFIGS[name])


def get_vqvae(name: str):
    """(VQVAE kwargs incl. name, input_size) of a residual config."""
    cfg, size = VQVAE[name]
    return copy.deepcopy(cfg), tuple(size)


def load_yaml(path: str) -> dict:
    """`train.model` (Trainer) or `train.flows` (ResidualTrainer) of a reference-style YAML."""
    with open(path) as f:
        cfg = yaml.safe_load(f)["train"]
    return cfg.get("model") or cfg.get("flows")
